"""Times pz_dev_wire_validators alone (16 states x 1,048,576 genesis-style validators, the
bench's wire workload) with HIP events; small enough to run under rocprofv3 --pmc."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from prysm_amd import _lib  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):  # A/B against another build of the library
    _lib.library_path = os.environ["PZ_PROBE_LIB"]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    n = 16 << 20
    rng = np.random.default_rng(7)
    cols_np = [rng.integers(16, 49, size=n, dtype=np.uint64), np.zeros(n, np.uint64),
               np.full(n, 9999999999999999999, np.uint64)]
    cols_t = [torch.from_numpy(a.view(np.int64)).cuda() for a in cols_np]
    out = torch.empty(int(_lib.lib.dll.pz_wire_validators_bound(n, 0)), dtype=torch.uint8, device="cuda")
    scr = torch.empty(int(_lib.lib.dll.pz_wire_scratch_bytes(n)) // 8, dtype=torch.int64, device="cuda")
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    cols = _lib.ValidatorCols(None, None, None, None, None, None, *[t.data_ptr() for t in cols_t])
    sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        _lib.lib.call("pz_dev_wire_validators", ctypes.byref(cols), n, 11, out.data_ptr(), None, scr.data_ptr(),
                      tot.data_ptr(), sh)

    def timed():
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    us = timed()
    total = int(tot.item())
    alg = n * 24 + total
    print("wire: %d records, %d bytes, %.1f us/launch, %.0f GB/s algorithmic (%.1f%% of 8 TB/s)"
          % (n, total, us, alg / us / 1e3, alg / us / 1e3 / 80))
    geom = os.environ.get("WIRE_GEOM")
    if geom:  # tile-geometry variants (wire.hip PZ_WIRE_VAL_GEOM): exact output, compared with the product's
        want = out[:total].clone()
        for v in [int(x) for x in geom.split(",")]:
            _lib.lib.dll.pz_debug_set_wire_variant(v)
            out.zero_()
            us_v = timed()
            same = int(tot.item()) == total and bool(torch.equal(out[:total], want))
            print("  geometry %6d: %.1f us/launch (%.1f%% of 8 TB/s), output identical: %s"
                  % (v, us_v, alg / us_v / 1e3 / 80, same), flush=True)
        _lib.lib.dll.pz_debug_set_wire_variant(0)
    if len(sys.argv) > 2:  # ablation (wire.hip wire_val_body V, one tile per workgroup): results wrong for V != 0
        names = {1: "tile = blockIdx (no ticket)", 2: "no stage build", 4: "no look-back", 8: "no store",
                 7: "1+2+4", 15: "1+2+4+8", 16: "reload values for the build",
                 512: "no mid-build re-read of the window",
                 1024: "look-back reduced by LDS atomic + block scan",
                 2048: "sub-tile scans by shfl_up", 4096: "default-policy column loads",
                 8192: "nontemporal output stores", 12288: "default-policy loads, nontemporal stores"}
        for v in (0, 4096, 8192, 12288, 0, 4096, 8192, 12288, 1, 2, 4, 8, 0):
            _lib.lib.dll.pz_debug_set_wire_variant(v)
            print("  variant %2d %-28s %.1f us" % (v, names.get(v, "product"), timed()))
        _lib.lib.dll.pz_debug_set_wire_variant(0)


if __name__ == "__main__":
    main()
