"""Times pz_dev_check_attestations alone on the bench's attcheck workload (4M attestations at
configs[2]'s committee shape) with HIP events.  PZ_PROBE_LIB selects another build of the
library for a same-box A/B."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from prysm_amd import _lib  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):
    _lib.library_path = os.environ["PZ_PROBE_LIB"]
import bench  # noqa: E402


def main():
    natt = 1 << 22
    cols, tab = bench.attcheck_columns(natt, seed=11)
    b, t = bench.attcheck_batch(torch, torch.device("cuda", 0), cols, tab, natt, last_byte=True)  # the bench's batch
    st, cm, ps = t["status"], t["committee"], t["pstart"]
    sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(200):
        _lib.lib.call("pz_dev_check_attestations", ctypes.byref(b), sh)
    torch.cuda.synchronize()
    def timed(reps=100):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            _lib.lib.call("pz_dev_check_attestations", ctypes.byref(b), sh)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    ms = timed()
    digest = int(st.sum().item()) * 31 + int(cm.sum().item()) * 7 + int(ps.sum().item())
    print("attcheck: %d attestations  %.4f ms  %.1f G/s  result digest %d" % (natt, ms, natt / ms / 1e6, digest),
          flush=True)
    dll = _lib.lib.dll
    if hasattr(dll, "pz_debug_set_attcheck_variant"):  # same-process A/B (PZ_PROBE_LIB=build/ab/...)
        # 0 the product (persistent blocks, the committee table in LDS, 3 blocks per CU), 1 round 5's
        # x2 kernel (the walk in global memory), 2 / 3 the product at 2 / 1 blocks per CU
        for v in [int(x) for x in os.environ.get("VARIANTS", "0,1,2,3,0,1").split(",")]:
            dll.pz_debug_set_attcheck_variant(v)
            ms = timed()
            d = int(st.sum().item()) * 31 + int(cm.sum().item()) * 7 + int(ps.sum().item())
            print("  variant %d  %.4f ms  same digest %s" % (v, ms, d == digest), flush=True)
        dll.pz_debug_set_attcheck_variant(0)


if __name__ == "__main__":
    main()
