"""Fixed workloads for rocprofv3 --pmc passes (tools/gpu_pmc.sh), one per summary: the
summary averages counters per kernel NAME, so workloads that launch the same kernel at
different shapes or cache states get their own run.

  main           3 launches each of the bench's hash (1M x 512 B), validator-span encode
                 (16.7 M records), attestation checks (4M) and attestation encode (1M), plus a
                 134 MB torch copy (the FETCH_SIZE yardstick)
  epoch65k       3 steps of the bench's configs[2] epoch (65,536 validators x 256 instances)
  epoch1m        3 steps of configs[3]'s size on one GPU (1,048,576 x 16)
  epoch65k_cold  the configs[2] step rotated over 6 distinct instance sets (6 x 134 MB of
                 streamed state with the u32 balance offsets, 3x the 256 MiB Infinity Cache):
                 every step reads its set cold from HBM (bench.py's epoch.cold)
  epoch1m_cold   the same at 1,048,576 x 16
  epoch_single   20 steps of ONE 65,536-validator instance (the single-launch latency path)
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):  # (A/B: another build of the library)
    from prysm_amd import _lib as _pl
    _pl.library_path = os.environ["PZ_PROBE_LIB"]
from prysm_amd import _lib, casper, synth  # noqa: E402
from prysm_amd.native import NativeEpoch  # noqa: E402

DEV = torch.device("cuda", 0)


def _epoch_sets(nval, B, nsets):
    shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
    return [NativeEpoch(synth.epoch_batch(nval, B, seed=3 + k, shuffled=shuffled), device=0) for k in range(nsets)]


def epoch(nval, B, nsets, rounds):
    """The bench's epoch path (pz_epoch_state, one-pass step); with nsets > 1 the steps rotate
    over the sets on one stream (pz_epoch_state_bind_stream)."""
    sets = _epoch_sets(nval, B, nsets)
    s = torch.cuda.Stream(device=DEV)  # a real stream (a null handle means the state's own)
    for de in sets:
        de.bind_stream(s.cuda_stream)
    for _ in range(rounds):
        for de in sets:
            de.step()
    torch.cuda.synchronize()
    for de in sets:
        de.free()
    print("pmc epoch workload done: %d x %d, %d set(s), %d round(s)" % (nval, B, nsets, rounds))


def main_workload():
    s = torch.cuda.current_stream(DEV)
    sh = ctypes.c_void_p(s.cuda_stream)
    n = 1 << 20
    d_in = torch.from_numpy(synth.attestation_records_512(n, seed=2).reshape(-1)).to(DEV)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=DEV)
    for _ in range(3):
        _lib.lib.call("pz_dev_blake2b512_fixed", d_in.data_ptr(), 512, 512, n, d_out.data_ptr(), 32, sh)
    x = torch.empty(1 << 24, dtype=torch.int64, device=DEV)
    y = torch.empty_like(x)
    for _ in range(3):
        x.copy_(y)
    # the bench's wire and attcheck legs, same inputs
    import bench  # noqa: E402
    nw = 16 << 20
    rng = np.random.default_rng(7)
    cols_t = [torch.from_numpy(a.view(np.int64)).to(DEV) for a in (
        rng.integers(16, 49, size=nw, dtype=np.uint64), np.zeros(nw, np.uint64),
        np.full(nw, 9999999999999999999, np.uint64))]
    w_out = torch.empty(int(_lib.lib.dll.pz_wire_validators_bound(nw, 0)), dtype=torch.uint8, device=DEV)
    w_scr = torch.empty(int(_lib.lib.dll.pz_wire_scratch_bytes(nw)) // 8, dtype=torch.int64, device=DEV)
    w_tot = torch.zeros(1, dtype=torch.int64, device=DEV)
    vc = _lib.ValidatorCols(None, None, None, None, None, None, *[t.data_ptr() for t in cols_t])
    for _ in range(3):
        _lib.lib.call("pz_dev_wire_validators", ctypes.byref(vc), nw, 11, w_out.data_ptr(), None, w_scr.data_ptr(),
                      w_tot.data_ptr(), sh)
    del cols_t, w_out, w_scr
    na = 1 << 22
    cols, tab = bench.attcheck_columns(na, seed=11)
    b, keep = bench.attcheck_batch(torch, DEV, cols, tab, na)
    for _ in range(3):
        _lib.lib.call("pz_dev_check_attestations", ctypes.byref(b), sh)
    del keep
    # the bench's wire_att leg: the 1M config-2 records encoded from their columns
    from prysm_amd import wire
    cols = synth.attestation_columns_512(n, seed=2)
    tc = {k: torch.from_numpy(cols[k].view(np.int64) if cols[k].dtype == np.uint64 else cols[k]).to(DEV)
          for k in wire.ATT_COLS}
    ac = _lib.AttestationCols(*[tc[k].data_ptr() for k in wire.ATT_COLS])
    a_out = torch.empty(n * 512 + 16, dtype=torch.uint8, device=DEV)
    a_offs = torch.empty(n + 1, dtype=torch.int64, device=DEV)
    a_scr = torch.empty(int(_lib.lib.dll.pz_wire_attestations_scratch_bytes(n)), dtype=torch.uint8, device=DEV)
    for _ in range(3):
        _lib.lib.call("pz_dev_wire_attestations", ctypes.byref(ac), n, 0, a_out.data_ptr(), a_offs.data_ptr(),
                      a_scr.data_ptr(), sh)
    torch.cuda.synchronize()
    print("pmc main workload done")


WORKLOADS = {
    "main": main_workload,
    "epoch65k": lambda: epoch(65536, 256, 1, 3),
    "epoch1m": lambda: epoch(1 << 20, 16, 1, 3),
    "epoch65k_cold": lambda: epoch(65536, 256, 6, 2),
    "epoch1m_cold": lambda: epoch(1 << 20, 16, 6, 2),
    "epoch_single": lambda: epoch(65536, 1, 1, 20),
}


if __name__ == "__main__":
    WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "main"]()
