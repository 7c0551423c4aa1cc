"""Small fixed workload for rocprofv3 --pmc passes: 3 hash launches (1M x 512 B), 3 epoch
steps (65,536 validators x 256 instances), 3 validator-span encodings (16.7 M records) and 3
attestation-check batches (4M) and 3 attestation encodings (1M), the bench's workloads, plus a torch copy as a bandwidth
yardstick."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from prysm_amd import _lib, casper, synth  # noqa: E402
from prysm_amd.native import NativeEpoch  # noqa: E402


def epoch_1m():
    """Only the bench's configs[3]-sized epoch on one GPU (1,048,576 validators x 16
    instances), 3 steps: its own counter passes, since the summary averages per kernel name."""
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    nval, B = 1 << 20, 16
    inst = synth.epoch_batch(nval, B, seed=3,
                             shuffled=casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32)))
    de = NativeEpoch(inst, device=0)  # the bench's path (pz_epoch_state, one-pass step)
    for _ in range(3):
        de.step()
    de.sync()
    torch.cuda.synchronize()
    print("pmc epoch_1m workload done")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "epoch_1m":
        return epoch_1m()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(s.cuda_stream)
    n = 1 << 20
    d_in = torch.from_numpy(synth.attestation_records_512(n, seed=2).reshape(-1)).to(dev)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    for _ in range(3):
        _lib.lib.call("pz_dev_blake2b512_fixed", d_in.data_ptr(), 512, 512, n, d_out.data_ptr(), 32, sh)
    nval, B = 65536, 256
    inst = synth.epoch_batch(nval, B, seed=3,
                             shuffled=casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32)))
    de = NativeEpoch(inst, device=0)  # the bench's path (pz_epoch_state, one-pass step)
    for _ in range(3):
        de.step()
    de.sync()
    x = torch.empty(nval * B, dtype=torch.int64, device=dev)
    y = torch.empty_like(x)
    for _ in range(3):
        x.copy_(y)
    # the bench's wire and attcheck legs, same inputs
    import bench  # noqa: E402
    nw = 16 << 20
    rng = np.random.default_rng(7)
    cols_t = [torch.from_numpy(a.view(np.int64)).to(dev) for a in (
        rng.integers(16, 49, size=nw, dtype=np.uint64), np.zeros(nw, np.uint64),
        np.full(nw, 9999999999999999999, np.uint64))]
    w_out = torch.empty(int(_lib.lib.dll.pz_wire_validators_bound(nw, 0)), dtype=torch.uint8, device=dev)
    w_scr = torch.empty(int(_lib.lib.dll.pz_wire_scratch_bytes(nw)) // 8, dtype=torch.int64, device=dev)
    w_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    vc = _lib.ValidatorCols(None, None, None, None, None, None, *[t.data_ptr() for t in cols_t])
    for _ in range(3):
        _lib.lib.call("pz_dev_wire_validators", ctypes.byref(vc), nw, 11, w_out.data_ptr(), None, w_scr.data_ptr(),
                      w_tot.data_ptr(), sh)
    cols, tab = bench.attcheck_columns(1 << 22, seed=11)
    t = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v.view(np.int32) if v.dtype == np.uint32
                             else v).to(dev) for k, v in list(cols.items()) + list(tab.items())}
    na = 1 << 22
    st = torch.empty(na, dtype=torch.int32, device=dev)
    cm = torch.empty(na, dtype=torch.int32, device=dev)
    ps = torch.empty(na, dtype=torch.int64, device=dev)
    b = _lib.AttCheckBatch(na, t["slot"].data_ptr(), t["justified_slot"].data_ptr(), t["shard_id"].data_ptr(),
                           t["n_oblique"].data_ptr(), t["bits"].data_ptr(), t["boffs"].data_ptr(),
                           t["block_slot"].data_ptr(), 0, 0, 128, 256, t["arr_offs"].data_ptr(),
                           t["arr_shard"].data_ptr(), t["arr_comm"].data_ptr(), t["coffs"].data_ptr(),
                           st.data_ptr(), cm.data_ptr(), ps.data_ptr())
    for _ in range(3):
        _lib.lib.call("pz_dev_check_attestations", ctypes.byref(b), sh)
    # the bench's wire_att leg: the 1M config-2 records encoded from their columns
    from prysm_amd import wire
    cols = synth.attestation_columns_512(n, seed=2)
    tc = {k: torch.from_numpy(cols[k].view(np.int64) if cols[k].dtype == np.uint64 else cols[k]).to(dev)
          for k in wire.ATT_COLS}
    ac = _lib.AttestationCols(*[tc[k].data_ptr() for k in wire.ATT_COLS])
    a_out = torch.empty(n * 512 + 16, dtype=torch.uint8, device=dev)
    a_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    a_scr = torch.empty(int(_lib.lib.dll.pz_wire_attestations_scratch_bytes(n)), dtype=torch.uint8, device=dev)
    for _ in range(3):
        _lib.lib.call("pz_dev_wire_attestations", ctypes.byref(ac), n, 0, a_out.data_ptr(), a_offs.data_ptr(),
                      a_scr.data_ptr(), sh)
    torch.cuda.synchronize()
    print("pmc workload done")


if __name__ == "__main__":
    main()
