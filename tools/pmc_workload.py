"""Small fixed workload for rocprofv3 --pmc passes: 3 hash launches (1M x 512 B) and 3
epoch steps (65,536 validators x 256 instances), plus a torch copy as a bandwidth yardstick."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from prysm_amd import _lib, casper, synth  # noqa: E402
from prysm_amd.epoch import DeviceEpoch  # noqa: E402


def main():
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
    de = DeviceEpoch(inst, dev)
    for _ in range(3):
        de.step(s)
    x = torch.empty(nval * B, dtype=torch.int64, device=dev)
    for _ in range(3):
        x.copy_(de.balance.view(-1))
    torch.cuda.synchronize()
    print("pmc workload done")


if __name__ == "__main__":
    main()
