"""Same-process A/B of the one-pass epoch step's build-time choices (tools/ only):
python tools/epoch_ab.py [ROUNDS]
Each arm sets environment knobs read when a pz_epoch_state is created (PZ_EPOCH_MULTI: one launch
over the B instances instead of pre + fused + mid; PZ_EPOCH_WIN_FUSED: winners in the fused waves,
no mid; PZ_EPOCH_SE64: the 64-bit start/end stream), builds 65,536 x 256 and 1M x 16 states and prints the device ms per step (one event
pair around 48 back-to-back steps, as bench.py's epoch leg)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from prysm_amd import casper, synth  # noqa: E402
from prysm_amd.native import NativeEpoch  # noqa: E402

ARMS = [("product", {}), ("multi", {"PZ_EPOCH_MULTI": "1"}), ("se64", {"PZ_EPOCH_SE64": "1"})]


def time_state(inst, dev, steps=48):
    for k, v in ARM_ENV.items():
        os.environ[k] = v
    try:
        de = NativeEpoch(inst, device=0)
    finally:
        for k in ARM_ENV:
            os.environ.pop(k, None)
    stream = torch.cuda.ExternalStream(de.shard(0)[3], device=dev)
    for _ in range(5):
        de.step()
    stream.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        de.step()
    e1.record(stream)
    stream.synchronize()
    de.free()
    return e0.elapsed_time(e1) / steps


ARM_ENV = {}


def main():
    global ARM_ENV
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda", 0)
    for nval, ninst in ((65536, 256), (1 << 20, 16)):
        shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
        inst = synth.epoch_batch(nval, ninst, seed=3, shuffled=shuffled)
        for r in range(rounds):
            for name, env in ARMS:
                ARM_ENV = env
                ms = time_state({k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in inst.items()}, dev)
                print("%7d x %3d round %d %-11s step %.4f ms" % (nval, ninst, r, name, ms), flush=True)


if __name__ == "__main__":
    main()
