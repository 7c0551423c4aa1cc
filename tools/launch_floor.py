"""The floor under a single-kernel latency measured the way bench.py's epoch.single_instance
is: the median HIP-event pair around (a) nothing, (b) one tiny torch kernel, (c) the one-launch
epoch step at 65,536 validators, on the same stream, plus back-to-back rates.

    python tools/launch_floor.py [STEPS]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from prysm_amd import casper, synth  # noqa: E402
from prysm_amd.native import NativeEpoch  # noqa: E402


def pairs(stream, fn, k):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for e0, e1 in evs:
        e0.record(stream)
        fn()
        e1.record(stream)
    stream.synchronize()
    b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b0.record(stream)
    for _ in range(k):
        fn()
    b1.record(stream)
    stream.synchronize()
    t = [e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]
    return np.median(t), np.percentile(t, 10), b0.elapsed_time(b1) * 1e3 / k


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(65536, dtype=np.uint32))  # as bench.py
    de = NativeEpoch(synth.epoch_batch(65536, 1, seed=3, shuffled=shuffled), device=0)
    stream = torch.cuda.ExternalStream(de.shard(0)[3], device=dev)
    x = torch.zeros(1, device=dev)
    for _ in range(50):
        de.step()
    stream.synchronize()

    def tiny():
        with torch.cuda.stream(stream):
            x.add_(1)

    for name, fn in (("nothing", lambda: None), ("tiny torch kernel", tiny), ("epoch one-launch step", de.step)):
        pairs(stream, fn, 20)
        med, p10, b2b = pairs(stream, fn, k)
        print("%-24s event pair median %6.2f us  p10 %6.2f us  back-to-back %6.2f us/step" % (name, med, p10, b2b))
    t0 = time.perf_counter()
    for _ in range(k):
        de.step()
    stream.synchronize()
    print("epoch step host wall %.2f us/step" % ((time.perf_counter() - t0) / k * 1e6))
    de.free()


if __name__ == "__main__":
    main()
