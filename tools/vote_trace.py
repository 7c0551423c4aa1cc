"""Where a replay's vote tally spends its time, from inside the kernel (tools/ only): one
configs[4] replay with PZ_VOTE_TRACE=1, then the per-wave phase stamps of its first flushes
(votes_dev.h PZ_VSTAMP, wall clock at 100 MHz) summarised per phase as the median over flushes
of the wave median and the wave maximum, in us since the flush's first wave started.

    python3 tools/vote_trace.py [nval=65536] [nblocks=10000]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PZ_VOTE_TRACE"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

from prysm_amd import _lib, synth  # noqa: E402
from prysm_amd.blockchain import BeaconChain, serialize_blocks  # noqa: E402

NAMES = ["wave start", "record loaded", "members/unions", "balances loaded", "word atomics returned",
         "wave done", "block flushed", "gather stored (last block)"]
FLUSHES, WAVES = 256, 512


def main():
    nval = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    nblocks = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    blocks = synth.chain_blocks(nval, nblocks, seed=6)
    data, offs = serialize_blocks(blocks)
    BeaconChain(nval).process_serialized(data, offs)  # warm-up (kernels loaded)
    ch = BeaconChain(nval)
    torch.cuda.synchronize()
    ch.process_serialized(data, offs)
    torch.cuda.synchronize()
    buf = np.zeros((FLUSHES, WAVES, 8), dtype=np.uint64)
    waves = np.zeros(FLUSHES, dtype=np.uint64)
    fn = _lib.lib.dll.pz_debug_vote_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    n = fn(ch._h, buf.ctypes.data, waves.ctypes.data, FLUSHES)
    per = [[] for _ in range(8)]
    for f in range(n):
        w = int(waves[f])
        if not w:
            continue
        t = buf[f, :w].astype(np.int64)
        t0 = t[:, 0][t[:, 0] > 0].min()
        for p in range(8):
            x = t[:, p][t[:, p] > 0]
            if len(x):
                per[p].append(((np.median(x) - t0) / 100.0, (x.max() - t0) / 100.0))
    print("%d flushes traced (%s waves each)" % (sum(1 for f in range(n) if waves[f]),
                                                  sorted(set(int(x) for x in waves[:n] if x))))
    for p in range(8):
        if per[p]:
            a = np.array(per[p])
            print("  %-28s wave median %6.2f us, wave max %6.2f us (medians over flushes)"
                  % (NAMES[p], np.median(a[:, 0]), np.median(a[:, 1])))


if __name__ == "__main__":
    main()
