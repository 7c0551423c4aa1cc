"""Per-transition host timeline of one configs[4] replay (pz_debug_chain_timeline), written as
JSON for correlation with a rocprofv3 kernel trace of the same run (tools/ only):

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 tools/replay_timeline.py OUT/timeline.json

Each transition: CLOCK_MONOTONIC ns at the flush's start, after its tally launch returned, after
the epoch's launches returned, and when the totals' sequence word was seen (rocprofv3's kernel
timestamps are on the same clock)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from prysm_amd import _lib, synth  # noqa: E402
from prysm_amd.blockchain import BeaconChain, serialize_blocks  # noqa: E402


def main():
    out = sys.argv[1]
    nval, nblocks = 65536, 10000
    blocks = synth.chain_blocks(nval, nblocks, seed=6)
    data, offs = serialize_blocks(blocks)
    BeaconChain(nval).process_serialized(data, offs)  # warm-up
    ch = BeaconChain(nval)
    torch.cuda.synchronize()
    ch.process_serialized(data, offs)
    torch.cuda.synchronize()
    buf = np.zeros(4 * 4096, dtype=np.uint64)
    fn = _lib.lib.dll.pz_debug_chain_timeline
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    n = fn(ch._h, buf.ctypes.data, 4096)
    tl = buf[: 4 * min(n, 4096)].reshape(-1, 4).tolist()
    with open(out, "w") as f:
        json.dump({"transitions": tl}, f)
    d = np.diff(np.array(tl, dtype=np.int64), axis=1) / 1e3
    print("transitions %d: launch %.1f us, epoch launches %.1f us, wait %.1f us (medians)"
          % (len(tl), *np.median(d, axis=0)))


if __name__ == "__main__":
    main()
