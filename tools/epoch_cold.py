"""The product epoch step on cold data (tools/ only): python tools/epoch_cold.py
bench.py's epoch.cold form -- the timed steps rotated over distinct instance sets (>= 800 MB of
streamed state, far above the 256 MiB Infinity Cache) on one stream -- for configs[2]
(65,536 x 256) and the 1M x 16 shape, REPS times each, with the two stock-kernel yardsticks."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from prysm_amd import casper  # noqa: E402

REPS = int(os.environ.get("REPS", "2"))
SHAPES = [(65536, 256), (1 << 20, 16)]


def main():
    dev = torch.device("cuda", 0)
    args = types.SimpleNamespace(steps=48)
    for nval, ninst in SHAPES:
        shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
        for rep in range(REPS):
            r = bench.epoch_cold(args, torch, dev, nval, ninst, shuffled, "epoch65k" if nval == 65536 else "epoch1m")
            print("%7d x %3d rep %d: step %.4f ms  frac(layout) %.3f  yardstick %.4f ms  layout yardstick %.4f ms  (%s)"
                  % (nval, ninst, rep, r["step_device_ms"], r["frac"], r["yardstick"]["ms"],
                     r["yardstick_layout"]["ms"], r["what"]), flush=True)


if __name__ == "__main__":
    main()
