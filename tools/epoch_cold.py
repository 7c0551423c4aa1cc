"""The product epoch step on cold data (tools/ only): python tools/epoch_cold.py
bench.py's epoch.cold form -- the timed steps rotated over distinct instance sets (>= 800 MB of
streamed state, far above the 256 MiB Infinity Cache) on one stream -- for configs[2]
(65,536 x 256) and the 1M x 16 shape, REPS times each, with the two stock-kernel yardsticks.
With PZ_PROBE_LIB=build/ab/libprysm_hip.so, ABL=a,b,... repeats it per window-pass ablation
(epoch_window.hip: bits 1 no tallies, 2 no prologue count, 4 no reward lookups, 8 no vote-bit
placement; depth << 8 the full kernel at that prefetch depth)."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from prysm_amd import _lib, casper  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):  # (A/B: another build of the library)
    _lib.library_path = os.environ["PZ_PROBE_LIB"]

REPS = int(os.environ.get("REPS", "2"))
SHAPES = [(65536, 256), (1 << 20, 16)]
ABL = [int(x, 0) for x in os.environ.get("ABL", "").split(",") if x]


def main():
    dev = torch.device("cuda", 0)
    args = types.SimpleNamespace(steps=48)
    dll = None
    if ABL:
        dll = _lib.lib.dll
    for nval, ninst in SHAPES:
        shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
        for abl in ABL or [None]:
            if dll is not None:
                dll.pz_debug_set_window_ablation(abl)
            for rep in range(REPS):
                r = bench.epoch_cold(args, torch, dev, nval, ninst, shuffled, "epoch65k" if nval == 65536 else "epoch1m")
                print("%7d x %3d %s rep %d: step %.4f ms  frac(layout) %.3f  yardstick %.4f ms  layout yardstick %.4f ms  (%s)"
                      % (nval, ninst, "" if abl is None else "abl 0x%x" % abl, rep, r["step_device_ms"], r["frac"],
                         r["yardstick"]["ms"], r["yardstick_layout"]["ms"], r["what"]), flush=True)
    if dll is not None:
        dll.pz_debug_set_window_ablation(0)


if __name__ == "__main__":
    main()
