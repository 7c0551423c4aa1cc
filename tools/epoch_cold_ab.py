"""A/B of the epoch step's variants on cold data (tools/ only): python tools/epoch_cold_ab.py
Rotates the timed steps over 4 distinct instance sets on one stream (bench.py's --epoch-cold
form) for configs[2] (65,536 x 256) and the 1M x 16 shape, with pz_debug_set_fused_variant(v)
for each v in VARIANTS, and prints the device ms per step."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from prysm_amd import _lib, casper  # noqa: E402

VARIANTS = [int(x) for x in os.environ.get("VARIANTS", "0,128,0,128").split(",")]


def main():
    dev = torch.device("cuda", 0)
    args = types.SimpleNamespace(steps=48)
    for nval, ninst in ((65536, 256), (1 << 20, 16)):
        shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
        for v in VARIANTS:
            old = _lib.lib.dll.pz_debug_set_fused_variant(v)
            try:
                r = bench.epoch_cold(args, torch, dev, nval, ninst, shuffled, "epoch65k" if nval == 65536 else "epoch1m")
            finally:
                _lib.lib.dll.pz_debug_set_fused_variant(old)
            print("%7d x %3d variant %3d: step %.4f ms  frac(8d) %.3f  yardstick %.4f ms" % (
                nval, ninst, v, r["step_device_ms"], r["frac"], r["yardstick"]["ms"]), flush=True)


if __name__ == "__main__":
    main()
