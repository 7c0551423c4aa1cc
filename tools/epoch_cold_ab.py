"""A/B of the epoch step's variants on cold data (tools/ only): python tools/epoch_cold_ab.py
Rotates the timed steps over 4 distinct instance sets on one stream (bench.py's --epoch-cold
form) for configs[2] (65,536 x 256) and the 1M x 16 shape, with pz_debug_set_fused_variant(v)
for each v in VARIANTS, and prints the device ms per step.  An entry "v/64" runs variant v with
PZ_EPOCH_BAL64 set (the u64 balance column instead of the product's u32 offsets; read at state
creation), "v/nl" with PZ_EPOCH_NO_LASTCO (no position-order reward-bit gather), "v/64/nl" both."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from prysm_amd import _lib, casper  # noqa: E402

VARIANTS = os.environ.get("VARIANTS", "0,0/64,0,0/64").split(",")


def main():
    dev = torch.device("cuda", 0)
    args = types.SimpleNamespace(steps=48)
    for nval, ninst in ((65536, 256), (1 << 20, 16)):
        shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
        for tag in VARIANTS:
            v, *flags = tag.split("/")
            v = int(v)
            for flag, env in (("64", "PZ_EPOCH_BAL64"), ("nl", "PZ_EPOCH_NO_LASTCO")):
                if flag in flags:
                    os.environ[env] = "1"
                else:
                    os.environ.pop(env, None)
            old = _lib.lib.dll.pz_debug_set_fused_variant(v)
            try:
                r = bench.epoch_cold(args, torch, dev, nval, ninst, shuffled, "epoch65k" if nval == 65536 else "epoch1m")
            finally:
                _lib.lib.dll.pz_debug_set_fused_variant(old)
            print("%7d x %3d variant %9s: step %.4f ms  frac(layout) %.3f  yardstick %.4f ms  layout yardstick "
                  "%.4f ms  (%s)" % (nval, ninst, tag, r["step_device_ms"], r["frac"], r["yardstick"]["ms"],
                                     r["yardstick_layout"]["ms"], r["what"]), flush=True)


if __name__ == "__main__":
    main()
