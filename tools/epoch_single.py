"""The single-instance epoch's latency (tools/ only): python tools/epoch_single.py
bench.py's epoch.single_instance measure (one 65,536-validator instance, the single launch,
HIP-event pair per step, median) per A/B form of the single launch (PZ_PROBE_LIB=build/ab/...,
ONE=a,b,...: pz_debug_set_one_variant -- 0 the product, 1 the piece positions from the item
table, round 5's form)."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from prysm_amd import _lib, casper  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):  # (A/B: another build of the library)
    _lib.library_path = os.environ["PZ_PROBE_LIB"]
import bench  # noqa: E402

VARIANTS = [int(x, 0) for x in os.environ.get("ONE", "0,1,0,1").split(",") if x]


def main():
    dev = torch.device("cuda", 0)
    args = types.SimpleNamespace(steps=200, warmup=20)
    shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(65536, dtype=np.uint32))
    dll = _lib.lib.dll
    ab = hasattr(dll, "pz_debug_set_one_variant")
    for v in VARIANTS if ab else [0]:
        if ab:
            dll.pz_debug_set_one_variant(v)
        r = bench.epoch_single_instance(args, torch, dev, 65536, shuffled)
        print("variant %d: device %.4f ms median (net of the event floor %.4f)  back-to-back %.4f ms  window pass %.4f"
              % (v, r["device_ms_median"], r["device_ms_net_of_event_floor"], r["back_to_back_ms_per_step"],
                 r["window_pass"]["device_ms_median"]), flush=True)
    if ab:
        dll.pz_debug_set_one_variant(0)


if __name__ == "__main__":
    main()
