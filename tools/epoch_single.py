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
    if os.environ.get("TRACE") == "1":
        return trace(args, dev, shuffled, dll)
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


def trace(args, dev, shuffled, dll):
    dll.pz_debug_set_one_trace.argtypes = [_lib.ctypes.c_void_p]
    buf = torch.zeros(8 * 4096, dtype=torch.int64, device=dev)
    dll.pz_debug_set_one_trace(buf.data_ptr())
    r = bench.epoch_single_instance(args, torch, dev, 65536, shuffled)
    torch.cuda.synchronize(dev)
    dll.pz_debug_set_one_trace(None)
    t = buf.view(-1, 8).cpu().numpy()
    t = t[t[:, 0] != 0]
    t0 = t[:, 0].min()
    us = lambda x: x * 0.01  # noqa: E731 (100 MHz)
    ph = {"start (after the first block's)": t[:, 0] - t0, "stream landed": t[:, 1] - t[:, 0],
          "count + barrier": t[:, 2] - t[:, 1], "tallies, rewards, stores": t[:, 3] - t[:, 2],
          "tail (block end, winners reset, drain)": t[:, 4] - t[:, 3]}
    print("traced kernel: %d blocks, span %.2f us (device median of the timed loop %.4f ms)"
          % (len(t), us(t[:, 4].max() - t0), r["device_ms_median"]), flush=True)
    for k, v in ph.items():
        print("  %-40s p50 %.2f  max %.2f us" % (k, us(np.median(v)), us(v.max())), flush=True)
    many = np.nonzero(t[:, 6])[0]
    if len(many):
        print("  several-attestation loop: " + ", ".join("block %d %.2f us (its sums done at %.2f)"
                                                      % (b, us(t[b, 6]), us(t[b, 7])) for b in many), flush=True)
    slow = np.argsort(t[:, 3] - t[:, 2])[-3:][::-1]
    print("  slowest 'tallies, rewards, stores' blocks (index: phase us): " +
          ", ".join("%d: %.2f" % (b, us(t[b, 3] - t[b, 2])) for b in slow), flush=True)


if __name__ == "__main__":
    main()
