"""The product epoch step on WARM data (tools/ only): python tools/epoch_warm.py
bench.py's epoch leg -- K back-to-back steps of ONE instance set, so the balances the step
writes may still sit in the 256 MiB Infinity Cache when the next step reads them -- for
configs[2] (65,536 x 256) and 1M x 16, per window-pass ablation (ABL=a,b,... with
PZ_PROBE_LIB=build/ab/libprysm_hip.so; epoch_window.hip's A/B bits)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from prysm_amd import _lib, casper, synth  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):  # (A/B: another build of the library)
    _lib.library_path = os.environ["PZ_PROBE_LIB"]
from prysm_amd.native import NativeEpoch  # noqa: E402

SHAPES = [(65536, 256), (1 << 20, 16)]
ABL = [int(x, 0) for x in os.environ.get("ABL", "0").split(",") if x]
STEPS, REPS = int(os.environ.get("STEPS", "40")), int(os.environ.get("REPS", "2"))


def main():
    dll = _lib.lib.dll if any(ABL) else None
    for nval, ninst in SHAPES:
        shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
        de = NativeEpoch(synth.epoch_batch(nval, ninst, seed=3, shuffled=shuffled), device=0)
        stream = torch.cuda.Stream(device=0)
        de.bind_stream(stream.cuda_stream)
        for abl in ABL:
            if dll is not None:
                dll.pz_debug_set_window_ablation(abl)
            for rep in range(REPS):
                for _ in range(5):
                    de.step()
                stream.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(STEPS):
                    de.step()
                e1.record(stream)
                stream.synchronize()
                ms = e0.elapsed_time(e1) / STEPS
                bpv = 2 * de.balance_bytes + de.dynasty_bytes + 0.25
                print("%7d x %3d abl 0x%x rep %d: warm step %.4f ms  frac(layout) %.3f"
                      % (nval, ninst, abl, rep, ms, nval * ninst * bpv / (ms * 1e-3) / 8e12), flush=True)
        if dll is not None:
            dll.pz_debug_set_window_ablation(0)
        de.free()


if __name__ == "__main__":
    main()
