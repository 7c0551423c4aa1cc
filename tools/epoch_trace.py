"""Phase stamps of the window pass (tools/ only; the A/B library's pz_debug_set_window_trace):
python tools/epoch_trace.py -- per block {start, prologue done, loop done, end} by
s_memrealtime (100 MHz) on cold steps of bench.py's rotation, summarised per step: the
dispatch spread of the block starts, each phase's median / max, and the last block's phases."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from prysm_amd import _lib, casper, synth  # noqa: E402

_lib.library_path = os.environ.get("PZ_PROBE_LIB") or os.path.join(ROOT, "build", "ab", "libprysm_hip.so")
from prysm_amd.native import NativeEpoch  # noqa: E402

SHAPES = [(1 << 20, 16), (65536, 256)]
NSETS, STEPS = 6, 4


def main():
    dll = _lib.lib.dll
    dll.pz_debug_set_window_trace.argtypes = [_lib.ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    abl = int(os.environ.get("ABL", "0"), 0)
    dll.pz_debug_set_window_ablation(abl)
    for nval, ninst in SHAPES:
        shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
        stream = torch.cuda.Stream(device=dev)
        sets = []
        for k in range(NSETS):
            de = NativeEpoch(synth.epoch_batch(nval, ninst, seed=3 + k, shuffled=shuffled), device=0)
            de.bind_stream(stream.cuda_stream)
            sets.append(de)
        for _ in range(2):
            for de in sets:
                de.step()
        stream.synchronize()
        tr = torch.zeros(4 * 8192, dtype=torch.int64, device=dev)
        for s in range(STEPS):
            tr.zero_()
            torch.cuda.synchronize()
            dll.pz_debug_set_window_trace(tr.data_ptr())
            sets[s % NSETS].step()
            stream.synchronize()
            dll.pz_debug_set_window_trace(None)
            t = tr.cpu().numpy().reshape(-1, 4)
            t = t[t[:, 0] != 0].astype(np.float64) / 100.0  # -> us
            t0 = t[:, 0].min()
            st, pro, loop, epi = t[:, 0] - t0, t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
            last = int(np.argmax(t[:, 3]))
            print("%7d x %3d abl 0x%x step %d: %d blocks, span %.1f us | start spread p50 %.1f max %.1f | prologue p50 "
                  "%.1f max %.1f | loop p50 %.1f max %.1f | epilogue p50 %.1f max %.1f | last block %d: start %.1f "
                  "prologue %.1f loop %.1f epilogue %.1f"
                  % (nval, ninst, abl, s, len(t), t[:, 3].max() - t0, np.median(st), st.max(), np.median(pro),
                     pro.max(), np.median(loop), loop.max(), np.median(epi), epi.max(), last, st[last], pro[last],
                     loop[last], epi[last]), flush=True)
        for de in sets:
            de.free()
    dll.pz_debug_set_window_ablation(0)


if __name__ == "__main__":
    main()
