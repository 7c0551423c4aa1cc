"""Drop-in Hash() latency: pz_blake2b512_batch (host pointers) for n messages of `len` bytes,
GPU route (small-batch threshold 0) vs calling-thread route, median wall time per call."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (binds the library to torch's HIP runtime, as the bench does)

from prysm_amd import _lib  # noqa: E402


def timed(data, offs, n, reps):
    out = np.empty(n * 32, dtype=np.uint8)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _lib.lib.call("pz_blake2b512_batch", _lib.ptr(data), _lib.ptr(offs), n, _lib.ptr(out), 32)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def main():
    _lib.lib.call("pz_init", 0)
    rng = np.random.default_rng(1)
    rows = []
    for ln in (100, 300, 600):
        for n in (1, 2, 4, 8, 16, 32, 64, 128, 256, 1024, 4096):
            data = rng.integers(0, 256, size=n * ln + 16, dtype=np.uint8)
            offs = np.arange(n + 1, dtype=np.uint64) * ln
            comps = n * ((ln + 127) // 128)
            with _lib.small_batch_threshold(0):
                timed(data, offs, n, 5)
                gpu = timed(data, offs, n, 50)
            with _lib.small_batch_threshold(1 << 62):
                host = timed(data, offs, n, 50)
            rows.append({"len": ln, "n": n, "compressions": comps, "gpu_us": gpu, "host_us": host})
            print(json.dumps(rows[-1]), flush=True)
    cross = [r["compressions"] for r in rows if r["host_us"] > r["gpu_us"]]
    print(json.dumps({"summary": "first batch size (compressions) where the GPU route wins, per length",
                      "per_len": {ln: min([r["compressions"] for r in rows if r["len"] == ln and r["host_us"] > r["gpu_us"]],
                                          default=None) for ln in (100, 300, 600)},
                      "min_over_lengths": min(cross) if cross else None}))


if __name__ == "__main__":
    main()
