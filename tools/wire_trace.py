"""Per-tile phase timeline of pz_wire_val_kernel (wire.hip variant 32: the product kernel plus
100 MHz wall-clock stamps per tile) on the bench's wire workload (16 states x 1,048,576
validators).  Prints the median duration of each phase of a tile's life, the dispatch spread
and how many tiles were resident over time: where the lifetime that bounds the kernel goes."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from prysm_amd import _lib  # noqa: E402

PHASES = ["ticket", "sizes+publish", "stage build", "look-back wait", "store"]


def main():
    n = 16 << 20
    rng = np.random.default_rng(7)
    cols_np = [rng.integers(16, 49, size=n, dtype=np.uint64), np.zeros(n, np.uint64),
               np.full(n, 9999999999999999999, np.uint64)]
    cols_t = [torch.from_numpy(a.view(np.int64)).cuda() for a in cols_np]
    dll = _lib.lib.dll
    out = torch.empty(int(dll.pz_wire_validators_bound(n, 0)), dtype=torch.uint8, device="cuda")
    scr = torch.empty(int(dll.pz_wire_scratch_bytes(n)) // 8, dtype=torch.int64, device="cuda")
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    nt = (n + 4095) // 4096
    trace = torch.zeros(nt * 16, dtype=torch.int64, device="cuda")
    cols = _lib.ValidatorCols(None, None, None, None, None, None, *[t.data_ptr() for t in cols_t])
    sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        _lib.lib.call("pz_dev_wire_validators", ctypes.byref(cols), n, 11, out.data_ptr(), None, scr.data_ptr(),
                      tot.data_ptr(), sh)

    for _ in range(5):
        run()
    ref = out[:int(tot.item())].clone()
    dll.pz_debug_set_wire_trace(ctypes.c_void_p(trace.data_ptr()))
    variant = int(sys.argv[1]) if len(sys.argv) > 1 else 32  # 34: no stage build, 36: no look-back, 288: time the first poll
    dll.pz_debug_set_wire_variant(variant)
    res = []
    for rep in range(5):
        run()
        torch.cuda.synchronize()
        t = trace.cpu().numpy().reshape(nt, 16)
        ts = t[:, :6].astype(np.int64)
        same = bool(torch.equal(out[:ref.numel()], ref)) if variant in (32, 544) else None
        t0 = ts[:, 0].min()
        d = np.diff(ts, axis=1) * 10 / 1e3  # us (100 MHz)
        life = (ts[:, 5] - ts[:, 0]) * 10 / 1e3
        span = (ts[:, 5].max() - t0) * 10 / 1e3
        # residency: tiles alive at each 1-us point
        grid = np.arange(0, span, 1.0)
        st, en = (ts[:, 0] - t0) * 10 / 1e3, (ts[:, 5] - t0) * 10 / 1e3
        alive = np.searchsorted(np.sort(st), grid, side="right") - np.searchsorted(np.sort(en), grid, side="right")
        xcc = t[:, 6] & 15
        res.append({
            "output_identical_to_product": same,
            "span_us": round(float(span), 1),
            "lifetime_us": {"median": round(float(np.median(life)), 2), "p90": round(float(np.percentile(life, 90)), 2)},
            "phase_median_us": {p: round(float(np.median(d[:, k])), 2) for k, p in enumerate(PHASES)},
            "phase_p90_us": {p: round(float(np.percentile(d[:, k], 90)), 2) for k, p in enumerate(PHASES)},
            "phase_share_of_lifetime": {p: round(float(d[:, k].sum() / life.sum()), 3) for k, p in enumerate(PHASES)},
            "resident_tiles_median": int(np.median(alive[len(alive) // 10: -len(alive) // 10 or None])),
            "tiles_per_xcc": np.bincount(xcc, minlength=8).tolist(),
            "first_wave_lookback_us": round(float(np.median(d[np.argsort(ts[:, 0])[:512], 3])), 2),
            "late_wave_lookback_us": round(float(np.median(d[np.argsort(ts[:, 0])[-1024:], 3])), 2),
            "thread0_repolls": {"median": float(np.median(t[1:, 9])), "p90": float(np.percentile(t[1:, 9], 90)),
                                "max": int(t[1:, 9].max())},
            "nearest_prefix_distance": {"median": float(np.median(t[1:, 10])),
                                        "p90": float(np.percentile(t[1:, 10], 90))},
            "build_end_last_wave_after_thread0_us": round(float(np.median((t[:, 11] - ts[:, 3]) * 10 / 1e3)), 2),
            "repolls_most_of_any_thread": {"median": float(np.median(t[1:, 12])), "p90": float(np.percentile(t[1:, 12], 90))},
            "first_window_round_trip_us": (round(float(np.median((t[1:, 8] - ts[1:, 2]) * 10 / 1e3)), 2)
                                           if variant & 256 else None),
            # thread 0 inside the look-back (tiles > 0): build end -> every flag seen -> window
            # reduced (its barrier) -> the phase's end
            "lookback_flags_us": round(float(np.median((t[1:, 13] - ts[1:, 3]) * 10 / 1e3)), 2),
            "lookback_reduce_us": round(float(np.median((t[1:, 14] - t[1:, 13]) * 10 / 1e3)), 2),
            "lookback_tail_us": round(float(np.median((ts[1:, 4] - t[1:, 14]) * 10 / 1e3)), 2),
            "lookback_return_us": round(float(np.median((t[1:, 15] - t[1:, 14]) * 10 / 1e3)), 2),
            "prefix_store_us": (round(float(np.median((t[1:, 8] - t[1:, 15]) * 10 / 1e3)), 2)
                                if not variant & 256 else None),
        })
    dll.pz_debug_set_wire_variant(0)
    dll.pz_debug_set_wire_trace(None)
    print(json.dumps({"tiles": nt, "variant": variant, "runs": res}, indent=1))


if __name__ == "__main__":
    main()
