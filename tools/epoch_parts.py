"""Per-part device time of the two-pass epoch step (HIP events, one process, interleaved rounds).
Needs the A/B library's part entry points: PZ_PROBE_LIB=build/ab/libprysm_hip.so python tools/epoch_parts.py"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from prysm_amd import _lib, casper, synth  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):
    _lib.library_path = os.environ["PZ_PROBE_LIB"]
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from torch_epoch import DeviceEpoch  # noqa: E402


def main(nval=65536, ninst=256, rounds=5, reps=10):
    dll = _lib.lib.dll

    dev = torch.device("cuda", 0)
    sh_ = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
    inst = synth.epoch_batch(nval, ninst, seed=3, shuffled=sh_)
    de = DeviceEpoch(inst, dev)
    s = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(s.cuda_stream)
    bp = ctypes.byref(de.batch)
    parts = {
        "count_val": lambda: dll.pz_debug_epoch_count(bp, 1, 0, 0, sh),
        "count_pop": lambda: dll.pz_debug_epoch_count(bp, 0, 1, 0, sh),
        "count_xl": lambda: dll.pz_debug_epoch_count(bp, 0, 0, 1, sh),
        "count_all": lambda: dll.pz_debug_epoch_count(bp, 1, 1, 1, sh),
        "reward": lambda: dll.pz_debug_epoch_reward(bp, sh),
        # yardsticks on the same 16.7M x u64 balance array (same process, same device)
        "torch_copy": lambda: yard.copy_(de.balance.view(-1)),
        "torch_inplace_add": lambda: yard.add_(1),
    }
    yard = torch.empty(de.balance.numel(), dtype=torch.int64, device=dev)
    # overlap probes: the crosslink gathers on a second stream beside the validator stream
    s2 = torch.cuda.Stream(dev)
    sh2 = ctypes.c_void_p(s2.cuda_stream)
    ev_a, ev_b = torch.cuda.Event(), torch.cuda.Event()

    def two_streams(fa, fb):
        ev_a.record(s)
        s2.wait_event(ev_a)
        fa()
        fb()
        ev_b.record(s2)
        s.wait_event(ev_b)

    parts["xl_beside_val"] = lambda: two_streams(lambda: dll.pz_debug_epoch_count(bp, 1, 0, 0, sh),
                                                 lambda: dll.pz_debug_epoch_count(bp, 0, 0, 1, sh2))
    parts["xl_then_val_1stream"] = lambda: (dll.pz_debug_epoch_count(bp, 0, 0, 1, sh),
                                            dll.pz_debug_epoch_count(bp, 1, 0, 0, sh))
    # The parts run on the batch's CURRENT buffers: after a step those are the next step's
    # (zeroed) scal, so pass 2 would see pop = nact = 0 (threshold not met, general path).
    # Every pass-2 timing therefore restores a snapshot of a real pass-1 result first; the
    # restore alone is timed as "scal_restore" and subtracted.
    torch.cuda.synchronize()
    de.scal.zero_()
    dll.pz_dev_epoch_count(bp, sh)
    torch.cuda.synchronize()
    snap = de.red.clone()
    restore = lambda: de.red.copy_(snap)  # noqa: E731
    for k in [k for k in parts if k.startswith("reward")]:
        f0 = parts[k]
        parts[k] = (lambda f0=f0: (restore(), f0()))
    parts["scal_restore"] = restore
    parts["step"] = lambda: None  # timed separately below (it flips the buffers)
    res = {k: [] for k in parts}
    for r in range(rounds):
        for k, f in parts.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                f()
            e1.record(s)
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / reps * 1e3)
    med = {k: float(np.median(v)) for k, v in res.items()}
    for k in [k for k in med if k.startswith("reward")]:
        med[k] -= med["scal_restore"]
    st = []
    for r in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            de.step(s)
        e1.record(s)
        torch.cuda.synchronize()
        st.append(e0.elapsed_time(e1) / reps * 1e3)
    med["step"] = float(np.median(st))
    vb = nval * ninst
    print(json.dumps({"nval": nval, "ninst": ninst, "median_us": med,
                      "val_GBps": vb * 16 / (med["count_val"] * 1e-6) / 1e9,
                      "reward_GBps": vb * 16 / (med["reward"] * 1e-6) / 1e9,
                      "xl_GBps_algorithmic": vb * 12 / (med["count_xl"] * 1e-6) / 1e9}))


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    main(*a)
