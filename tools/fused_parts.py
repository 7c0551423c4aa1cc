"""Ablation of the one-pass epoch kernel (pz_debug_set_fused_variant): device time of a
pz_epoch_state step per variant, interleaved rounds, HIP events on the state's stream.
Variant bits (epoch.hip fused_body): 1 no tallies, 2 no last-bitfield lookups, 4 no store,
8 no start/end loads, 16 default-policy
start/end loads, 32 instance-major grid, 64 the piece from its index (no item -> stream hop), 1024
the packed start/end column (1024 alone: the product's kernel without the reward-bit gather).  Results are wrong for variants != 0 (timing only)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from prysm_amd import _lib, casper, synth  # noqa: E402
from prysm_amd.native import NativeEpoch  # noqa: E402

VARIANTS = [int(x) for x in os.environ.get("VARIANTS", "0,128,1,2,4,8,15,16,32").split(",")]


def run(nval, ninst, rounds=5, reps=10):
    dll = _lib.lib.dll
    dev = torch.device("cuda", 0)
    sh_ = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
    inst = synth.epoch_batch(nval, ninst, seed=3, shuffled=sh_)
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass
    _, _, _, sp = ne.shard(0)
    s = torch.cuda.ExternalStream(sp, device=dev)
    yard = torch.empty(nval * ninst, dtype=torch.int64, device=dev)
    yard2 = torch.empty_like(yard)
    res = {v: [] for v in VARIANTS}
    res["torch_copy_balance"] = []
    for _ in range(3):
        ne.step()
    ne.sync()
    for _ in range(rounds):
        for v in VARIANTS + ["torch_copy_balance"]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                if v == "torch_copy_balance":
                    e0.record(s)
                    for _ in range(reps):
                        yard2.copy_(yard)
                    e1.record(s)
                else:
                    dll.pz_debug_set_fused_variant(v)
                    ne.step()  # warm this variant
                    e0.record(s)
                    for _ in range(reps):
                        ne.step()
                    e1.record(s)
                    dll.pz_debug_set_fused_variant(0)
            e1.synchronize()
            res[v].append(e0.elapsed_time(e1) * 1e3 / reps)
    ne.free()
    return {str(k): round(float(np.median(x)), 2) for k, x in res.items()}


def main():
    out = {"note": "us per pz_epoch_state step (pre + fused + winners) by fused variant; "
                   "1 no tallies, 2 no last-bitfield lookups, 4 no store, 8 no start/end loads, "
                   "16 default-policy start/end loads, 32 instance-major grid, 128 reward bits looked up in the fused pass (no position-order gather)",
           "65536x256": run(65536, 256), "1048576x16": run(1 << 20, 16)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
