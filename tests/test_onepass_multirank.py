"""N>1 path of the ONE-PASS epoch step (committee-order layout, epoch_state.hip
step_sharded_fused) on CPU: the library's own host planner ``pz_epoch_plan`` (no device call)
places every rank, the numpy test double ``tests/onepass_model.py`` stands in for the three
kernels of one rank, and the collectives run over ``gloo`` at world sizes 2, 3 and 5:
u64 SUM of the scalars, u32 MIN of the owner-proposed winners, then SUM of vote/total
(``pz_epoch_state_tallies``).  Every rank's results are checked bit-exact against the oracle
(blockchain/core.go:433-464).  The GPU tests (tests/test_native_gpu.py) run the same protocol
with the HIP kernels over the loopback and RCCL communicators."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inst(n, B, seed=5, dup=0, density=0.75):
    """synth.epoch_batch (every validator active) with ``dup`` attestations moved to another
    committee of the same size: committees with zero and with several attestations."""
    from prysm_amd import synth
    shuffled = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    inst = synth.epoch_batch(n, B, seed=seed, shuffled=shuffled, density=density)
    if dup:
        rng = np.random.default_rng(seed + 1)
        coffs = inst["coffs"].astype(np.int64)
        size = np.diff(coffs)
        natt = inst["natt"]
        inst["att_comm"] = ac = inst["att_comm"].copy()
        for _ in range(dup):
            g = int(rng.integers(0, natt - 1))  # keep the final (nval-bit) attestation
            for b in range(B):
                c = int(ac[b * natt + g])
                same = np.flatnonzero(size == size[c])
                ac[b * natt + g] = same[int(rng.integers(0, same.size))]
    return inst


def _worker(rank, world, port, n, B, dup, steps):
    for p in (ROOT, HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    from epoch_ref_helpers import oracle_epoch
    from onepass_model import rank_step
    from prysm_amd.native import epoch_plan

    dist.init_process_group("gloo", rank=rank, world_size=world, init_method="tcp://127.0.0.1:%d" % port)
    try:
        inst = _inst(n, B, dup=dup)
        lo, hi, layout = epoch_plan(inst, world, rank)
        assert layout == 2, layout
        co = inst["committee"].astype(np.int64)
        natt = inst["natt"]
        for _ in range(steps):
            parts = [rank_step(inst, b, rank, lo, hi) for b in range(B)]
            scal = torch.tensor([[p[1], p[2], p[3]] for p in parts], dtype=torch.int64)
            win = torch.tensor(np.stack([p[6] for p in parts]), dtype=torch.int64)
            dist.all_reduce(scal, op=dist.ReduceOp.SUM)
            dist.all_reduce(win, op=dist.ReduceOp.MIN)
            # before the tallies collective: vote/total complete exactly where this rank owns
            coffs = inst["coffs"].astype(np.int64)
            for b in range(B):
                cb = coffs[inst["att_comm"][b * natt:(b + 1) * natt]]
                own = (cb >= lo) & ((cb < hi) | ((cb == n) & (hi == n)))
                _, _, _, v, t, _ = oracle_epoch(inst, b)
                np.testing.assert_array_equal(parts[b][4][own], v[own])
                np.testing.assert_array_equal(parts[b][5][own], t[own])
            tallies = torch.tensor(np.stack([np.stack([p[4], p[5]]) for p in parts]).view(np.int64))
            dist.all_reduce(tallies, op=dist.ReduceOp.SUM)
            tallies = tallies.numpy().view(np.uint64)
            for b in range(B):
                nb, applied, nxt, v, t, w = oracle_epoch(inst, b)
                assert int(scal[b, 0]) == int(np.unpackbits(inst["bits"][
                    inst["boffs"][b * natt]:inst["boffs"][(b + 1) * natt]]).sum()), (rank, b)
                assert bool(scal[b, 1]) == applied, (rank, b)
                assert int(scal[b, 2]) % (1 << 64) == nxt, (rank, b)
                np.testing.assert_array_equal(parts[b][0], nb[co[lo:hi]])
                np.testing.assert_array_equal(tallies[b, 0], v)
                np.testing.assert_array_equal(tallies[b, 1], t)
                np.testing.assert_array_equal(win[b].numpy().astype(np.uint32), w)
                inst["balance"][b] = nb
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,B,dup", [(2, 4096, 2, 0), (2, 5000, 2, 20), (3, 4099, 2, 40), (5, 3000, 3, 30)])
def test_onepass_sharded_cpu_gloo(world, n, B, dup):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), n, B, dup, 2), nprocs=world, join=True)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8, 16])
def test_epoch_plan_committee_aligned(world):
    """pz_epoch_plan (host only): the ranks' ranges tile [0, N) in order, every boundary is a
    committee start (so no committee straddles two ranks), and each is the committee start
    nearest the even split."""
    from prysm_amd.native import epoch_plan
    n = 20000
    inst = _inst(n, 1)
    coffs = inst["coffs"].astype(np.int64)
    starts = set(coffs.tolist())
    prev = 0
    for r in range(world):
        lo, hi, layout = epoch_plan(inst, world, r)
        assert layout == 2
        assert lo == prev and hi >= lo
        assert lo in starts and hi in starts
        if world > 1 and r + 1 < world:
            t = n * (r + 1) // world
            assert abs(hi - t) == np.abs(coffs - t).min()  # nearest committee start
        prev = hi
    assert prev == n


def test_epoch_plan_layouts():
    """The plan's layout choice (epoch_state.hip plan_layout): one pass when every validator is
    active, the committees partition the set and no attestation names a shard >= nrec;
    committee order with the two-pass step for such a shard or on request; index order (and
    64-aligned ranges) when some validator is inactive or on request."""
    from prysm_amd.native import epoch_plan
    n = 5000
    inst = _inst(n, 2)
    assert epoch_plan(inst, 2, 0)[2] == 2
    assert epoch_plan(inst, 2, 0, layout="twopass")[2] == 1
    assert epoch_plan(inst, 2, 0, layout="index")[2] == 0
    lo, hi, _ = epoch_plan(inst, 2, 0, layout="twopass")
    assert (lo, hi) == (0, 64 * ((n + 127) // 128))  # 64-aligned split unless one pass
    shard = dict(inst, att_shard=inst["att_shard"].copy())
    shard["att_shard"][3] = 10 ** 6
    assert epoch_plan(shard, 1, 0)[2] == 1
    inactive = dict(inst, end=inst["end"].copy())
    inactive["end"][1, 17] = 0
    assert epoch_plan(inactive, 1, 0)[2] == 0
    bad = dict(inst, committee=inst["committee"].copy())
    bad["committee"][0] = bad["committee"][1]  # not a partition: index order
    assert epoch_plan(bad, 1, 0)[2] == 0
    from prysm_amd._lib import PzError
    with pytest.raises(PzError):
        epoch_plan(inst, 2, 2)
