"""N>1 path of the epoch transition (validator-range shards + all-reduce / all-gather):
``tests/torch_epoch.py DeviceEpoch``'s multi-rank orchestration at world sizes 2 and 3, checked
bit-exact against the single-instance oracle.

* CPU (``-m "not gpu"``): gloo on CPU tensors, with the device passes replaced by the numpy
  test double ``tests/epoch_kernel_model.py`` — covers shard ranges, the reduced-buffer
  layout and the collective sequence.
* GPU (``-m gpu``): the same orchestration with the real HIP kernels (C ABI), two ranks
  sharing cuda:0 over gloo — covers the kernels' shard arithmetic (val_offset, popcount
  chunk split, partial crosslink tallies, the gathered-mask global compaction).
"""
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


def _worker(rank, world, port, n, B, inactive, use_gpu, steps):
    for p in (ROOT, HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    from epoch_ref_helpers import oracle_epoch
    from oracle import ref
    from prysm_amd import _lib, casper, synth
    from torch_epoch import DeviceEpoch, shard_range

    dist.init_process_group("gloo", rank=rank, world_size=world, init_method="tcp://127.0.0.1:%d" % port)
    shuffled = casper.shuffle_indices(ref.bytes_to_hash(b"A"), np.arange(n, dtype=np.uint32)) if use_gpu \
        else np.random.default_rng(7).permutation(n).astype(np.uint32)
    inst = synth.epoch_batch(n, B, seed=11, shuffled=shuffled)
    if inactive:  # general rank path: rank != index
        rng = np.random.default_rng(2)
        inst["start"][:, rng.random(n) < 0.1] = 7
        inst["end"][:, rng.random(n) < 0.1] = 1
    try:
        if use_gpu:
            _lib.lib.call("pz_init", 0)
            dev, kernels = torch.device("cuda", 0), None
        else:
            from epoch_kernel_model import NumpyEpochKernels
            dev, kernels = torch.device("cpu"), NumpyEpochKernels()
        de = DeviceEpoch(inst, dev, rank=rank, world=world, kernels=kernels)
        assert de.general == (inactive and world > 1)
        lo, hi = shard_range(n, rank, world)
        for _ in range(steps):
            de.step()
            if use_gpu:
                torch.cuda.synchronize()
            bal, scal, vote, total, win = de.results()
            for b in range(B):
                nb, applied, nxt, v, t, w = oracle_epoch(inst, b)
                assert bool(scal[b, _lib.SCAL_APPLIED]) == applied, (rank, b)
                np.testing.assert_array_equal(bal[b], nb[lo:hi])
                assert int(scal[b, _lib.SCAL_NEXT_BAL]) == nxt, (rank, b)
                np.testing.assert_array_equal(vote[b], v)
                np.testing.assert_array_equal(total[b], t)
                np.testing.assert_array_equal(win[b], w)
                inst["balance"][b] = nb
    finally:
        dist.destroy_process_group()


def _spawn(world, n, B, inactive, use_gpu, steps=2):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), n, B, inactive, use_gpu, steps), nprocs=world, join=True)


@pytest.mark.parametrize("world,n,B,inactive", [(2, 4096, 2, False), (2, 4096, 2, True), (3, 5000, 2, True),
                                                (8, 20000, 1, True)])
def test_multirank_epoch_cpu_gloo(world, n, B, inactive):
    _spawn(world, n, B, inactive, use_gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("n,B,inactive", [(65536, 3, False), (20000, 2, True)])
def test_multirank_epoch_gpu_gloo(n, B, inactive):
    _spawn(2, n, B, inactive, use_gpu=True)


@pytest.mark.gpu
@pytest.mark.parametrize("inactive", [False, True])
def test_multirank_epoch_gpu_gloo_configs3(inactive):
    """BASELINE configs[3] exactly: 1,048,576 validators sharded over 8 ranks (131,072 each),
    the real 1M shuffle (65 committees per slot), every rank's HIP kernels on cuda:0 and the
    sums combined over gloo; bit-exact against the oracle on every rank's balance slice."""
    _spawn(8, 1 << 20, 1, inactive, use_gpu=True, steps=1)
