"""e1: the H batch shard over one process per GPU (no collective in the hash; the digests are
all-gathered only to hand every rank the whole batch).  World 2 and 3 over gloo: on CPU the
kernel is replaced by hashlib (the test double), on the GPU the C-ABI kernels of every rank
share cuda:0.  Bit-exact against hashlib either way."""
import hashlib
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


def _batch(seed, n):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 900, size=n)
    msgs = [rng.bytes(int(k)) for k in lens]
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    return msgs, np.frombuffer(b"".join(msgs) + bytes(16), np.uint8), offs


def _cpu_hasher(data, offs):
    n = len(offs) - 1
    return np.array([np.frombuffer(hashlib.blake2b(data[int(offs[i]):int(offs[i + 1])].tobytes()).digest()[:32],
                                   np.uint8) for i in range(n)], dtype=np.uint8).reshape(n, 32)


def _worker(rank, world, port, n, use_gpu):
    for p in (ROOT, HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist

    from prysm_amd import _lib, types
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method="tcp://127.0.0.1:%d" % port)
    try:
        if use_gpu:
            _lib.lib.call("pz_init", 0)
        msgs, data, offs = _batch(n, n)
        with _lib.small_batch_threshold(0) if use_gpu else _Null():
            got = types.hash_batch_sharded(data, offs, rank, world, hasher=None if use_gpu else _cpu_hasher)
        want = np.array([np.frombuffer(hashlib.blake2b(m).digest()[:32], np.uint8) for m in msgs]).reshape(n, 32)
        np.testing.assert_array_equal(got, want)
        lo, hi = types.message_shard(n, rank, world)
        mine = types.hash_batch_sharded(data, offs, rank, world, group=False,
                                        hasher=None if use_gpu else _cpu_hasher)
        np.testing.assert_array_equal(mine, want[lo:hi])
    finally:
        dist.destroy_process_group()


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        pass


def _spawn(world, n, use_gpu):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), n, use_gpu), nprocs=world, join=True)


@pytest.mark.parametrize("world,n", [(2, 1001), (3, 5), (2, 1)])
def test_hash_shard_cpu_gloo(world, n):
    _spawn(world, n, use_gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("world,n", [(2, 20001), (3, 7)])
def test_hash_shard_gpu_gloo(world, n):
    _spawn(world, n, use_gpu=True)
