"""The SHM communicator's process group (prysm_amd/csrc/shm_group.cpp) on the host alone: the
collectives pz_comm_init_shm stages through host memory, run by separate processes (no GPU
involved).  The GPU side -- the sharded epoch and one chain over processes sharing cuda:0 --
is tests/test_shm_multiprocess_gpu.py."""
import ctypes
import multiprocessing as mp
import os
import uuid

import numpy as np
import pytest

from ab_lib import ab_dll
from prysm_amd import _lib


def _dll():
    d = ab_dll()
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    d.pz_debug_shm_open.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, u64,
                                    ctypes.POINTER(vp)]
    d.pz_debug_shm_sum_u64.argtypes = [vp, vp, u64]
    d.pz_debug_shm_min_u32.argtypes = [vp, vp, u64]
    d.pz_debug_shm_sum_min.argtypes = [vp, vp, u64, vp, u64]
    d.pz_debug_shm_allgather.argtypes = [vp, vp, vp, u64]
    d.pz_debug_shm_close.argtypes = [vp]
    d.pz_debug_shm_error.restype = ctypes.c_char_p
    return d


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _inputs(rank, n):
    rng = np.random.default_rng(100 + rank)
    return (rng.integers(0, 2**64, size=n, dtype=np.uint64), rng.integers(0, 2**32, size=n, dtype=np.uint32),
            rng.integers(0, 256, size=3 * n + 5, dtype=np.uint8))


def _worker(name, world, rank, n, slot, mode, q):
    d = _dll()
    g = ctypes.c_void_p()
    rc = d.pz_debug_shm_open(name.encode(), world, rank, 20000 if mode != "timeout" else 1500, slot, ctypes.byref(g))
    if rc:
        q.put((rank, "open", rc, d.pz_debug_shm_error().decode()))
        return
    s, m, b = _inputs(rank, n)
    out = {}
    try:
        if mode == "ok":
            x = s.copy()
            assert d.pz_debug_shm_sum_u64(g, _p(x), n) == 0, d.pz_debug_shm_error()
            y = m.copy()
            assert d.pz_debug_shm_min_u32(g, _p(y), n) == 0, d.pz_debug_shm_error()
            xs, ym = s.copy(), m[: n // 2 + 1].copy()
            assert d.pz_debug_shm_sum_min(g, _p(xs), n, _p(ym), len(ym)) == 0, d.pz_debug_shm_error()
            recv = np.zeros(world * b.size, dtype=np.uint8)
            assert d.pz_debug_shm_allgather(g, _p(b), _p(recv), b.size) == 0, d.pz_debug_shm_error()
            out = dict(sum=x, min=y, sm_sum=xs, sm_min=ym, gather=recv)
            q.put((rank, "ok", 0, out))
        elif mode == "diverge":
            # rank 1 skips the sum and goes straight to the all-gather (what a host-side decision
            # that differs between ranks would do): both must fail, naming the two calls
            if rank == 1:
                recv = np.zeros(world * b.size, dtype=np.uint8)
                rc = d.pz_debug_shm_allgather(g, _p(b), _p(recv), b.size)
            else:
                rc = d.pz_debug_shm_sum_u64(g, _p(s.copy()), n)
            q.put((rank, "diverge", rc, d.pz_debug_shm_error().decode()))
        elif mode == "timeout":
            # rank 1 never calls the collective
            rc = d.pz_debug_shm_sum_u64(g, _p(s.copy()), n) if rank == 0 else 0
            q.put((rank, "timeout", rc, d.pz_debug_shm_error().decode()))
    finally:
        if mode == "timeout" and rank == 1:
            import time
            time.sleep(3.0)  # hold the group open past rank 0's timeout
        d.pz_debug_shm_close(g)


def _run(world, n, slot, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = "/pz_test_%d_%s" % (os.getpid(), uuid.uuid4().hex[:8])
    ps = [ctx.Process(target=_worker, args=(name, world, r, n, slot, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r = q.get(timeout=60)
            res[r[0]] = r[1:]
        for p in ps:
            p.join(30)
            assert p.exitcode == 0
        assert not os.path.exists("/dev/shm" + name), "segment left behind"
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
                p.join()
        if os.path.exists("/dev/shm" + name):  # (a killed rank 0 leaves its segment behind)
            os.unlink("/dev/shm" + name)
    return res


@pytest.mark.parametrize("world,n,slot", [(2, 1000, 1 << 20), (3, 5000, 4096), (5, 1, 4096)])
def test_shm_collectives_exact(world, n, slot):
    """Sum (mod 2^64), min, the grouped sum+min and all-gather equal numpy's on every rank;
    slot 4096 forces every collective through several chunk rounds."""
    res = _run(world, n, slot, "ok")
    ins = [_inputs(r, n) for r in range(world)]
    want_sum = np.zeros(n, dtype=np.uint64)
    for s, _, _ in ins:
        want_sum += s  # numpy uint64 wraps like Go's uint64
    want_min = np.min(np.stack([m for _, m, _ in ins]), axis=0)
    want_gather = np.concatenate([b for _, _, b in ins])
    for r in range(world):
        kind, rc, out = res[r]
        assert (kind, rc) == ("ok", 0)
        assert np.array_equal(out["sum"], want_sum)
        assert np.array_equal(out["min"], want_min)
        assert np.array_equal(out["sm_sum"], want_sum)
        assert np.array_equal(out["sm_min"], want_min[: n // 2 + 1])
        assert np.array_equal(out["gather"], want_gather)


def test_shm_divergent_collectives_fail_loudly():
    """Ranks that issue different collectives fail with PZ_EINVAL naming both calls (RCCL would
    hang), instead of exchanging mismatched buffers."""
    res = _run(2, 64, 4096, "diverge")
    for r in (0, 1):
        kind, rc, msg = res[r]
        assert rc == _lib.PZ_EINVAL, (r, rc, msg)
        assert "diverged" in msg and "all-gather" in msg and "u64 sum" in msg, msg


def test_shm_missing_rank_times_out():
    res = _run(2, 64, 4096, "timeout")
    kind, rc, msg = res[0]
    assert rc == _lib.PZ_EDEVICE and "waited" in msg and "rank 1" in msg, msg
