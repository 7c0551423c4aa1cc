"""The chain engine's block parser on host threads (pz_debug_parse, CPU-only: no device call):
the same records and the same first malformed block for every thread count.  The walk relies
on it (pz_chain_process_blocks parses a call's blocks on PZ_PARSE_THREADS threads, DESIGN.md
§7); the GPU replay tests check the results end to end."""
import ctypes

import numpy as np
import pytest

from prysm_amd import _lib, synth
from prysm_amd.blockchain import serialize_blocks


def _parse(data, offs, threads):
    from ab_lib import ab_dll
    dll = ab_dll()
    fn = dll.pz_debug_parse
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    sec, cs = ctypes.c_double(), ctypes.c_uint64()
    rc = fn(data.ctypes.data, offs.ctypes.data, len(offs) - 1, threads, 1, ctypes.byref(sec), ctypes.byref(cs))
    dll.pz_last_error.restype = ctypes.c_void_p
    msg = dll.pz_last_error()
    return rc, cs.value, ctypes.cast(msg, ctypes.c_char_p).value.decode() if rc else ""


@pytest.fixture(scope="module")
def chain():
    blocks = synth.chain_blocks(1024, 260, seed=11)
    data, offs = serialize_blocks(blocks)
    return np.ascontiguousarray(data, np.uint8), np.ascontiguousarray(offs, np.uint64)


def test_threads_parse_identically(chain):
    data, offs = chain
    ref = _parse(data, offs, 1)
    assert ref[0] == 0
    for t in (2, 3, 8, 64):
        assert _parse(data, offs, t) == ref, t


@pytest.mark.parametrize("bad", [0, 7, 131, 259])
def test_first_malformed_block_named_for_every_thread_count(chain, bad):
    data, offs = chain
    d = data.copy()
    d[int(offs[bad])] = 0  # field number 0: not a canonical BeaconBlock
    for t in (1, 2, 5, 8):
        rc, _, msg = _parse(d, offs, t)
        assert rc == _lib.PZ_EINVAL
        assert "block %d " % bad in msg, (t, msg)


def test_empty_and_tiny_calls(chain):
    data, offs = chain
    for n in (1, 2, 3):
        o = np.ascontiguousarray(offs[: n + 1])
        assert _parse(data, o, 1) == _parse(data, o, 8)


def test_parse_in_a_forked_child(chain):
    """The parse's worker pool is per process: a child forked after the parent parsed starts
    its own workers instead of waiting on the parent's (chain.hip work_pool)."""
    import os
    data, offs = chain
    ref = _parse(data, offs, 8)
    pid = os.fork()
    if pid == 0:
        os._exit(0 if _parse(data, offs, 8) == ref else 3)
    _, st = os.waitpid(pid, 0)
    assert os.WIFEXITED(st) and os.WEXITSTATUS(st) == 0
    assert _parse(data, offs, 8) == ref
