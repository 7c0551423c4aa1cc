"""ORACLE (test infrastructure only) — ctypes view of the C restatement in oracle/c."""
import ctypes
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "liboracle_c.so")
_dll = None


def dll():
    global _dll
    if _dll is None:
        _dll = ctypes.CDLL(_PATH)
        vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        _dll.oracle_blake2b512_fixed.argtypes = [vp, u64, u64, u64, vp, u32]
        _dll.oracle_blake2b512_csr.argtypes = [vp, vp, u64, vp, u32]
    return _dll


def hash_fixed(records, length, out_bytes=32):
    """records: (n, stride) uint8 -> (n, out_bytes) uint8."""
    records = np.ascontiguousarray(records, dtype=np.uint8)
    n, stride = records.shape
    out = np.empty((n, out_bytes), dtype=np.uint8)
    dll().oracle_blake2b512_fixed(records.ctypes.data, stride, length, n, out.ctypes.data, out_bytes)
    return out


def hash_csr(data, offsets, out_bytes=32):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    out = np.empty((n, out_bytes), dtype=np.uint8)
    dll().oracle_blake2b512_csr(data.ctypes.data if data.size else None, offsets.ctypes.data, n,
                                out.ctypes.data, out_bytes)
    return out
