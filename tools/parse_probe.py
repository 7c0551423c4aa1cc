"""Host parse of the configs[4] chain (pz_debug_parse, best of 20) by thread count, with the
arena on the heap and in pooled pinned memory (PZ_DEBUG_PARSE_PIN, set per run by this script
through a child process).

    python tools/parse_probe.py [heap|pin]"""
import ctypes
import os
import subprocess
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode):
    from prysm_amd import _lib, synth
    from prysm_amd.blockchain import serialize_blocks
    blocks = synth.chain_blocks(65536, 10000, seed=6)
    data, offs = serialize_blocks(blocks)
    data = np.ascontiguousarray(data, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    fn = _lib.lib.dll.pz_debug_parse
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    for t in (1, 2, 4, 8, 16):
        sec, cs = ctypes.c_double(), ctypes.c_uint64()
        rc = fn(data.ctypes.data, offs.ctypes.data, len(offs) - 1, t, 20, ctypes.byref(sec), ctypes.byref(cs))
        print("%-4s threads %2d: %.3f ms (best of 20), rc %d, %.1f MB" % (mode, t, sec.value * 1e3, rc, offs[-1] / 1e6),
              flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for m in ("heap", "pin"):
            env = dict(os.environ, PZ_DEBUG_PARSE_PIN="1" if m == "pin" else "0")
            rc = subprocess.call([sys.executable, os.path.abspath(__file__), m], env=env)
            if rc:
                sys.exit(rc)
