"""Profile the GPU block pipeline on a synthetic chain (BASELINE configs[4] shape):
python tools/replay_profile.py NVAL NBLOCKS [--cprofile]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from prysm_amd import _lib, synth  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):  # A/B against another build of the library
    _lib.library_path = os.environ["PZ_PROBE_LIB"]
from prysm_amd.blockchain import BeaconChain, serialize_blocks  # noqa: E402


def main():
    nval, nblocks = int(sys.argv[1]), int(sys.argv[2])
    t = time.perf_counter()
    blocks = synth.chain_blocks(nval, nblocks, seed=6)
    print("generate %.3f s" % (time.perf_counter() - t), flush=True)
    t = time.perf_counter()
    ch = BeaconChain(nval)
    torch.cuda.synchronize()
    print("genesis %.3f s" % (time.perf_counter() - t), flush=True)
    ch.process_serialized(*serialize_blocks(blocks))  # warm-up (kernels loaded, pinned pool filled)
    ch = BeaconChain(nval)
    prof = cProfile.Profile() if "--cprofile" in sys.argv else None
    t = time.perf_counter()
    data, offs = serialize_blocks(blocks)
    print("serialize %.3f s (%.1f MB)" % (time.perf_counter() - t, offs[-1] / 1e6), flush=True)
    t = time.perf_counter()
    if prof:
        prof.enable()
    br, ar = ch.process_serialized(data, offs)
    torch.cuda.synchronize()
    if prof:
        prof.disable()
    dt = time.perf_counter() - t
    print("process_serialized %.3f s -> %.1f blocks/s (%d processed, %d attestations)"
          % (dt, nblocks / dt, int((br["status"] == 0).sum()), len(ar)), flush=True)
    import ctypes
    from prysm_amd import _lib
    pv = (ctypes.c_double * 16)()
    fn = _lib.lib.dll.pz_debug_chain_profile
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    k = fn(ch._h, pv, 16)
    names = ["parse", "digests1", "att_checks+msg", "vote_queue", "vote_flush", "state_recalc", "msg_digests",
             "walk(all)", "process(all)", "count_atts", "flush_arena_wait", "msg_send",
             "msg_hash_log", "msg_wait"]
    print("phases (s): " + ", ".join("%s %.4f" % (names[i], pv[i]) for i in range(k)), flush=True)
    t = time.perf_counter()
    ch.roots()
    print("roots %.3f s" % (time.perf_counter() - t), flush=True)
    if prof:
        pstats.Stats(prof).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
