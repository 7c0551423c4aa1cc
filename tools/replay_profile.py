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
    prof = cProfile.Profile() if "--cprofile" in sys.argv else None
    t = time.perf_counter()
    data, offs = serialize_blocks(blocks)
    print("serialize %.3f s (%.1f MB)" % (time.perf_counter() - t, offs[-1] / 1e6), flush=True)
    import ctypes
    names = ["parse", "digests1", "att_checks+msg", "vote_queue", "vote_flush", "state_recalc", "msg_digests",
             "walk(all)", "process(all)", "count_atts", "flush_arena_wait", "msg_send",
             "msg_hash_log", "msg_wait", "totals_wait", "poll_fallbacks(count)", "vote_id_rows(count)"]
    # AB=VAR: alternate the environment variable VAR over the values AB_VALUES (default "0,1")
    # across the replays (an A/B of a per-call knob such as PZ_VOTE_PATH in one process); REPS
    # replays per value
    ab = os.environ.get("AB")
    vals = os.environ.get("AB_VALUES", "0,1").split(",")
    reps = int(os.environ.get("REPS", "3"))
    res = {}
    for r in range(reps * (len(vals) if ab else 1)):
        val = vals[r % len(vals)] if ab else None
        if ab:
            os.environ[ab] = val
        ch = BeaconChain(nval)
        torch.cuda.synchronize()
        t = time.perf_counter()
        if prof:
            prof.enable()
        br, ar = ch.process_serialized(data, offs)
        torch.cuda.synchronize()
        if prof:
            prof.disable()
        dt = time.perf_counter() - t
        res.setdefault(val, []).append(nblocks / dt)
        print("%sprocess_serialized %.3f s -> %.1f blocks/s (%d processed, %d attestations)"
              % ("[%s=%s] " % (ab, val) if ab else "", dt, nblocks / dt, int((br["status"] == 0).sum()), len(ar)),
              flush=True)
        pv = (ctypes.c_double * len(names))()
        fn = _lib.lib.dll.pz_chain_phase_times
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        k = fn(ch._h, pv, len(names))
        print("  phases (s): " + ", ".join("%s %.4f" % (names[i], pv[i]) for i in range(min(k, len(names)))),
              flush=True)
    for val, xs in res.items():
        print("median%s: %.1f blocks/s over %d replays" % ("" if val is None else " [%s=%s]" % (ab, val),
                                                          float(sorted(xs)[len(xs) // 2]), len(xs)), flush=True)
    t = time.perf_counter()
    ch.roots()
    print("roots %.3f s" % (time.perf_counter() - t), flush=True)
    if prof:
        pstats.Stats(prof).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
