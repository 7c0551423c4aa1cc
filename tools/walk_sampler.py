"""Where the chain walk's host time goes: wall-clock samples (interrupted PC + 15 callers) of
the thread that runs pz_chain_process_blocks (pz_debug_sample_start/stop,
prysm_amd/csrc/sampler.cpp), symbolized with llvm-symbolizer (inline frames included)
against the library's -g1 build.

    make -C prysm_amd/csrc prof
    PZ_PROBE_LIB=build/prof/libprysm_hip.so python tools/walk_sampler.py [NBLOCKS] [REPS] [INTERVAL_US]

Each sample is charged to the innermost line of the chain engine's own sources on its stack
(time in libc / the HIP runtime below it included), and its leaf is reported per object and
function."""
import collections
import ctypes
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from prysm_amd import _lib, synth  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):
    _lib.library_path = os.environ["PZ_PROBE_LIB"]
from prysm_amd.blockchain import BeaconChain, serialize_blocks  # noqa: E402

SYMBOLIZER = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"
OURS = ("chain.hip", "votes.hip", "runtime.hip", "epoch.hip", "blake2b.hip", "serial_hash.cpp", "wire.hip")


def symbolize(path, offsets):
    """offset -> [(function, file:line)], innermost first."""
    uniq = sorted(set(offsets))
    if not uniq:
        return {}
    inp = "\n".join("0x%x" % o for o in uniq) + "\n"
    out = subprocess.run([SYMBOLIZER, "--obj=" + path, "-i", "-C", "-f"], input=inp, capture_output=True,
                         text=True).stdout
    res = {}
    for o, blk in zip(uniq, out.split("\n\n")):
        ln = [x for x in blk.splitlines() if x.strip()]
        fr = []
        for k in range(0, len(ln) - 1, 2):
            loc = ln[k + 1]
            parts = loc.rsplit(":", 2)
            fr.append((ln[k].split("(")[0][:90], "%s:%s" % (os.path.basename(parts[0]), parts[1] if len(parts) > 1 else "?")))
        res[o] = fr or [("?", "?")]
    return res


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    us = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    nval = 65536
    blocks = synth.chain_blocks(nval, nb, seed=6)
    data, offs = serialize_blocks(blocks)
    BeaconChain(nval).process_serialized(*serialize_blocks(blocks[:130]))  # warm-up
    dll = _lib.lib.dll
    dll.pz_debug_sample_start.argtypes = [ctypes.c_int, ctypes.c_uint64]
    dll.pz_debug_sample_stop.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p,
                                         ctypes.c_uint64]
    dll.pz_debug_sample_stop.restype = ctypes.c_int64
    D = dll.pz_debug_sample_depth()
    cap = 1 << 18
    offs_o = (ctypes.c_uint64 * (cap * D))()
    obj_o = (ctypes.c_uint32 * (cap * D))()
    names = ctypes.create_string_buffer(1 << 16)
    walls = []
    chains = [BeaconChain(nval) for _ in range(reps)]
    torch.cuda.synchronize()
    base = []  # unsampled walls after, for the sampler's overhead
    assert dll.pz_debug_sample_start(us, cap) == 0
    for ch in chains:
        t = time.perf_counter()
        ch.process_serialized(data, offs)
        walls.append(time.perf_counter() - t)
    n = dll.pz_debug_sample_stop(offs_o, obj_o, cap, names, len(names))
    for _ in range(2):
        ch = BeaconChain(nval)
        torch.cuda.synchronize()
        t = time.perf_counter()
        ch.process_serialized(data, offs)
        base.append(time.perf_counter() - t)
    objs = names.value.decode().splitlines()
    print("replays: sampled %s ms, unsampled %s ms (%d blocks each); %d samples at %d us" % (
        ", ".join("%.1f" % (w * 1e3) for w in walls), ", ".join("%.1f" % (w * 1e3) for w in base), nb, n, us))
    # symbolize every (object, offset) seen; callers' return addresses - 1
    want = collections.defaultdict(set)
    for i in range(n * D):
        if obj_o[i] != 0xFFFFFFFF:
            want[obj_o[i]].add(offs_o[i] - (1 if i % D else 0))
    sym = {k: symbolize(objs[k], v) for k, v in want.items()}
    leaf_obj, leaf_fn, line_c, fn_c, pair_c, chain_c = (collections.Counter() for _ in range(6))
    for i in range(n):
        fr = []
        for d in range(D):
            k = obj_o[i * D + d]
            if k == 0xFFFFFFFF:
                break
            o = offs_o[i * D + d] - (1 if d else 0)
            fr.append((os.path.basename(objs[k]), sym[k].get(o, [("?", "?")])))
        if not fr:
            continue
        leaf_obj[fr[0][0]] += 1
        leaf_fn["%s: %s" % (fr[0][0], fr[0][1][0][0])] += 1
        ours = None
        for ob, chain in fr:
            for fn, loc in chain:
                if loc.split(":")[0] in OURS:
                    ours = (fn, loc)
                    break
            if ours:
                break
        own = [loc for ob, ch in fr for fn, loc in ch if loc.split(":")[0] in OURS]
        chain_c[" <- ".join(own[:4])] += 1
        if ours is None:
            ours = ("(no engine frame)", "")
        line_c["%s  %s" % (ours[1], ours[0])] += 1
        fn_c[ours[0]] += 1
        if fr[0][0] != os.path.basename(_lib.library_path):
            pair_c["%s <- %s" % (fr[0][1][0][0][:40], ours[1])] += 1
    for title, cnt, k in (("leaf object", leaf_obj, 10), ("leaf function", leaf_fn, 25),
                          ("engine function (innermost own-source frame)", fn_c, 25),
                          ("engine line", line_c, 60), ("outside the library: leaf <- engine line", pair_c, 30),
                          ("engine call chains (innermost four own-source frames)", chain_c, 40)):
        print("\n%s, %% of samples:" % title)
        for f, c in cnt.most_common(k):
            print("  %6.2f%%  %s" % (100.0 * c / n, f[:160]))


if __name__ == "__main__":
    main()
