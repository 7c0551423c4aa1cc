"""Shared checker: the GPU chain engine's per-block / per-attestation results and roots
against the C restatement of the block pipeline (oracle/c/replay_ref.c) on the same
serialized chain."""
import numpy as np

from oracle import cport


def port_replay(data, offs, nval, natt, bitmap_dedup=True):
    r = cport.Replay(nval, bitmap_dedup=bitmap_dedup)
    try:
        return r.process(data, offs, natt), r.roots()
    finally:
        r.close()


def mismatches(br, ar, gpu_roots, out, port_roots):
    """List of differences (empty when bit-exact).  Attestation statuses compare by class:
    processed / not processed / rejected (the engine names the failed check, the port does
    not); the digests compare for every processed attestation."""
    bad = []
    n = len(br)
    if not np.array_equal(br["hash"].reshape(n, 32), out["hash"]):
        bad.append("block hashes")
    if not np.array_equal(br["status"], out["status"]):
        bad.append("block statuses")
    if not np.array_equal(br["transition"].astype(bool), out["transition"].astype(bool)):
        bad.append("transitions")
    st = np.minimum(ar["status"], 2)
    if not np.array_equal(st, out["att_status"][:len(ar)]):
        bad.append("attestation statuses")
    ok = ar["status"] == 0
    for k_gpu, k_port, w in (("key", "key", 32), ("hash", "att_hash", 32), ("msg", "msg", 64)):
        g = ar[k_gpu].reshape(len(ar), w)[ok]
        if not np.array_equal(g, out[k_port][:len(ar)][ok]):
            bad.append("attestation " + k_gpu)
    if not np.array_equal(ar["msg_len"][ok], out["msg_len"][:len(ar)][ok]):
        bad.append("message lengths")
    for k in ("chain_active", "chain_crystallized", "cand_active", "cand_crystallized", "vote_totals"):
        if gpu_roots.get(k) != port_roots.get(k):
            bad.append(k)
    return bad
