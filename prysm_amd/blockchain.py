"""Block pipeline of the reference's beacon chain (blockchain/service.go:229-363 over
blockchain/core.go) — Python face of the native engine in ``prysm_amd/csrc/chain.hip``.

``BeaconChain.process_serialized(data, offsets)`` feeds canonical BeaconBlock encodings (as
the sync service receives them, sync/service.go:147-164) through ``pz_chain_process_blocks``:
a C++ walk with the control flow of ``ChainService.blockProcessing`` (parent check,
processAttestation, calculateBlockVoteCache, updateHead, saveBlock, IsCycleTransition ->
stateRecalc, computeNewActiveState), keeping the reference's object-sharing and ordering
semantics (restated by the oracle in oracle/replay.py).  The device does the
heavy work, batched per call:

* H  block digests, attestation ``Hash``/``Key`` (one CSR BLAKE2b launch before the walk),
     the 64-byte processAttestation message digests (``core.go:277-290``, one launch after
     it) and the Active/Crystallized state roots;
* T  the block vote cache (``core.go:300-345``) lives in HBM — a dedup bitmap and a u64
     total per signed parent hash — fed by the vote-tally kernel once per stretch of blocks
     between balance changes;
* R  stateRecalc's processCrosslinks + CalculateRewards + next-cycle balance run as one epoch
     instance on the HBM-resident validator arrays.

Where the reference panics, ``ChainPanic`` is raised and the chain object is spent.
"""
import ctypes

import numpy as np

from prysm_amd import _lib, wire
from prysm_amd._lib import PzError, lib

BLOCK_RESULT = np.dtype([("hash", "u1", 32), ("status", "<i4"), ("transition", "<i4"),
                         ("first_att", "<u4"), ("natt", "<u4")])
ATT_RESULT = np.dtype([("status", "<i4"), ("msg_len", "<u4"), ("key", "u1", 32), ("hash", "u1", 32),
                       ("msg", "u1", 64)])
BLOCK_STATUS = {0: "processed", 1: "no_parent", 2: "attestations_rejected", 3: "saved_not_candidate"}
ATT_PROCESSED, ATT_NOT_PROCESSED = 0, 1
ATT_ERRORS = {2: "slot too high", 3: "slot too low", 4: "justified slot mismatch", 5: "no committee",
              6: "bitfield length", 7: "non-zero trailing bits"}


def check_attestations(atts, block_slots, last_justified_slot, last_state_recalc, n_recent,
                       shard_and_committees):
    """processAttestation's checks (blockchain/core.go:240-297, :348-394) for a batch of
    attestations on the GPU (``pz_check_attestations``, one lane each).

    ``atts``: AttestationRecord-like objects; ``block_slots[i]``: the slot of the block that
    carries ``atts[i]``; the chain state: ``last_justified_slot``, ``last_state_recalc``,
    ``n_recent`` = len(RecentBlockHashes) and ``shard_and_committees`` = ShardAndCommitteesForSlots
    as a list (one per slot) of lists of ``(shard_id, committee)`` pairs.  Returns
    ``(status, committee_index, parents_start)``: status PZ_ATT_PROCESSED, the first failed
    check (PZ_ATT_*), or PZ_ERANGE / PZ_EINDEX where Go panics; committee_index counts the
    table's (shard, committee) entries in order (-1 if not reached)."""
    n = len(atts)
    u64 = np.uint64
    cols = {k: np.ascontiguousarray([getattr(a, k) for a in atts], dtype=u64)
            for k in ("slot", "justified_slot", "shard_id")}
    n_obl = np.ascontiguousarray([len(a.oblique_parent_hashes) for a in atts], dtype=u64)
    bslot = np.ascontiguousarray(block_slots, dtype=u64)
    bf = [bytes(a.attester_bitfield) for a in atts]
    boffs = np.zeros(n + 1, dtype=u64)
    boffs[1:] = np.cumsum([len(x) for x in bf], dtype=u64)
    bits = np.frombuffer(b"".join(bf) + b"\0", dtype=np.uint8)
    arr_offs = np.zeros(len(shard_and_committees) + 1, dtype=u64)
    arr_offs[1:] = np.cumsum([len(arr) for arr in shard_and_committees], dtype=u64)
    entries = [e for arr in shard_and_committees for e in arr]
    arr_shard = np.ascontiguousarray([e[0] for e in entries] or [0], dtype=u64)
    arr_comm = np.arange(max(len(entries), 1), dtype=np.uint32)
    coffs = np.zeros(len(entries) + 1, dtype=u64)
    coffs[1:] = np.cumsum([len(e[1]) for e in entries], dtype=u64)
    status = np.zeros(max(n, 1), dtype=np.int32)
    comm = np.zeros(max(n, 1), dtype=np.uint32)
    pstart = np.zeros(max(n, 1), dtype=u64)
    b = _lib.AttCheckBatch(
        n, _lib.ptr(cols["slot"]), _lib.ptr(cols["justified_slot"]), _lib.ptr(cols["shard_id"]), _lib.ptr(n_obl),
        _lib.ptr(bits), _lib.ptr(boffs), _lib.ptr(bslot), last_justified_slot, last_state_recalc, n_recent,
        len(shard_and_committees), _lib.ptr(arr_offs), _lib.ptr(arr_shard), _lib.ptr(arr_comm), _lib.ptr(coffs),
        _lib.ptr(status), _lib.ptr(comm), _lib.ptr(pstart))
    lib.call("pz_check_attestations", ctypes.byref(b))
    ci = comm[:n].astype(np.int64)
    ci[comm[:n] == 0xFFFFFFFF] = -1
    return status[:n], ci, pstart[:n]


class ChainPanic(RuntimeError):
    """The reference would panic here (index out of range / nil map / nil state)."""


def serialize_blocks(blocks):
    """pb.BeaconBlock list -> (uint8 data, uint64 offsets[n+1]) of canonical encodings."""
    enc = [wire.beacon_block(b) for b in blocks]
    offs = np.zeros(len(enc) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(e) for e in enc], dtype=np.uint64)
    return np.frombuffer(b"".join(enc) + bytes(16), dtype=np.uint8), offs


class BeaconChain:
    """A chain from the genesis states of ``nval`` validators on one GPU."""

    def __init__(self, nval, device=None, comm=None, msg_batch=0, tally_forms=0):
        """``comm`` (a ``prysm_amd.native.Comm``): one chain over the communicator's ranks,
        each holding a validator range of the balances, the vote cache and the epoch
        (pz_chain_new_comm).  ``msg_batch`` / ``tally_forms``:
        pz_chain_options (message batches sent during the walk; the tally's general forms
        forced, _lib.TALLY_*)."""
        idx = 0
        if device is not None:
            import torch
            d = torch.device(device)
            idx = d.index or 0
        self._h = ctypes.c_void_p()
        self.comm = comm  # kept alive as long as the chain
        if comm is not None:
            lib.call("pz_chain_new_comm", nval, comm.h, ctypes.byref(self._h))
        else:
            lib.call("pz_chain_new", nval, idx, ctypes.byref(self._h))
        self.nval = nval
        if msg_batch or tally_forms:
            opts = _lib.ChainOptions(int(msg_batch), int(tally_forms))
            lib.call("pz_chain_set_options", self._h, ctypes.byref(opts))

    @classmethod
    def from_state(cls, crystallized_bytes, saved_hashes=(), device=None):
        """NewBeaconChain with a stored CrystallizedState (blockchain/core.go:86-95): resume
        from its encoding with the genesis ActiveState; ``saved_hashes`` are the block hashes
        the database holds (hasBlock)."""
        idx = 0
        if device is not None:
            import torch
            idx = torch.device(device).index or 0
        self = cls.__new__(cls)
        self._h = ctypes.c_void_p()
        cs = np.frombuffer(bytes(crystallized_bytes), dtype=np.uint8)
        hs = np.frombuffer(b"".join(bytes(h) for h in saved_hashes), dtype=np.uint8)
        lib.call("pz_chain_new_from_state", _lib.ptr(cs), cs.size, _lib.ptr(hs), len(saved_hashes), idx,
                 ctypes.byref(self._h))
        self.nval = None
        return self

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.dll.pz_chain_free(h)
            self._h = None

    def process_serialized(self, data, offsets):
        """Run serialized blocks; returns (block results, attestation results) as numpy
        structured arrays (``BLOCK_RESULT`` / ``ATT_RESULT``)."""
        n = len(offsets) - 1
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        br = np.zeros(max(n, 1), dtype=BLOCK_RESULT)
        cnt = ctypes.c_uint64(0)
        lib.call("pz_count_attestations", _lib.ptr(data), _lib.ptr(offsets), n, ctypes.byref(cnt))
        natt_cap = max(1, cnt.value)
        ar = np.zeros(natt_cap, dtype=ATT_RESULT)
        try:
            lib.call("pz_chain_process_blocks", self._h, _lib.ptr(data), _lib.ptr(offsets), n,
                     br.ctypes.data, ar.ctypes.data, natt_cap)
        except PzError as e:
            if e.code == _lib.PZ_EINDEX:
                raise ChainPanic(str(e)) from None
            raise
        natt = int(br["natt"][:n].sum()) if n else 0
        return br[:n], ar[:natt]

    def process_blocks(self, blocks):
        """pb.BeaconBlock list -> per-block records (the oracle/replay.py record format)."""
        data, offs = serialize_blocks(blocks)
        br, ar = self.process_serialized(data, offs)
        recs = []
        for b, r in zip(blocks, br):
            rec = {"hash": r["hash"].tobytes(), "slot": b.slot_number, "atts": [],
                   "status": BLOCK_STATUS[int(r["status"])], "transition": bool(r["transition"])}
            for x in ar[int(r["first_att"]):int(r["first_att"]) + int(r["natt"])]:
                st = int(x["status"])
                if st == ATT_NOT_PROCESSED:
                    continue
                if st == ATT_PROCESSED:
                    rec["atts"].append({"key": x["key"].tobytes(), "hash": x["hash"].tobytes(),
                                        "msg": x["msg"].tobytes(), "msg_len": int(x["msg_len"])})
                else:
                    rec["atts"].append({"error": ATT_ERRORS.get(st, st)})
            recs.append(rec)
        return recs

    STATES = ("chain_active", "chain_crystallized", "cand_active", "cand_crystallized")

    def state_bytes(self, which):
        """The persisted proto3 encoding of a state (blockchain/core.go:161-177): ``which`` in
        ``STATES``; None for a candidate state when there is no candidate."""
        w = self.STATES.index(which)
        n = ctypes.c_uint64(0)
        try:
            lib.call("pz_chain_state_bytes", self._h, w, None, 0, ctypes.byref(n))
        except PzError as e:
            if w >= 2 and e.code == _lib.PZ_EINVAL:
                return None
            raise
        buf = np.zeros(max(n.value, 1), dtype=np.uint8)
        lib.call("pz_chain_state_bytes", self._h, w, buf.ctypes.data, n.value, ctypes.byref(n))
        return buf[:n.value].tobytes()

    def roots(self):
        """State roots (types/state.go:138-149, 237-248) of the chain's and the candidate's
        states, and the vote cache totals {hash: VoteTotalDeposit}."""
        out = (ctypes.c_uint8 * 128)()
        cand = ctypes.c_int(0)
        lib.call("pz_chain_roots", self._h, out, ctypes.byref(cand))
        raw = bytes(out)
        r = {"chain_active": raw[:32], "chain_crystallized": raw[32:64]}
        if cand.value:
            r["cand_active"], r["cand_crystallized"] = raw[64:96], raw[96:128]
        cnt = ctypes.c_uint64(0)
        lib.call("pz_chain_vote_totals", self._h, None, None, 0, ctypes.byref(cnt))
        n = cnt.value
        hashes = np.zeros(max(n, 1) * 32, dtype=np.uint8)
        totals = np.zeros(max(n, 1), dtype=np.uint64)
        if n:
            lib.call("pz_chain_vote_totals", self._h, hashes.ctypes.data, totals.ctypes.data, n, ctypes.byref(cnt))
        r["vote_totals"] = {hashes[32 * i:32 * i + 32].tobytes(): int(totals[i]) for i in range(n)}
        return r
