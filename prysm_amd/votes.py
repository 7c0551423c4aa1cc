"""Host-side mirror of the block vote cache (types/state.go:27-31 ``VoteCache`` and
blockchain/core.go:300-345 ``calculateBlockVoteCache``) over the GPU tally kernel.

The Go map ``map[[32]byte]*VoteCache`` becomes a host dict ``hash -> slot`` plus, per slot,
an nval-bit voter bitmap and the ``VoteTotalDeposit`` u64.  ``VoterIndices`` is a set here
(the bitmap; ascending order on read-out) — the reference's insertion order is never
serialized or hashed.
"""
import numpy as np

from prysm_amd import _lib
from prysm_amd._lib import lib, ptr


class VoteCache:
    def __init__(self, nval):
        self.nval = nval
        self.words = (nval + 31) // 32
        self.slot_of = {}
        self.bitmaps = np.zeros((0, self.words), dtype=np.uint32)
        self.totals = np.zeros(0, dtype=np.uint64)

    def slot(self, h):
        """Slot of hash ``h``, created empty if absent (core.go:321-324)."""
        s = self.slot_of.get(h)
        if s is None:
            s = len(self.slot_of)
            self.slot_of[h] = s
            if s >= self.totals.shape[0]:
                cap = max(16, 2 * s)
                bm = np.zeros((cap, self.words), dtype=np.uint32)
                bm[:self.bitmaps.shape[0]] = self.bitmaps
                tt = np.zeros(cap, dtype=np.uint64)
                tt[:self.totals.shape[0]] = self.totals
                self.bitmaps, self.totals = bm, tt
        return s

    def __contains__(self, h):
        return h in self.slot_of

    def total(self, h):
        s = self.slot_of.get(h)
        return 0 if s is None else int(self.totals[s])

    def voters(self, h):
        s = self.slot_of[h]
        bits = np.unpackbits(self.bitmaps[s].view(np.uint8), bitorder="little")[:self.nval]
        return np.nonzero(bits)[0].astype(np.uint32)

    def tally(self, committee, coffs, att_comm, bits, boffs, items, balance, comm=None):
        """Apply work items [(attestation index, slot)] in one GPU launch; with ``comm`` (a
        ``prysm_amd.native.Comm``) sharded by validator range over its ranks, the per-slot
        totals combined by one all-reduce (pz_comm_vote_tally)."""
        if not items:
            return
        ia = np.ascontiguousarray([a for a, _ in items], dtype=np.uint32)
        isl = np.ascontiguousarray([s for _, s in items], dtype=np.uint32)
        bm = np.ascontiguousarray(self.bitmaps)
        tt = np.ascontiguousarray(self.totals)
        args = (ptr(committee), ptr(coffs), len(coffs) - 1, ptr(att_comm), ptr(bits), ptr(boffs),
                len(att_comm), ptr(ia), ptr(isl), len(items), ptr(np.ascontiguousarray(balance, dtype=np.uint64)),
                self.nval, ptr(bm), bm.shape[0], self.words, ptr(tt))
        if comm is None:
            lib.call("pz_vote_tally", *args)
        else:
            lib.call("pz_comm_vote_tally", comm.h, *args)
        self.bitmaps, self.totals = bm, tt


__all__ = ["VoteCache", "_lib"]
