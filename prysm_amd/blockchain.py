"""Block pipeline of the reference's beacon chain (blockchain/service.go:229-363 over
blockchain/core.go) with every data-parallel step on the GPU.

``BeaconChain.process_blocks(blocks)`` feeds a batch of blocks, in order, through the same
control flow as ``ChainService.blockProcessing`` (parent check, processAttestation,
calculateBlockVoteCache, updateHead, saveBlock, IsCycleTransition -> stateRecalc,
computeNewActiveState), keeping the reference's object-sharing and ordering semantics
(documented in DESIGN.md §7 and restated by the oracle in oracle/replay.py).  The host walks
the blocks with scalar checks only; the heavy work is batched onto the device:

* H  block digests (one CSR BLAKE2b launch for the whole batch, before the walk: blocks are
     immutable inputs), attestation ``Hash``/``Key`` digests (one launch), the 64-byte
     processAttestation message digests (``core.go:277-290``, one launch after the walk) and
     the Active/Crystallized state roots;
* T  the block vote cache (``core.go:300-345``) is device-resident: a dedup bitmap and a
     u64 total per signed parent hash, fed by ``pz_dev_vote_tally`` in one launch per
     stretch of blocks between balance changes (flushed before each stateRecalc, whose
     justification loop reads 64 totals back);
* R  stateRecalc's processCrosslinks + CalculateRewards + next-cycle balance run as one
     epoch instance (``pz_dev_epoch_count`` / ``pz_dev_epoch_finish``) on the resident
     validator arrays; the host applies the crosslink winners and the scalars.

Go panics surface as ``ChainPanic`` (the reference process would crash at that point).
"""
import ctypes

import numpy as np

from prysm_amd import _lib, pb, wire
from prysm_amd._lib import EpochBatch, PzError, lib
from prysm_amd.params import CYCLE_LENGTH, SHARD_COUNT
from prysm_amd.types import bytes_to_hash, copy32, new_genesis_states, new_genesis_block

M64 = (1 << 64) - 1


class ChainPanic(RuntimeError):
    """The reference would panic here (index out of range / nil map / nil state)."""


class _Rejected(Exception):
    """processAttestation returned an error (the attestation is not processed)."""


class Active:
    """types.ActiveState: the proto plus the block vote cache map (shared, like Go's)."""

    def __init__(self, data, cache):
        self.data, self.cache = data, cache


class DeviceVoteCache:
    """The Go ``map[[32]byte]*VoteCache`` (types/state.go:27-31) with its values in HBM:
    a host dict hash -> slot, and per slot an nval-bit voter bitmap and VoteTotalDeposit."""

    def __init__(self, nval, device, torch):
        self.torch, self.dev = torch, device
        self.nval = nval
        self.words = (nval + 31) // 32
        self.slot_of = {}
        self.cap = 0
        self.bitmaps = torch.zeros(0, dtype=torch.int32, device=device)
        self.totals = torch.zeros(0, dtype=torch.int64, device=device)

    def slot(self, h):
        s = self.slot_of.get(h)
        if s is None:
            s = len(self.slot_of)
            self.slot_of[h] = s
            if s >= self.cap:
                self._grow(max(64, 2 * self.cap))
        return s

    def _grow(self, cap):
        torch = self.torch
        bm = torch.zeros(cap * self.words, dtype=torch.int32, device=self.dev)
        tt = torch.zeros(cap, dtype=torch.int64, device=self.dev)
        if self.cap:
            bm[:self.cap * self.words].copy_(self.bitmaps)
            tt[:self.cap].copy_(self.totals)
        self.bitmaps, self.totals, self.cap = bm, tt, cap

    def totals_of(self, hashes):
        """VoteTotalDeposit of each hash (0 when absent), one D2H copy."""
        slots = [self.slot_of.get(h, -1) for h in hashes]
        have = [s for s in slots if s >= 0]
        got = {}
        if have:
            idx = self.torch.tensor(have, dtype=self.torch.int64, device=self.dev)
            vals = self.totals.index_select(0, idx).cpu().numpy().view(np.uint64)
            got = dict(zip(have, (int(v) for v in vals)))
        return [got.get(s, 0) if s >= 0 else None for s in slots]

    def all_totals(self):
        t = self.totals[:len(self.slot_of)].cpu().numpy().view(np.uint64)
        return {h: int(t[s]) for h, s in self.slot_of.items()}


class _Committees:
    """ShardAndCommitteesForSlots as a device CSR of the distinct committee arrays (the
    genesis state repeats one 64-slot cycle four times, types/state.go:75-78) plus the host
    lookup (array index, shard id) -> committee id of getAttesterIndices (core.go:363-374)."""

    def __init__(self, arrays, device, torch):
        ids = {}
        members, offs = [], [0]
        self.lookup = []
        for arr in arrays:
            m = {}
            for sc in arr.array_shard_and_committee:
                key = id(sc.committee)
                if key not in ids:
                    ids[key] = len(offs) - 1
                    members.append(np.asarray(sc.committee, dtype=np.uint32))
                    offs.append(offs[-1] + len(sc.committee))
                m.setdefault(int(sc.shard_id), ids[key])  # the first match wins
            self.lookup.append(m)
        self.sizes = np.diff(np.array(offs, dtype=np.int64))
        self.committee = torch.from_numpy(np.concatenate(members).view(np.int32) if members
                                          else np.zeros(1, np.int32)).to(device)
        self.coffs = torch.from_numpy(np.array(offs, dtype=np.uint64).view(np.int64)).to(device)

    def find(self, index, shard):
        """-> committee id, or raises like getAttesterIndices."""
        if index < 0 or index >= len(self.lookup):
            raise ChainPanic("ShardAndCommitteesForSlots index %d out of range [0,%d)" % (index, len(self.lookup)))
        c = self.lookup[index].get(shard)
        if c is None:
            raise _Rejected("unable to find attestation based on slot, shardID: %d" % shard)
        return c


def _csr(blobs):
    offs = np.zeros(len(blobs) + 1, dtype=np.uint64)
    if blobs:
        offs[1:] = np.cumsum([len(b) for b in blobs], dtype=np.uint64)
    return np.frombuffer(b"".join(blobs) + bytes(16), dtype=np.uint8), offs


def hash_csr(blobs, out_bytes):
    """BLAKE2b-512 (first ``out_bytes``) of many messages in one GPU launch."""
    if not blobs:
        return []
    data, offs = _csr(blobs)
    out = _lib.blake2b512_csr(data, offs, out_bytes)
    return [bytes(r) for r in out]


def _message(att, parents):
    """blockchain/core.go:277-290: 10 zero bytes with uvarint(slot % 64) then uvarint(shard)
    written at offset 0, the signed hashes each followed by ' ', the shard block hash."""
    head = bytearray(10)
    v = wire.varint(att.slot % CYCLE_LENGTH)
    head[:len(v)] = v
    v = wire.varint(att.shard_id)
    head[:len(v)] = v
    return bytes(head) + b"".join(h + b" " for h in parents) + bytes(att.shard_block_hash)


class BeaconChain:
    """BeaconChain (core.go) + the ChainService fields the block pipeline uses, on one GPU."""

    def __init__(self, nval, device=None):
        import torch
        self.torch = torch
        self.dev = torch.device(device if device is not None else "cuda")
        idx = self.dev.index or 0
        lib.call("pz_init", idx)
        self.stream = torch.cuda.current_stream(self.dev)
        active, crystallized = new_genesis_states(nval)
        self.nval = nval
        self.A = Active(active.data, {})
        self.C = crystallized.data
        self.saved = set()
        self.candidate = None
        self.votes = DeviceVoteCache(nval, self.dev, torch)
        self.comm = _Committees(self.C.shard_and_committees_for_slots, self.dev, torch)
        v = self.C.validators
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(self.dev)  # noqa: E731
        self.balance, self.start, self.end = T(v.balance), T(v.start_dynasty), T(v.end_dynasty)
        self._host_balance_valid = True
        # vote tally queue (flushed in one launch)
        self._q_bits, self._q_comm, self._q_items_att, self._q_items_slot = [], [], [], []
        # epoch scratch (one instance)
        self._act_mask = torch.zeros((nval + 63) // 64 + 1, dtype=torch.int64, device=self.dev)
        self._blk_cnt = torch.zeros((nval + 2047) // 2048 + 1, dtype=torch.int32, device=self.dev)
        self._act_list = torch.zeros(max(nval, 1), dtype=torch.int32, device=self.dev)
        self.genesis_hash = hash_csr([wire.beacon_block(new_genesis_block().data)], 32)[0]

    # ---- device helpers -------------------------------------------------------------------
    def _sh(self):
        return ctypes.c_void_p(self.stream.cuda_stream)

    def _up(self, a, dtype):
        a = np.ascontiguousarray(a, dtype=dtype)
        if not a.flags.writeable:
            a = a.copy()
        if a.size == 0:
            a = np.zeros(1, dtype=dtype)
        view = {np.uint64: np.int64, np.uint32: np.int32, np.uint8: np.uint8}[dtype]
        return self.torch.from_numpy(a.view(view)).to(self.dev)

    def flush_votes(self):
        """Run every queued (attestation, hash slot) tally item in one launch."""
        if not self._q_items_att:
            return
        torch = self.torch
        bits, boffs = _csr(self._q_bits)
        d_bits = self._up(bits, np.uint8)
        d_boffs = self._up(boffs, np.uint64)
        d_comm = self._up(np.array(self._q_comm, dtype=np.uint32), np.uint32)
        d_ia = self._up(np.array(self._q_items_att, dtype=np.uint32), np.uint32)
        d_is = self._up(np.array(self._q_items_slot, dtype=np.uint32), np.uint32)
        err = torch.zeros(1, dtype=torch.int64, device=self.dev)
        vb = _lib.VoteBatch()
        vb.committee, vb.coffs = self.comm.committee.data_ptr(), self.comm.coffs.data_ptr()
        vb.att_comm, vb.bits, vb.boffs = d_comm.data_ptr(), d_bits.data_ptr(), d_boffs.data_ptr()
        vb.item_att, vb.item_slot, vb.nitems = d_ia.data_ptr(), d_is.data_ptr(), len(self._q_items_att)
        vb.balance, vb.nval = self.balance.data_ptr(), self.nval
        vb.bitmaps, vb.words_per_slot = self.votes.bitmaps.data_ptr(), self.votes.words
        vb.totals, vb.err = self.votes.totals.data_ptr(), err.data_ptr()
        lib.call("pz_dev_vote_tally", ctypes.byref(vb), self._sh())
        self._q_bits, self._q_comm, self._q_items_att, self._q_items_slot = [], [], [], []
        if int(err.item()):
            raise ChainPanic("calculateBlockVoteCache: CheckBit / validator index out of range")

    # ---- core.go --------------------------------------------------------------------------
    def _recent(self, A):
        """RecentBlockHashes() (types/state.go:189-195), memoised per ActiveState: only the
        genesis list holds non-32-byte entries, and the list object is replaced (never
        edited) whenever it changes."""
        lst = A.data.recent_block_hashes
        memo = getattr(A, "_recent_memo", None)
        if memo is None or memo[0] is not lst:
            memo = (lst, [h if len(h) == 32 else bytes_to_hash(h) for h in lst])
            A._recent_memo = memo
        return memo[1]

    def _signed_parents(self, A, block_slot, att):
        """core.go:348-360 (Go slices up to cap: beyond len panics)."""
        start = (block_slot - att.slot) & M64
        end = (block_slot - att.slot - len(att.oblique_parent_hashes) + CYCLE_LENGTH) & M64
        recent = self._recent(A)
        if start > end or end > len(recent):
            raise ChainPanic("slice bounds out of range [%d:%d] with length %d" % (start, end, len(recent)))
        return recent[start:end] + [bytes_to_hash(h) for h in att.oblique_parent_hashes]

    def _committee(self, C, att):
        return self.comm.find((att.slot - C.last_state_recalc) & M64 if att.slot >= C.last_state_recalc
                              else -1, att.shard_id)

    def _process_attestation(self, block_slot, att):
        """core.go:240-297 -> the message whose digest the reference logs."""
        if att.slot > block_slot:
            raise _Rejected("attestation slot number can't be higher than block slot number")
        if att.slot < block_slot - CYCLE_LENGTH:
            raise _Rejected("attestation slot number can't be lower than block slot number by one CycleLength")
        if att.justified_slot != self.C.last_justified_slot:
            raise _Rejected("attestation's last justified slot has to match")
        parents = self._signed_parents(self.A, block_slot, att)
        c = self._committee(self.C, att)
        k = int(self.comm.sizes[c])
        bf = bytes(att.attester_bitfield)
        if (k + 7) // 8 != len(bf):  # validateAttesterBitfields, core.go:377-394
            raise _Rejected("attestation has incorrect bitfield length")
        if k % 8 and bf[-1] & (0xFF >> (k % 8)):
            raise _Rejected("attestation has non-zero trailing bits")
        return _message(att, parents)

    def _queue_vote_cache(self, block_slot, att):
        """core.go:300-345: queue one tally item per signed parent hash (device work)."""
        if self.A.cache is None:
            raise ChainPanic("assignment to entry in nil map")
        parents = self._signed_parents(self.A, block_slot, att)
        c = self._committee(self.C, att)
        obl = {bytes(o) for o in att.oblique_parent_hashes}
        a = len(self._q_comm)
        self._q_comm.append(c)
        self._q_bits.append(bytes(att.attester_bitfield))
        for h in parents:
            if h in obl:
                continue
            self._q_items_att.append(a)
            self._q_items_slot.append(self.votes.slot(h))
        if len(self._q_items_att) > (1 << 22):
            self.flush_votes()

    def _state_recalc(self, C, A, block_slot):
        """core.go:398-497 -> (new C, new A).  Balances and crosslink records of ``C`` are
        updated in place (shared with the new C), like the reference."""
        self.flush_votes()
        streak, justified, finalized = C.justified_streak, C.last_justified_slot, C.last_finalized_slot
        lsr = C.last_state_recalc
        recent = self._recent(A)
        totals = self.votes.totals_of(recent[:CYCLE_LENGTH]) if A.cache is not None else [None] * CYCLE_LENGTH
        for i in range(CYCLE_LENGTH):
            slot = (lsr - CYCLE_LENGTH + i) & M64
            bal = totals[i] or 0
            if (3 * bal) & M64 >= (2 * C.total_deposits) & M64:
                if slot > justified:
                    justified = slot
                streak = (streak + 1) & M64
            else:
                streak = 0
            if streak >= CYCLE_LENGTH + 1 and ((slot - CYCLE_LENGTH) & M64) > finalized:
                finalized = (slot - CYCLE_LENGTH) & M64
        pending = list(A.data.pending_attestations)
        nxt = self._epoch_on_device(C, pending, block_slot)
        nc = pb.CrystallizedState(
            validators=C.validators, last_state_recalc=(lsr + CYCLE_LENGTH) & M64,
            shard_and_committees_for_slots=C.shard_and_committees_for_slots,
            last_justified_slot=justified, justified_streak=streak, last_finalized_slot=finalized,
            crosslinking_start_shard=0, crosslink_records=C.crosslink_records,
            dynasty_seed_last_reset=C.dynasty_seed_last_reset, total_deposits=nxt)
        hashes = []
        for h in recent:
            hashes.append(h)
            while len(hashes) > 2 * CYCLE_LENGTH:
                hashes = hashes[1:]
        na = pb.ActiveState(pending_attestations=[a for a in pending if a.slot > lsr], recent_block_hashes=hashes)
        return nc, Active(na, A.cache)

    def _epoch_on_device(self, C, pending, block_slot):
        """processCrosslinks (core.go:502-558) + CalculateRewards (incentives.go:14-32) +
        the next-cycle balance (core.go:459-464) as one device epoch instance."""
        torch = self.torch
        comm = []
        for att in pending:
            try:
                comm.append(self._committee(C, att))
            except _Rejected as e:  # stateRecalc errors out; the caller then dereferences nil
                raise ChainPanic("stateRecalc failed (%s): nil state dereference" % e)
        bits, boffs = _csr([bytes(a.attester_bitfield) for a in pending])
        recs = C.crosslink_records
        d = dict(
            bits=self._up(bits, np.uint8), boffs=self._up(boffs, np.uint64),
            att_comm=self._up(np.array(comm, dtype=np.uint32), np.uint32),
            att_shard=self._up(np.array([min(a.shard_id, 0xFFFFFFFF) for a in pending], dtype=np.uint32),
                               np.uint32),
            rec_dyn=self._up(np.array([r.dynasty for r in recs], dtype=np.uint64), np.uint64),
            dynasty=self._up(np.array([C.current_dynasty], dtype=np.uint64), np.uint64),
            tdep=self._up(np.array([C.total_deposits], dtype=np.uint64), np.uint64),
            scal=torch.zeros(8, dtype=torch.int64, device=self.dev),
            vote=torch.zeros(max(len(pending), 1), dtype=torch.int64, device=self.dev),
            total=torch.zeros(max(len(pending), 1), dtype=torch.int64, device=self.dev),
            winner=torch.zeros(max(len(recs), 1), dtype=torch.int32, device=self.dev))
        b = EpochBatch()
        b.ninst, b.nval, b.val_offset, b.nval_global = 1, self.nval, 0, self.nval
        b.kind = _lib.KIND_ACTIVE
        b.balance, b.start, b.end = self.balance.data_ptr(), self.start.data_ptr(), self.end.data_ptr()
        b.dynasty, b.total_deposit = d["dynasty"].data_ptr(), d["tdep"].data_ptr()
        b.natt, b.bits, b.boffs = len(pending), d["bits"].data_ptr(), d["boffs"].data_ptr()
        b.max_inst_bytes = int(boffs[-1])
        b.pop_rank, b.pop_world = 0, 1
        b.committee, b.coffs = self.comm.committee.data_ptr(), self.comm.coffs.data_ptr()
        b.att_comm, b.att_shard = d["att_comm"].data_ptr(), d["att_shard"].data_ptr()
        b.nrec, b.rec_dynasty, b.winner = len(recs), d["rec_dyn"].data_ptr(), d["winner"].data_ptr()
        b.vote, b.total, b.scal = d["vote"].data_ptr(), d["total"].data_ptr(), d["scal"].data_ptr()
        b.act_mask, b.blk_cnt, b.act_list = (self._act_mask.data_ptr(), self._blk_cnt.data_ptr(),
                                             self._act_list.data_ptr())
        b.scal_next = None
        if any(a.shard_id > 0xFFFFFFFF for a in pending):
            raise ChainPanic("crosslink record index out of range")
        lib.call("pz_dev_epoch_count", ctypes.byref(b), self._sh())
        lib.call("pz_dev_epoch_finish", ctypes.byref(b), self._sh())
        scal = d["scal"].cpu().numpy().view(np.uint64)
        if scal[_lib.SCAL_ERR_XL]:
            raise ChainPanic("processCrosslinks: index out of range (member, bitfield or shard)")
        dep = (int(scal[_lib.SCAL_POP]) * 32) & M64
        thr = (dep * 3) & M64 >= (C.total_deposits * 2) & M64
        if thr and scal[_lib.SCAL_NACT] > 0 and scal[_lib.SCAL_ERR_RWD]:
            raise ChainPanic("CalculateRewards: CheckBit index out of range (incentives.go:23)")
        win = d["winner"].cpu().numpy().view(np.uint32)
        for s in np.nonzero(win[:len(recs)] != 0xFFFFFFFF)[0]:
            att = pending[int(win[s])]
            recs[int(s)] = pb.CrosslinkRecord(dynasty=C.current_dynasty, blockhash=bytes(att.shard_block_hash),
                                              slot=block_slot)
        if scal[_lib.SCAL_APPLIED]:
            self._host_balance_valid = False
        return int(scal[_lib.SCAL_NEXT_BAL])

    # ---- service.go -----------------------------------------------------------------------
    def _update_head(self):
        _, self.A, self.C = self.candidate
        self.candidate = None

    def process_blocks(self, blocks):
        """Feed ``blocks`` (pb.BeaconBlock, in order) through blockProcessing.  Returns
        per-block records (digest, status, transition, processed attestations' Key / Hash /
        64-byte message digests) -- the data the reference stores or logs."""
        n = len(blocks)
        bh = hash_csr([wire.beacon_block(b) for b in blocks], 32)
        all_atts = [a for b in blocks for a in b.attestations]
        dig = hash_csr([wire.attestation_record(a) for a in all_atts]
                       + [_key_bytes(a) for a in all_atts], 32)
        att_hash, att_key = dig[:len(all_atts)], dig[len(all_atts):]
        recs, msgs, msg_slots = [], [], []
        ai = 0
        for bi in range(n):
            block = blocks[bi]
            h = bh[bi]
            slot = block.slot_number
            rec = {"hash": h, "slot": slot, "atts": [], "status": "processed", "transition": False}
            recs.append(rec)
            a0 = ai
            ai += len(block.attestations)
            if copy32(block.parent_hash) not in self.saved and slot > 1:
                rec["status"] = "no_parent"
                continue
            processed, can_atts = [], False
            for j, att in enumerate(block.attestations):
                try:
                    msg = self._process_attestation(slot, att)
                except _Rejected as e:
                    can_atts = False
                    rec["atts"].append({"error": str(e)})
                    continue
                can_atts = True
                rec["atts"].append({"key": att_key[a0 + j], "hash": att_hash[a0 + j]})
                msgs.append(msg)
                msg_slots.append(rec["atts"][-1])
                processed.append(att)
            if not can_atts:
                rec["status"] = "attestations_rejected"
                continue
            vote_cache = None
            for att in block.attestations:
                try:
                    self._queue_vote_cache(slot, att)
                    vote_cache = self.A.cache
                except _Rejected:
                    vote_cache = None
            if self.candidate is not None and slot > self.candidate[0].slot_number and slot > 1:
                self._update_head()
            self.saved.add(h)
            if self.candidate is not None:
                rec["status"] = "saved_not_candidate"
                continue
            A, C = self.A, self.C
            if slot >= C.last_state_recalc + CYCLE_LENGTH:
                rec["transition"] = True
                C, A = self._state_recalc(C, A, slot)
            A.cache = vote_cache
            A.data.pending_attestations.extend(processed)
            hashes = self._recent(A) + [h]
            while len(hashes) > 2 * CYCLE_LENGTH:
                hashes = hashes[1:]
            A.data.recent_block_hashes = hashes
            self.candidate = (block, A, C)
        self.flush_votes()
        for r, d in zip(msg_slots, hash_csr(msgs, 64)):
            r["msg"] = d
            r["msg_len"] = None
        for r, m in zip(msg_slots, msgs):
            r["msg_len"] = len(m)
        return recs

    # ---- roots ----------------------------------------------------------------------------
    def _sync_host_balances(self):
        if not self._host_balance_valid:
            self.C.validators.balance[:] = self.balance.cpu().numpy().view(np.uint64)
            self._host_balance_valid = True

    def roots(self):
        """State roots (types/state.go:138-149, 237-248) of the chain's and the candidate's
        states (one GPU launch) and the vote cache totals."""
        self._sync_host_balances()
        states = [wire.active_state(self.A.data), wire.crystallized_state(self.C)]
        if self.candidate is not None:
            _, A, C = self.candidate
            states += [wire.active_state(A.data), wire.crystallized_state(C)]
        d = hash_csr(states, 32)
        out = {"chain_active": d[0], "chain_crystallized": d[1]}
        if self.candidate is not None:
            out["cand_active"], out["cand_crystallized"] = d[2], d[3]
        cache = self.A.cache if self.candidate is None else self.candidate[1].cache
        out["vote_totals"] = {} if cache is None else self.votes.all_totals()
        return out


def _key_bytes(a):
    """types/attestation.go:61-77 Key() preimage."""
    from prysm_amd.types import Attestation
    return Attestation(a).key_bytes()


__all__ = ["BeaconChain", "ChainPanic", "DeviceVoteCache", "PzError", "SHARD_COUNT"]
