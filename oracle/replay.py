"""ORACLE (test infrastructure only) — scalar restatement of the reference's block pipeline.

``replay(blocks, nval)`` feeds blocks, in order, through a restatement of
``ChainService.blockProcessing`` (``blockchain/service.go:229-363``) and ``updateHead``
(``:170-227``) over ``BeaconChain`` (``blockchain/core.go``), with the per-step functions of
``oracle.ref``.  Go semantics kept on purpose (each one changes bytes that get hashed):

* object sharing: the chain's ActiveState is mutated in place by computeNewActiveState
  (``core.go:223-237``) until a cycle transition builds a new one; the block vote cache
  map is one object shared by every ActiveState (``core.go:494-496``,
  ``service.go:313-318``); CalculateRewards / processCrosslinks mutate the chain's
  CrystallizedState's validators and crosslink records in place (``core.go:433-457``);
* ordering: a block's attestations are checked and tallied against the chain state as of
  the previous block's ``updateHead``; ``updateHead`` (``service.go:320-322``) runs after
  the tally and before the transition;
* flags: ``canProcessAttestations`` is the outcome of the LAST attestation
  (``service.go:281-301``); a block without attestations is dropped (``:304-306``), and so
  is any block whose parent was never saved (``:261-269``);
* the vote cache returned by the last ``calculateBlockVoteCache`` call (nil on error) is
  what ``computeNewActiveState`` installs (``service.go:313-318,356``).

Not modelled (no effect on any hashed byte): the DB writes other than block existence,
logging, the p2p feeds, the fork-choice shuffle result (``service.go:185-194`` only logs
it), and ``verifyBlockTimeStamp`` (``core.go:203-220``) — with the genesis Timestamp{0,0}
it holds for every slot on any real clock.  Go panics surface as ``ref.GoPanic``.

Blocks may be any objects with the BeaconBlock / AttestationRecord attribute names
(converted to ``oracle.schema`` messages here).
"""
from oracle import ref
from oracle import schema as pb


def to_pb_block(b):
    o = pb.BeaconBlock(parent_hash=bytes(b.parent_hash), slot_number=b.slot_number,
                       randao_reveal=bytes(b.randao_reveal), pow_chain_ref=bytes(b.pow_chain_ref),
                       active_state_hash=bytes(b.active_state_hash),
                       crystallized_state_hash=bytes(b.crystallized_state_hash))
    if b.timestamp is not None:
        o.timestamp.SetInParent()
        o.timestamp.seconds = b.timestamp.seconds
        o.timestamp.nanos = b.timestamp.nanos
    for a in b.attestations:
        o.attestations.add(slot=a.slot, shard_id=a.shard_id, justified_slot=a.justified_slot,
                           justified_block_hash=bytes(a.justified_block_hash),
                           shard_block_hash=bytes(a.shard_block_hash),
                           attester_bitfield=bytes(a.attester_bitfield),
                           oblique_parent_hashes=[bytes(h) for h in a.oblique_parent_hashes],
                           aggregate_sig=list(a.aggregate_sig))
    return o


class _Active:
    """types.ActiveState: the proto plus the (shared) block vote cache map."""

    def __init__(self, data, cache):
        self.data, self.cache = data, cache


class Chain:
    """BeaconChain + the ChainService fields blockProcessing uses."""

    def __init__(self, nval):
        active, crystallized = ref.new_genesis_states(nval)
        self.A = _Active(active, {})            # beaconState.ActiveState
        self.C = crystallized                   # beaconState.CrystallizedState
        self.saved = set()                      # block hashes in the DB (hasBlock)
        self.candidate = None                   # (block, ActiveState, CrystallizedState)
        self.genesis = ref.new_genesis_block()

    @classmethod
    def reload(cls, crystallized_bytes, saved):
        """NewBeaconChain with a stored CrystallizedState (blockchain/core.go:59-64,86-95): the
        state is proto.Unmarshal'ed from the database, the ActiveState is the genesis one
        (types/state.go:46-57, an empty vote-cache map), and hasBlock answers from the
        database's saved blocks."""
        self = cls.__new__(cls)
        active, _ = ref.new_genesis_states(1)
        cs = pb.CrystallizedState()
        cs.ParseFromString(bytes(crystallized_bytes))
        self.A = _Active(active, {})
        self.C = cs
        self.saved = set(bytes(h) for h in saved)
        self.candidate = None
        self.genesis = ref.new_genesis_block()
        return self

    def update_head(self):
        """service.go:170-227: the candidate's states become the chain's states."""
        _, self.A, self.C = self.candidate
        self.candidate = None

    def process_block(self, block):
        """service.go:238-363 for one block -> a record of what happened."""
        h = ref.block_hash(block)
        slot = block.slot_number
        rec = {"hash": h, "slot": slot, "atts": [], "status": "processed", "transition": False}
        if ref.copy32(block.parent_hash) not in self.saved and slot > 1:
            rec["status"] = "no_parent"
            return rec
        processed = []
        can_atts = False
        for att in block.attestations:
            try:
                msg, digest = ref.process_attestation(self.C, self.A.data, slot, att)
            except ref.GoError as e:
                can_atts = False
                rec["atts"].append({"error": str(e)})
                continue
            can_atts = True
            rec["atts"].append({"key": ref.attestation_key(att), "hash": ref.attestation_hash(att),
                                "msg": digest, "msg_len": len(msg)})
            processed.append(att)
        if not can_atts:
            rec["status"] = "attestations_rejected"
            return rec
        vote_cache = None
        for att in block.attestations:
            try:
                if self.A.cache is None:  # a nil map: the first insert panics
                    raise ref.GoPanic("assignment to entry in nil map")
                ref.calculate_block_vote_cache(self.C, self.A.data, self.A.cache, slot, att)
                vote_cache = self.A.cache
            except ref.GoError:
                vote_cache = None
        if self.candidate is not None and slot > self.candidate[0].slot_number and slot > 1:
            self.update_head()
        self.saved.add(h)
        if self.candidate is not None:
            rec["status"] = "saved_not_candidate"
            return rec
        A, C = self.A, self.C
        if slot >= C.last_state_recalc + ref.CYCLE_LENGTH:  # IsCycleTransition (core.go:181-183)
            rec["transition"] = True
            nc, na = ref.state_recalc(C, A.data, A.cache if A.cache is not None else {}, slot)
            C, A = nc, _Active(na, A.cache)
        # computeNewActiveState (core.go:223-237)
        A.cache = vote_cache
        ref.compute_new_active_state(A.data, processed, h)
        self.candidate = (block, A, C)
        return rec

    def roots(self):
        """State roots (types/state.go:138-149, 237-248) of the chain's and the candidate's
        states, and the vote cache totals."""
        out = {"chain_active": ref.active_state_hash(self.A.data),
               "chain_crystallized": ref.crystallized_state_hash(self.C)}
        if self.candidate is not None:
            _, A, C = self.candidate
            out["cand_active"] = ref.active_state_hash(A.data)
            out["cand_crystallized"] = ref.crystallized_state_hash(C)
        cache = self.A.cache if self.candidate is None else self.candidate[1].cache
        out["vote_totals"] = {} if cache is None else {h: e[1] for h, e in cache.items()}
        return out


    def state_bytes(self):
        """The persisted encodings (blockchain/core.go:161-177) of the same four states."""
        out = {"chain_active": ref.marshal(self.A.data), "chain_crystallized": ref.marshal(self.C)}
        if self.candidate is not None:
            _, A, C = self.candidate
            out["cand_active"] = ref.marshal(A.data)
            out["cand_crystallized"] = ref.marshal(C)
        return out


def replay_from(chain, blocks, with_state_bytes=False):
    """Run ``blocks`` through an existing ``Chain`` (e.g. ``Chain.reload``)."""
    recs = [chain.process_block(to_pb_block(b)) for b in blocks]
    if with_state_bytes:
        return recs, chain.roots(), chain.state_bytes()
    return recs, chain.roots()


def replay(blocks, nval, with_state_bytes=False):
    """Run ``blocks`` (BeaconBlock-like objects, in order) through a fresh genesis chain of
    ``nval`` validators -> (per-block records, roots dict[, state bytes dict])."""
    chain = Chain(nval)
    recs = [chain.process_block(to_pb_block(b)) for b in blocks]
    if with_state_bytes:
        return recs, chain.roots(), chain.state_bytes()
    return recs, chain.roots()
