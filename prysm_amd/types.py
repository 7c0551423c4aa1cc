"""Host-side mirror of the reference's ``beacon-chain/types`` package.

``Hash()`` = proto3 encoding (``prysm_amd.wire``) -> BLAKE2b-512 on the GPU -> first 32 bytes,
exactly ``types/block.go:67-77``, ``attestation.go:49-59``, ``state.go:138-149,237-248``.
The batch helpers (``hash_blocks``, ``hash_attestations``, ``attestation_keys``) are the
coarse cgo entry points SURVEY.md §7 step 7 asks for: one GPU launch for many messages.
A nil message (``data is None``) raises ``PzError(PZ_ENIL)`` where Go returns an error.
"""
import numpy as np

from prysm_amd import _lib, casper, pb, wire
from prysm_amd._lib import PZ_ENIL, PzError
from prysm_amd.params import (BOOTSTRAPPED_VALIDATORS_COUNT, CYCLE_LENGTH, DEFAULT_BALANCE,
                              DEFAULT_END_DYNASTY, SHARD_COUNT)


def _hash_many(blobs):
    return _lib.blake2b512_batch(blobs, out_bytes=32)


def _nil(what):
    return PzError(PZ_ENIL, "could not marshal %s proto data: proto: Marshal called with nil" % what)


def bytes_to_hash(b):
    """go-ethereum common.BytesToHash: keep the last 32 bytes, right-aligned."""
    b = bytes(b)[-32:]
    return bytes(32 - len(b)) + b


def copy32(b):
    """``var h [32]byte; copy(h[:], b)``: left-aligned, truncated."""
    b = bytes(b)[:32]
    return b + bytes(32 - len(b))


def _put_uvarint(buf, x):
    v = wire.varint(x)
    buf[:len(v)] = v


class Block:
    """types/block.go."""

    def __init__(self, data):
        self.data = data

    def marshal(self):
        if self.data is None:
            raise _nil("block")
        return wire.beacon_block(self.data)

    def hash(self):
        return _hash_many([self.marshal()])[0]

    def parent_hash(self):
        return copy32(self.data.parent_hash)

    def slot_number(self):
        return self.data.slot_number

    def attestations(self):
        return self.data.attestations


def new_genesis_block():
    """types/block.go:43-55 (Timestamp{0,0} is a non-nil empty message)."""
    return Block(pb.BeaconBlock(timestamp=pb.Timestamp(0, 0), parent_hash=b""))


class Attestation:
    """types/attestation.go."""

    def __init__(self, data):
        self.data = data

    def marshal(self):
        if self.data is None:
            raise _nil("attestation")
        return wire.attestation_record(self.data)

    def hash(self):
        return _hash_many([self.marshal()])[0]

    def key_bytes(self):
        """attestation.go:61-77: both uvarints are written at offset 0 of a 10-byte buffer
        (shard id over slot), then the raw shard block hash, then each oblique parent hash
        copied into a 32-byte array."""
        key = bytearray(10)
        _put_uvarint(key, self.data.slot)
        _put_uvarint(key, self.data.shard_id)
        key += bytes(self.data.shard_block_hash)
        for h in self.data.oblique_parent_hashes:
            key += copy32(h)
        return bytes(key)

    def key(self):
        return _hash_many([self.key_bytes()])[0]


def hash_blocks(blocks):
    return _hash_many([b.marshal() for b in blocks])


def hash_attestations(atts):
    return _hash_many([a.marshal() for a in atts])


def attestation_keys(atts):
    return _hash_many([a.key_bytes() for a in atts])


class ActiveState:
    """types/state.go:14-19 (+ the block vote cache, kept by the caller)."""

    def __init__(self, data, block_vote_cache=None):
        self.data = data
        self.block_vote_cache = {} if block_vote_cache is None else block_vote_cache

    def marshal(self):
        if self.data is None:
            raise _nil("active state")
        return wire.active_state(self.data)

    def hash(self):
        return _hash_many([self.marshal()])[0]

    def recent_block_hashes(self):
        return [bytes_to_hash(h) for h in self.data.recent_block_hashes]


class CrystallizedState:
    """types/state.go:21-25."""

    def __init__(self, data):
        self.data = data

    def marshal(self):
        if self.data is None:
            raise _nil("crystallized state")
        return wire.crystallized_state(self.data)

    def hash(self):
        return _hash_many([self.marshal()])[0]


def hash_states(states):
    """Many Active/CrystallizedState roots in one launch."""
    return _hash_many([s.marshal() for s in states])


def new_genesis_states(num_validators=BOOTSTRAPPED_VALIDATORS_COUNT):
    """types/state.go:44-112 with ``BootstrappedValidatorsCount`` as a parameter."""
    active = ActiveState(pb.ActiveState(recent_block_hashes=[b""] * (2 * CYCLE_LENGTH)))
    n = num_validators
    vals = pb.Validators(n, balance=np.full(n, DEFAULT_BALANCE, np.uint64),
                         start_dynasty=np.zeros(n, np.uint64),
                         end_dynasty=np.full(n, DEFAULT_END_DYNASTY, np.uint64))
    slots = casper.shuffle_validators_to_committees(bytes_to_hash(b""), vals.start_dynasty, vals.end_dynasty, 1, 0)
    arrs = [pb.ShardAndCommitteeArray([pb.ShardAndCommittee(s, c) for s, c in slot]) for slot in slots]
    arrs = arrs + arrs
    cs = pb.CrystallizedState(
        current_dynasty=1, total_deposits=(n * DEFAULT_BALANCE) & wire.M64,
        crosslink_records=[pb.CrosslinkRecord() for _ in range(SHARD_COUNT)],
        validators=vals, shard_and_committees_for_slots=arrs + arrs)
    return active, CrystallizedState(cs)


def message_shard(n, rank, world):
    """The contiguous slice ``[lo, hi)`` of an n-message batch that ``rank`` of ``world``
    hashes: the same split as pz_comm_blake2b512_batch (message batches shard with no
    collective)."""
    return n * rank // world, n * (rank + 1) // world


def hash_batch_sharded(data, offsets, rank, world, group=None, out_bytes=32, hasher=None):
    """H over one process per GPU: rank ``rank`` hashes its slice of the CSR batch on its GPU
    (``hasher``: the C-ABI batch hash by default; tests substitute a CPU double), and the
    digests are all-gathered over ``torch.distributed`` so every rank returns all n of them
    (n x out_bytes uint8).  The gather is the caller's choice of output placement, not part of
    the hash: a node that consumes its own slice skips it (``group=False``)."""
    import torch
    import torch.distributed as dist

    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    lo, hi = message_shard(n, rank, world)
    local_offs = offsets[lo:hi + 1] - offsets[lo]
    local_data = np.ascontiguousarray(data[int(offsets[lo]):int(offsets[hi])], dtype=np.uint8)
    local_data = np.concatenate([local_data, np.zeros(16, np.uint8)])
    hasher = hasher or (lambda d, o: _lib.blake2b512_csr(d, o, out_bytes))
    mine = hasher(local_data, local_offs) if hi > lo else np.zeros((0, out_bytes), np.uint8)
    if group is False or world == 1:
        return mine
    per = -(-n // world)  # all-gather needs equal sizes: pad every slice to ceil(n / world)
    # RCCL ("nccl") gathers device tensors only: the slices go through this rank's GPU there
    on_dev = dist.get_backend(group) == "nccl"
    where = torch.device("cuda", torch.cuda.current_device()) if on_dev else torch.device("cpu")
    send = torch.zeros(per * out_bytes, dtype=torch.uint8, device=where)
    send[:mine.size] = torch.from_numpy(mine.reshape(-1).copy()).to(where)
    bufs = [torch.zeros_like(send) for _ in range(world)]
    dist.all_gather(bufs, send, group=group)
    out = np.zeros((n, out_bytes), np.uint8)
    for r in range(world):
        a, b = message_shard(n, r, world)
        out[a:b] = bufs[r].cpu().numpy()[:(b - a) * out_bytes].reshape(b - a, out_bytes)
    return out
