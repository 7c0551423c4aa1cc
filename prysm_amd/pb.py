"""Host-side message types mirroring ``proto/beacon/p2p/v1/messages.proto:37-125``.

Plain dataclasses with the Go struct's field names in snake_case.  ``None`` stands for a Go
nil message pointer (omitted on the wire); ``b""`` and ``None`` are the same for proto3
bytes scalars.  ``CrystallizedState.validators`` is a ``Validators`` SoA block (the layout
the GPU path and the vectorised encoder use) instead of ``[]*ValidatorRecord``.
"""
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np


@dataclass
class Timestamp:  # google/protobuf/timestamp.proto
    seconds: int = 0
    nanos: int = 0


@dataclass
class AttestationRecord:  # messages.proto:110-119, messages.pb.go:889-896
    slot: int = 0
    shard_id: int = 0
    justified_slot: int = 0
    justified_block_hash: bytes = b""
    shard_block_hash: bytes = b""
    attester_bitfield: bytes = b""
    oblique_parent_hashes: List[bytes] = field(default_factory=list)
    aggregate_sig: List[int] = field(default_factory=list)


@dataclass
class BeaconBlock:  # messages.proto:37-46, messages.pb.go:225-232
    parent_hash: bytes = b""
    slot_number: int = 0
    randao_reveal: bytes = b""
    pow_chain_ref: bytes = b""
    active_state_hash: bytes = b""
    crystallized_state_hash: bytes = b""
    timestamp: Optional[Timestamp] = None
    attestations: List[AttestationRecord] = field(default_factory=list)


@dataclass
class CrosslinkRecord:  # messages.proto:121-125
    dynasty: int = 0
    blockhash: bytes = b""
    slot: int = 0


@dataclass
class ShardAndCommittee:  # messages.proto:85-88 (committee packed)
    shard_id: int = 0
    committee: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=np.uint32))


@dataclass
class ShardAndCommitteeArray:  # messages.proto:76-78
    array_shard_and_committee: List[ShardAndCommittee] = field(default_factory=list)


@dataclass
class ActiveState:  # messages.proto:94-97
    pending_attestations: List[AttestationRecord] = field(default_factory=list)
    recent_block_hashes: List[bytes] = field(default_factory=list)


class Validators:
    """SoA block of ValidatorRecord (messages.proto:99-107).  Bytes fields are lists of
    bytes or None (all empty)."""

    def __init__(self, n=0, public_key=None, withdrawal_shard=None, withdrawal_address=None,
                 randao_commitment=None, balance=None, start_dynasty=None, end_dynasty=None):
        z = lambda a: np.zeros(n, np.uint64) if a is None else np.ascontiguousarray(a, dtype=np.uint64)  # noqa
        self.public_key = z(public_key)
        self.withdrawal_shard = z(withdrawal_shard)
        self.balance = z(balance)
        self.start_dynasty = z(start_dynasty)
        self.end_dynasty = z(end_dynasty)
        self.withdrawal_address = withdrawal_address
        self.randao_commitment = randao_commitment

    def __len__(self):
        return int(self.balance.shape[0])


@dataclass
class CrystallizedState:  # messages.proto:59-72
    last_state_recalc: int = 0
    justified_streak: int = 0
    last_justified_slot: int = 0
    last_finalized_slot: int = 0
    current_dynasty: int = 0
    crosslinking_start_shard: int = 0
    total_deposits: int = 0
    dynasty_seed: bytes = b""
    dynasty_seed_last_reset: int = 0
    crosslink_records: List[CrosslinkRecord] = field(default_factory=list)
    validators: Validators = field(default_factory=Validators)
    shard_and_committees_for_slots: List[ShardAndCommitteeArray] = field(default_factory=list)
