"""The product's proto3 encoder (prysm_amd/wire.py) emits the same bytes as Google's protobuf
runtime over the oracle schema (oracle/schema.py, pinned to the reference descriptor).  CPU."""
import numpy as np
import pytest

from oracle import ref
from oracle import schema as opb
from prysm_amd import pb, wire

M64 = (1 << 64) - 1


def rand_bytes(rng, lo, hi):
    return rng.integers(0, 256, size=int(rng.integers(lo, hi)), dtype=np.uint8).tobytes()


def rand_u64(rng):
    k = int(rng.integers(0, 5))
    return [0, 1, 127, 128, int(rng.integers(0, 1 << 63)) * 2 + 1][k]


def rand_att(rng):
    return pb.AttestationRecord(
        slot=rand_u64(rng), shard_id=rand_u64(rng), justified_slot=rand_u64(rng),
        justified_block_hash=rand_bytes(rng, 0, 40), shard_block_hash=rand_bytes(rng, 0, 40),
        attester_bitfield=rand_bytes(rng, 0, 300),
        oblique_parent_hashes=[rand_bytes(rng, 0, 33) for _ in range(int(rng.integers(0, 4)))],
        aggregate_sig=[rand_u64(rng) for _ in range(int(rng.integers(0, 3)))])


def o_att(a):
    return opb.AttestationRecord(slot=a.slot, shard_id=a.shard_id, justified_slot=a.justified_slot,
                                 justified_block_hash=a.justified_block_hash, shard_block_hash=a.shard_block_hash,
                                 attester_bitfield=a.attester_bitfield, oblique_parent_hashes=a.oblique_parent_hashes,
                                 aggregate_sig=a.aggregate_sig)


def o_block(b):
    o = opb.BeaconBlock(parent_hash=b.parent_hash, slot_number=b.slot_number, randao_reveal=b.randao_reveal,
                        pow_chain_ref=b.pow_chain_ref, active_state_hash=b.active_state_hash,
                        crystallized_state_hash=b.crystallized_state_hash)
    if b.timestamp is not None:
        o.timestamp.SetInParent()
        o.timestamp.seconds = b.timestamp.seconds
        o.timestamp.nanos = b.timestamp.nanos
    for a in b.attestations:
        o.attestations.add().CopyFrom(o_att(a))
    return o


def o_cstate(s):
    o = opb.CrystallizedState(last_state_recalc=s.last_state_recalc, justified_streak=s.justified_streak,
                              last_justified_slot=s.last_justified_slot, last_finalized_slot=s.last_finalized_slot,
                              current_dynasty=s.current_dynasty, crosslinking_start_shard=s.crosslinking_start_shard,
                              total_deposits=s.total_deposits, dynasty_seed=s.dynasty_seed,
                              dynasty_seed_last_reset=s.dynasty_seed_last_reset)
    for r in s.crosslink_records:
        o.crosslink_records.add(dynasty=r.dynasty, blockhash=r.blockhash, slot=r.slot)
    v = s.validators
    for i in range(len(v)):
        o.validators.add(public_key=int(v.public_key[i]), withdrawal_shard=int(v.withdrawal_shard[i]),
                         withdrawal_address=v.withdrawal_address[i] if v.withdrawal_address else b"",
                         randao_commitment=v.randao_commitment[i] if v.randao_commitment else b"",
                         balance=int(v.balance[i]), start_dynasty=int(v.start_dynasty[i]),
                         end_dynasty=int(v.end_dynasty[i]))
    for arr in s.shard_and_committees_for_slots:
        oa = o.shard_and_committees_for_slots.add()
        for sc in arr.array_shard_and_committee:
            oa.array_shard_and_committee.add(shard_id=sc.shard_id, committee=[int(x) for x in sc.committee])
    return o


@pytest.mark.parametrize("seed", range(20))
def test_attestation_and_block_bytes(seed):
    rng = np.random.default_rng(seed)
    a = rand_att(rng)
    assert wire.attestation_record(a) == o_att(a).SerializeToString()
    ts = None if seed % 3 == 0 else pb.Timestamp(int(rng.integers(-5, 1 << 40)), int(rng.integers(-3, 10 ** 9)))
    b = pb.BeaconBlock(parent_hash=rand_bytes(rng, 0, 33), slot_number=rand_u64(rng),
                       randao_reveal=rand_bytes(rng, 0, 33), pow_chain_ref=rand_bytes(rng, 0, 33),
                       active_state_hash=rand_bytes(rng, 0, 33), crystallized_state_hash=rand_bytes(rng, 0, 33),
                       timestamp=ts, attestations=[rand_att(rng) for _ in range(int(rng.integers(0, 4)))])
    assert wire.beacon_block(b) == o_block(b).SerializeToString()


def test_genesis_block_bytes():
    assert wire.beacon_block(pb.BeaconBlock(timestamp=pb.Timestamp())) == bytes([0x3A, 0x00])
    assert wire.beacon_block(pb.BeaconBlock()) == b""


def test_active_state_bytes():
    rng = np.random.default_rng(5)
    s = pb.ActiveState(pending_attestations=[rand_att(rng) for _ in range(5)],
                       recent_block_hashes=[b""] * 3 + [rand_bytes(rng, 32, 33) for _ in range(4)])
    o = opb.ActiveState(recent_block_hashes=s.recent_block_hashes)
    for a in s.pending_attestations:
        o.pending_attestations.add().CopyFrom(o_att(a))
    assert wire.active_state(s) == o.SerializeToString()
    assert wire.active_state(pb.ActiveState(recent_block_hashes=[b""] * 128)) == bytes([0x12, 0]) * 128


@pytest.mark.parametrize("n,with_bytes", [(0, False), (1, False), (300, False), (50, True)])
def test_crystallized_state_bytes(n, with_bytes):
    rng = np.random.default_rng(n)
    big = lambda: np.array([rand_u64(rng) for _ in range(n)], dtype=np.uint64)  # noqa: E731
    vals = pb.Validators(n, public_key=big(), withdrawal_shard=big(), balance=big(), start_dynasty=big(),
                         end_dynasty=big(),
                         withdrawal_address=[rand_bytes(rng, 0, 21) for _ in range(n)] if with_bytes else None,
                         randao_commitment=[rand_bytes(rng, 0, 3) for _ in range(n)] if with_bytes else None)
    arrs = [pb.ShardAndCommitteeArray([pb.ShardAndCommittee(int(rng.integers(0, 1024)),
                                                            rng.integers(0, 1 << 22, size=int(rng.integers(0, 9)),
                                                                         dtype=np.uint32))
                                       for _ in range(int(rng.integers(0, 3)))]) for _ in range(5)]
    s = pb.CrystallizedState(last_state_recalc=rand_u64(rng), justified_streak=7, last_justified_slot=0,
                             last_finalized_slot=rand_u64(rng), current_dynasty=1, crosslinking_start_shard=3,
                             total_deposits=rand_u64(rng), dynasty_seed=rand_bytes(rng, 0, 33),
                             dynasty_seed_last_reset=rand_u64(rng),
                             crosslink_records=[pb.CrosslinkRecord(rand_u64(rng), rand_bytes(rng, 0, 33), rand_u64(rng))
                                                for _ in range(7)],
                             validators=vals, shard_and_committees_for_slots=arrs)
    assert wire.crystallized_state(s) == o_cstate(s).SerializeToString()


def test_genesis_validator_record_13_bytes():
    v = pb.Validators(1, balance=[32], end_dynasty=[ref.DEFAULT_END_DYNASTY])
    assert wire.validators(v) == bytes.fromhex("5a0d282038ffff9fcfc8e0c8e38a01")


def test_c_port_validators_match_protobuf_runtime():
    """oracle/c/wire_ref.c (bench.py's wire cpu_baseline) against the runtime, bytes fields
    included."""
    from oracle import cport

    rng = np.random.default_rng(21)
    n = 500
    v = pb.Validators(n, public_key=[rand_u64(rng) for _ in range(n)],
                      withdrawal_shard=[rand_u64(rng) for _ in range(n)],
                      withdrawal_address=[rand_bytes(rng, 0, 3) * 50 for _ in range(n)],
                      randao_commitment=[rand_bytes(rng, 0, 40) for _ in range(n)],
                      balance=[rand_u64(rng) for _ in range(n)], start_dynasty=[rand_u64(rng) for _ in range(n)],
                      end_dynasty=[rand_u64(rng) for _ in range(n)])
    o = opb.CrystallizedState()
    for i in range(n):
        o.validators.add(public_key=int(v.public_key[i]), withdrawal_shard=int(v.withdrawal_shard[i]),
                         withdrawal_address=v.withdrawal_address[i], randao_commitment=v.randao_commitment[i],
                         balance=int(v.balance[i]), start_dynasty=int(v.start_dynasty[i]),
                         end_dynasty=int(v.end_dynasty[i]))
    assert cport.wire_validators(v) == o.SerializeToString() == wire.validators(v)


def test_c_port_attestations_match_protobuf_runtime():
    """oracle/c/wire_ref.c's AttestationRecord marshaller (bench.py's wire_att cpu_baseline)
    against the runtime, on records that hit every field rule."""
    from oracle import cport

    rng = np.random.default_rng(33)
    atts = [rand_att(rng) for _ in range(400)]
    port = cport.WireAtt(wire.attestation_columns(atts), len(atts))
    try:
        raw, offs = port.run()
    finally:
        port.close()
    for i, a in enumerate(atts):
        assert raw[int(offs[i]):int(offs[i + 1])] == o_att(a).SerializeToString(), i
