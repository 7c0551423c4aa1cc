"""Pin the oracle against every known-answer test the reference's own Go tests hold for the
hot path.  CPU only."""
import hashlib

import numpy as np

import pytest

from oracle import ref
from oracle import schema as pb


def _validators(specs):
    out = []
    for spec in specs:
        out.append(pb.ValidatorRecord(**spec))
    return out


def test_rfc7693_abc():
    # RFC 7693 Appendix A: BLAKE2b-512("abc")
    want = ("ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
            "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923")
    assert ref.sum512(b"abc").hex() == want
    assert ref.hash32(b"abc").hex() == want[:64]


def test_check_bit_kat():
    # utils/checkbit_test.go:7-27
    for a, b, c in [(200, 4, True), (148, 5, True), (146, 4, False), (179, 7, True), (49, 6, False)]:
        assert ref.check_bit(bytes([a]), b) is c


def test_bit_set_count_kat():
    # utils/checkbit_test.go:29-45
    for a, b in [(200, 3), (148, 3), (146, 3), (179, 5), (49, 3)]:
        assert ref.bit_set_count(a) == b
    for v in range(256):
        assert ref.bit_set_count(v) == bin(v).count("1")


def test_bit_length_kat():
    # utils/checkbit_test.go:47-61
    for a, b in [(200, 25), (34324, 4291), (146, 19), (179, 23), (49, 7)]:
        assert ref.bit_length(a) == b


def test_check_bit_panics():
    with pytest.raises(ref.GoPanic):
        ref.check_bit(b"\x01", 8)
    with pytest.raises(ref.GoPanic):
        ref.check_bit(b"", 0)


def test_has_voted():
    # casper/validator_test.go:68-92
    for i in range(1):
        assert ref.check_bit(bytes([255]), i)
    assert not ref.check_bit(bytes([85]), 0)


def test_compute_rewards_kat():
    # casper/incentives_test.go:9-43
    vals = _validators([dict(balance=32, start_dynasty=1, end_dynasty=10)] * 40)
    atts = [pb.AttestationRecord(attester_bitfield=bytes([200, 148, 146, 179, 49]))]
    out = ref.calculate_rewards(atts, vals, 1, 100)
    assert out[0].balance == 33
    assert out[7].balance == 31
    assert out[29].balance == 31


def test_validator_indices_kat():
    # casper/validator_test.go:94-141
    inf = 1 << 63  # uint64(math.Inf(0)) on amd64 == 0x8000000000000000
    vals = _validators([
        dict(start_dynasty=0, end_dynasty=2), dict(start_dynasty=0, end_dynasty=2),
        dict(start_dynasty=1, end_dynasty=2), dict(start_dynasty=0, end_dynasty=2),
        dict(start_dynasty=0, end_dynasty=3), dict(start_dynasty=2, end_dynasty=inf)])
    assert ref.active_validator_indices(vals, 1) == [0, 1, 2, 3, 4]
    assert ref.queued_validator_indices(vals, 1) == [5]
    assert ref.exited_validator_indices(vals, 1) == []
    vals = _validators([
        dict(start_dynasty=1, end_dynasty=inf), dict(start_dynasty=2, end_dynasty=inf),
        dict(start_dynasty=6, end_dynasty=inf), dict(start_dynasty=7, end_dynasty=inf),
        dict(start_dynasty=1, end_dynasty=2), dict(start_dynasty=1, end_dynasty=3)])
    assert ref.active_validator_indices(vals, 5) == [0, 1]
    assert ref.queued_validator_indices(vals, 5) == [2, 3]
    assert ref.exited_validator_indices(vals, 5) == [4, 5]


def test_rotate_validator_set_kat():
    # casper/validator_test.go:13-66
    E = ref.DEFAULT_END_DYNASTY
    vals = _validators([dict(balance=b, start_dynasty=s, end_dynasty=E)
                        for b, s in [(10, 0), (15, 1), (20, 2), (25, 3), (30, 4), (30, 15)]])
    ref.rotate_validator_set(vals, 10)
    assert ref.active_validator_indices(vals, 10) == [2, 3, 4, 5]
    assert ref.queued_validator_indices(vals, 10) == []
    assert ref.exited_validator_indices(vals, 10) == [0, 1]
    vals = _validators([dict(balance=b, start_dynasty=s, end_dynasty=E)
                        for b, s in [(10, 0), (15, 1), (20, 2), (25, 3), (30, 4)]])
    ref.rotate_validator_set(vals, 10)
    assert ref.active_validator_indices(vals, 10) == [2, 3, 4]
    assert ref.exited_validator_indices(vals, 10) == [0, 1]


def test_committee_params_kat():
    # casper/sharding_test.go:132-169
    assert ref.get_committee_params(64 * 128 // 4) == (1, 4)
    assert ref.get_committee_params(64 * 128) == (1, 1)
    assert ref.get_committee_params(64 * 128 * 8) == (5, 1)


@pytest.mark.parametrize("n,per_slot,size", [(64 * 128, 1, 128), (64 * 128 * 2, 2, 128), (64 * 128 // 2, 1, 64)])
def test_split_by_slot_shard_kat(n, per_slot, size):
    # casper/sharding_test.go:171-255
    arrs = ref.split_by_slot_shard(list(range(n)), 0)
    assert len(arrs) == 64
    for a in arrs:
        assert len(a.array_shard_and_committee) == per_slot
        for sc in a.array_shard_and_committee:
            assert len(sc.committee) == size


def test_split_indices_kat():
    # utils/shuffle_test.go:49-66
    split = ref.split_indices(list(range(64000)), 64)
    assert len(split) == 64 and all(len(s) == 1000 for s in split)


def test_shuffle_kats():
    # utils/shuffle_test.go:11-47 (MaxValidators error; two seeds differ)
    with pytest.raises(ref.GoError):
        ref.shuffle_indices(bytes(32), [0] * (ref.MAX_VALIDATORS + 1))
    h1 = ref.bytes_to_hash(b"abcdefg" * 5)
    h2 = ref.bytes_to_hash(b"1234567" * 5)
    l1 = ref.shuffle_indices(h1, list(range(100)))
    l2 = ref.shuffle_indices(h2, list(range(100)))
    assert l1 != l2
    assert sorted(l1) == list(range(100))


def test_sample_attesters_and_proposers_shape():
    # casper/sharding_test.go:57-130 (1000 and 20 validators -> 64 slots)
    for n in (1000, 20):
        vals = _validators([dict(start_dynasty=1, end_dynasty=100)] * n)
        arrs = ref.shuffle_validators_to_committees(ref.bytes_to_hash(b"A"), vals, 1, 0)
        assert len(arrs) == 64


def test_init_cycle_not_finalized():
    # blockchain/core_test.go:588-616
    active, cs = ref.new_genesis_states()
    cs.last_state_recalc = 64
    nc, na = ref.state_recalc(cs, active, {}, 0)
    assert nc.last_finalized_slot == 0
    assert nc.last_justified_slot == 0
    assert nc.justified_streak == 0
    assert len(na.recent_block_hashes) == 128


def test_init_cycle_finalized():
    # blockchain/core_test.go:619-671
    active, cs = ref.new_genesis_states()
    cs.last_state_recalc = 64
    hashes = [hashlib.blake2b(bytes([i]), digest_size=32).digest() for i in range(64)]
    cache = {h: [[], 100000] for h in hashes}
    del active.recent_block_hashes[:]
    active.recent_block_hashes.extend(hashes)
    nc, na = ref.state_recalc(cs, active, cache, 0)
    del na.recent_block_hashes[:]
    na.recent_block_hashes.extend(hashes)
    nc, na = ref.state_recalc(nc, na, cache, 0)
    assert nc.last_finalized_slot == 63
    assert nc.last_justified_slot == 127
    assert nc.justified_streak == 128
    assert len(na.recent_block_hashes) == 64


def test_process_crosslinks_kat():
    # blockchain/core_test.go:979-1024
    # the test's chain is a genesis chain (1000 validators): slot 0 / shard 0 is its committee
    _, cs = ref.new_genesis_states()
    records = [pb.CrosslinkRecord(dynasty=1, blockhash=b"A", slot=1) for _ in range(ref.SHARD_COUNT)]
    vals = _validators([dict(balance=10000, start_dynasty=0, end_dynasty=ref.DEFAULT_END_DYNASTY)]
                       * (ref.SHARD_COUNT * ref.MIN_COMMITTEE_SIZE))
    atts = [pb.AttestationRecord(slot=0, shard_id=0, shard_block_hash=b"a", attester_bitfield=b"zz")
            for _ in range(100)]
    out = ref.process_crosslinks(cs, records, vals, atts, 5, 50)
    assert out[0].dynasty == 5 and out[0].slot == 50 and out[0].blockhash == b"a"


def test_can_process_attestations_kat():
    # blockchain/core_test.go:406-519 (error cases of processAttestation)
    _, cs = ref.new_genesis_states()
    active = pb.ActiveState()
    with pytest.raises(ref.GoError):
        ref.process_attestation(cs, active, 1, pb.AttestationRecord(slot=2, shard_id=0))
    with pytest.raises(ref.GoError):
        ref.process_attestation(cs, active, 2 + 64, pb.AttestationRecord(slot=1, shard_id=0))
    active.recent_block_hashes.extend([b"X"] * 64)
    cs = pb.CrystallizedState()
    a = cs.shard_and_committees_for_slots.add()
    sc = a.array_shard_and_committee.add()
    sc.shard_id = 1
    sc.committee.extend([0, 1, 2, 3, 4, 5])
    att = pb.AttestationRecord(slot=0, shard_id=0, oblique_parent_hashes=[b"A", b"B", b"C"])
    with pytest.raises(ref.GoError):
        ref.process_attestation(cs, active, 1, att)
    sc.shard_id = 0
    with pytest.raises(ref.GoError):
        ref.process_attestation(cs, active, 0, pb.AttestationRecord(slot=0, shard_id=0, attester_bitfield=b"ABC"))
    with pytest.raises(ref.GoError):
        ref.process_attestation(cs, active, 0, pb.AttestationRecord(slot=0, shard_id=0, attester_bitfield=b"a"))
    ref.process_attestation(cs, active, 0, pb.AttestationRecord(slot=0, shard_id=0, attester_bitfield=b"0"))


def test_genesis_encodings():
    # types/block.go:43-55 -> Timestamp{0,0} encodes as 3a 00; genesis validator = 13 bytes
    assert ref.marshal(ref.new_genesis_block()) == bytes([0x3A, 0x00])
    v = pb.ValidatorRecord(start_dynasty=0, end_dynasty=ref.DEFAULT_END_DYNASTY, balance=32)
    assert ref.marshal(v) == bytes.fromhex("282038ffff9fcfc8e0c8e38a01")
    active, _ = ref.new_genesis_states()
    assert ref.marshal(active) == bytes([0x12, 0x00]) * 128


@pytest.mark.parametrize("bitfield,panics", [(b"\x00\x00", False), (b"zz", True)])
def test_process_crosslinks_shard_index_short_circuit(bitfield, panics):
    # blockchain/core.go:549: `3*vote >= 2*total && dynasty > crosslinkRecords[ShardId].Dynasty`
    # indexes the records only when the 2/3 test holds, so an out-of-range shard panics only then
    _, cs = ref.new_genesis_states()
    vals = _validators([dict(balance=10000, start_dynasty=0, end_dynasty=ref.DEFAULT_END_DYNASTY)] * 1000)
    att = pb.AttestationRecord(slot=0, shard_id=0, shard_block_hash=b"a", attester_bitfield=bitfield)
    if panics:
        with pytest.raises(ref.GoPanic):
            ref.process_crosslinks(cs, [], vals, [att], 5, 50)
    else:
        assert ref.process_crosslinks(cs, [], vals, [att], 5, 50) == []
    # the numpy twin agrees
    from oracle import epoch_np as onp
    vote = np.array([0 if not panics else 1], dtype=np.uint64)
    total = np.array([1], dtype=np.uint64)
    if panics:
        with pytest.raises(ref.GoPanic):
            onp.crosslink_winners(vote, total, np.array([0], np.uint32), np.zeros(0, np.uint64), 5)
    else:
        assert onp.crosslink_winners(vote, total, np.array([0], np.uint32), np.zeros(0, np.uint64), 5).size == 0


def test_c_shuffle_restatement_matches_scalar_oracle():
    # utils/shuffle.go:14-33: the C restatement (the large-n checker and CPU baseline) against
    # the scalar oracle, including the genesis seed Hash{} whose swap numbers contain a 0
    from oracle import cport
    for n in (0, 1, 2, 20, 255, 256, 257, 1000):
        for seed in (ref.bytes_to_hash(b"A"), ref.bytes_to_hash(b""), bytes(range(32))):
            assert cport.shuffle_indices(seed, np.arange(n)).tolist() == ref.shuffle_indices(seed, list(range(n)))


def test_oracle_reload_semantics():
    # blockchain/core.go:59-64,86-95: a reloaded chain has the stored CrystallizedState and the
    # genesis ActiveState; hasBlock answers from the saved blocks, so the next block extends it
    from oracle import replay
    from prysm_amd import synth
    blocks = synth.chain_blocks(1024, 140, seed=2)
    ch = replay.Chain(1024)
    for b in blocks[:70]:
        ch.process_block(replay.to_pb_block(b))
    c2 = replay.Chain.reload(ref.marshal(ch.C), ch.saved)
    assert ref.marshal(c2.C) == ref.marshal(ch.C)
    active, _ = ref.new_genesis_states(1)
    assert ref.marshal(c2.A.data) == ref.marshal(active) and c2.A.cache == {}
    recs, _ = replay.replay_from(c2, blocks[70:])
    assert recs[0]["status"] == "processed"
