"""Block pipeline parity (BASELINE configs[0] and the per-block work of configs[4]): the
GPU-batched ``prysm_amd.blockchain.BeaconChain`` vs the oracle's restatement of
``ChainService.blockProcessing`` (oracle/replay.py), bit-exact on every block digest,
attestation Hash/Key, 64-byte message digest, vote-cache total and final state root.

CPU: the oracle reproduces the committed fixture (tests/golden/replay_n1024.json, written by
tests/golden/make_golden.py) and the generator still produces the same blocks.
GPU: the product reproduces the fixture, a live oracle run at 65,536 validators (5
committees per block, 64 signed parent hashes each), and the reference's panic.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from prysm_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))


def golden():
    with open(os.path.join(HERE, "golden", "replay_n1024.json")) as f:
        return json.load(f)


def _hexrecs(recs):
    return [{"hash": r["hash"].hex(), "status": r["status"], "transition": r["transition"],
             "atts": [{k: (v.hex() if isinstance(v, bytes) else v) for k, v in a.items()} for a in r["atts"]]}
            for r in recs]


def _compare(recs, roots, g):
    got = _hexrecs(recs)
    assert len(got) == len(g["records"])
    for i, (a, b) in enumerate(zip(got, g["records"])):
        assert a == b, "block %d differs" % (i + 1)
    for k, v in g["roots"].items():
        assert roots[k].hex() == v, k
    assert {k.hex(): v for k, v in roots["vote_totals"].items()} == g["vote_totals"]


def test_generator_is_pinned():
    from oracle import replay
    g = golden()
    blocks = synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"])
    h = hashlib.sha256(b"".join(replay.to_pb_block(b).SerializeToString() for b in blocks)).hexdigest()
    assert h == g["blocks_sha256"]


def test_oracle_replay_matches_golden():
    from oracle import replay
    g = golden()
    recs, roots = replay.replay(synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"]), g["nval"])
    _compare(recs, roots, g)
    assert sum(r["transition"] for r in recs) == 2 and all(r["status"] == "processed" for r in recs)


def _product(nval, blocks, **opts):
    from prysm_amd.blockchain import BeaconChain
    ch = BeaconChain(nval, **opts)
    recs = ch.process_blocks(blocks)
    return recs, ch.roots()


@pytest.mark.gpu
def test_gpu_replay_matches_golden():
    g = golden()
    recs, roots = _product(g["nval"], synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"]))
    _compare(recs, roots, g)


@pytest.mark.gpu
@pytest.mark.parametrize("serial", ["host", "gpu"])
def test_gpu_replay_golden_roots_both_serial_routes(serial):
    """State roots are single long messages: hashed on host threads at or above the serial
    threshold, on one GPU lane below it.  Both routes reproduce the fixture's roots."""
    from prysm_amd import _lib
    g = golden()
    thr = 1000 if serial == "host" else _lib.SERIAL_ON_GPU
    with _lib.serial_threshold(thr):
        recs, roots = _product(g["nval"], synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"]))
    _compare(recs, roots, g)


@pytest.mark.gpu
def test_gpu_replay_in_two_batches_matches_golden():
    """Blocks fed in two batches (deferred work flushed between calls) give the same result."""
    from prysm_amd.blockchain import BeaconChain
    g = golden()
    blocks = synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"])
    ch = BeaconChain(g["nval"])
    recs = ch.process_blocks(blocks[:70]) + ch.process_blocks(blocks[70:])
    _compare(recs, ch.roots(), g)


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", ["ones", "mixed"])
def test_gpu_replay_block_by_block_matches_golden(sizes):
    """Many calls (one block each, or 1-9 blocks): every call reuses the engine's pinned arena,
    so the pending attestations that outlive a call are moved out of it and must stay valid
    across later calls, transitions and the deferred epoch (chain.hip keep_arenas)."""
    from prysm_amd.blockchain import BeaconChain
    g = golden()
    blocks = synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"])
    ch = BeaconChain(g["nval"])
    rng = np.random.default_rng(5)
    recs, i = [], 0
    while i < len(blocks):
        k = 1 if sizes == "ones" else int(rng.integers(1, 10))
        recs += ch.process_blocks(blocks[i:i + k])
        i += k
    _compare(recs, ch.roots(), g)


@pytest.mark.gpu
def test_gpu_replay_many_calls_equal_one_call_65536():
    """configs[4]'s shape over 400 blocks: the chain fed in calls of 1-40 blocks (several
    transitions inside and across calls) equals the chain fed in one call, record for record,
    with the same state roots and vote totals."""
    from prysm_amd.blockchain import BeaconChain, serialize_blocks
    nval = 65536
    blocks = synth.chain_blocks(nval, 400, seed=9)
    one = BeaconChain(nval)
    d, o = serialize_blocks(blocks)
    br1, ar1 = one.process_serialized(d, o)
    many = BeaconChain(nval)
    rng = np.random.default_rng(2)
    brs, ars, i = [], [], 0
    while i < len(blocks):
        k = int(rng.integers(1, 41))
        d, o = serialize_blocks(blocks[i:i + k])
        br, ar = many.process_serialized(d, o)
        br = br.copy()
        br["first_att"] += sum(len(a) for a in ars)
        brs.append(br)
        ars.append(ar.copy())
        i += k
    np.testing.assert_array_equal(np.concatenate(brs), br1)
    np.testing.assert_array_equal(np.concatenate(ars), ar1)
    assert many.roots() == one.roots()


@pytest.mark.gpu
@pytest.mark.parametrize("batch", ["1", "37", "5000"])
def test_gpu_replay_message_batches_equal_one_batch(batch):
    """pz_chain_options.msg_batch > 0 digests the processAttestation messages in batches sent after the
    transitions, on their own stream, while the walk goes on (chain.hip msg_send): every
    message digest, record and root equals the one-batch call's, over a chain fed in one call
    and in calls of 1-60 blocks."""
    from prysm_amd.blockchain import BeaconChain, serialize_blocks
    nval = 65536
    blocks = synth.chain_blocks(nval, 400, seed=9)
    d, o = serialize_blocks(blocks)
    one = BeaconChain(nval)
    br1, ar1 = one.process_serialized(d, o)
    two = BeaconChain(nval, msg_batch=int(batch))
    br2, ar2 = two.process_serialized(d, o)
    np.testing.assert_array_equal(br2, br1)
    np.testing.assert_array_equal(ar2, ar1)
    assert two.roots() == one.roots()
    many = BeaconChain(nval, msg_batch=int(batch))
    rng = np.random.default_rng(4)
    ars, i = [], 0
    while i < len(blocks):
        k = int(rng.integers(1, 61))
        d, o = serialize_blocks(blocks[i:i + k])
        ars.append(many.process_serialized(d, o)[1].copy())
        i += k
    np.testing.assert_array_equal(np.concatenate(ars), ar1)
    assert many.roots() == one.roots()


@pytest.mark.gpu
def test_gpu_replay_vs_live_oracle_65536():
    from oracle import replay
    nval = 65536
    blocks = synth.chain_blocks(nval, 70, seed=6)
    o_recs, o_roots = replay.replay(blocks, nval)
    recs, roots = _product(nval, blocks)
    assert _hexrecs(recs) == _hexrecs(o_recs)
    for k in ("chain_active", "chain_crystallized", "cand_active", "cand_crystallized"):
        assert roots[k] == o_roots[k], k
    assert roots["vote_totals"] == o_roots["vote_totals"]
    assert sum(len(r["atts"]) for r in recs) == 70 * 5


def _relink(blocks):
    """Recompute parent digests after editing blocks (as the generator does)."""
    from prysm_amd import pb, wire
    parent = hashlib.blake2b(wire.beacon_block(pb.BeaconBlock(timestamp=pb.Timestamp())), digest_size=64).digest()[:32]
    for b in blocks:
        b.parent_hash = parent
        parent = hashlib.blake2b(wire.beacon_block(b), digest_size=64).digest()[:32]
    return blocks


def edited_chain():
    """1,000 validators (15- and 16-member committees, so trailing bitfield bits exist) with
    invalid attestations mixed into valid blocks: canProcessAttestations follows the LAST
    attestation (service.go:281-301), the vote cache still tallies every attestation of a
    processed block (service.go:313-318), and a rejected block orphans its descendants."""
    import dataclasses
    blocks = synth.chain_blocks(1000, 24, seed=3)

    def bad(k, **kw):
        return dataclasses.replace(blocks[k].attestations[0], **kw)

    v = blocks[2].attestations[0]
    blocks[2].attestations = [bad(2, attester_bitfield=v.attester_bitfield + b"\x00"), v]
    v = blocks[5].attestations[0]
    blocks[5].attestations = [bad(5, attester_bitfield=v.attester_bitfield[:-1] + bytes([v.attester_bitfield[-1] | 1])), v]
    v = blocks[8].attestations[0]
    blocks[8].attestations = [v, bad(8, shard_id=999), v]
    v = blocks[11].attestations[0]
    blocks[11].attestations = [bad(11, justified_slot=7), v]
    v = blocks[14].attestations[0]
    blocks[14].attestations = [bad(14, oblique_parent_hashes=[b"\x05" * 5]), v]
    v = blocks[19].attestations[0]
    blocks[19].attestations = [v, bad(19, justified_slot=7)]
    return _relink(blocks)


def test_oracle_edited_chain_statuses():
    from oracle import replay
    recs, _ = replay.replay(edited_chain(), 1000)
    st = [r["status"] for r in recs]
    assert st[:19] == ["processed"] * 19 and st[19] == "attestations_rejected" and set(st[20:]) == {"no_parent"}
    errs = [a["error"] for r in recs for a in r["atts"] if "error" in a]
    assert len(errs) == 5


def shaped_message_chain():
    """processAttestation messages of every shape the device gather handles: ShardBlockHash of
    0-300 bytes (not a multiple of 4, crossing a 128-byte block edge) and 0-3 oblique parent
    hashes, full (32 B, logged ids) and short (7 B, zero-padded unvotable ids)."""
    import dataclasses
    blocks = synth.chain_blocks(1024, 40, seed=8)
    rng = np.random.default_rng(8)
    sb_lens = [0, 1, 3, 5, 31, 33, 100, 300]
    for bi, b in enumerate(blocks):
        atts = []
        for j, a in enumerate(b.attestations):
            sb = rng.integers(0, 256, sb_lens[(bi + j) % len(sb_lens)], dtype=np.uint8).tobytes()
            obl = [rng.integers(0, 256, 32 if q % 2 == 0 else 7, dtype=np.uint8).tobytes() for q in range((bi + 2 * j) % 4)]
            atts.append(dataclasses.replace(a, shard_block_hash=sb, oblique_parent_hashes=obl))
        b.attestations = atts
    return _relink(blocks)


def test_oracle_shaped_message_chain_processes():
    from oracle import replay
    recs, _ = replay.replay(shaped_message_chain(), 1024)
    assert all(r["status"] == "processed" for r in recs)
    assert all("error" not in a for r in recs for a in r["atts"])


@pytest.mark.gpu
@pytest.mark.parametrize("batch", ["0", "3"])
def test_gpu_replay_shaped_messages_vs_oracle(batch):
    from oracle import replay
    blocks = shaped_message_chain()
    o_recs, o_roots = replay.replay(blocks, 1024)
    recs, roots = _product(1024, blocks, msg_batch=int(batch))
    assert _hexrecs(recs) == _hexrecs(o_recs)
    for k in ("chain_active", "chain_crystallized", "cand_active", "cand_crystallized"):
        assert roots[k] == o_roots[k], k


def future_slot_chain():
    """An attestation from a future slot is rejected by processAttestation, but the vote
    cache loop still slices RecentBlockHashes with the wrapped start index: the reference
    panics (core.go:353)."""
    import dataclasses
    blocks = synth.chain_blocks(1024, 8, seed=4)
    v = blocks[5].attestations[0]
    blocks[5].attestations = [dataclasses.replace(v, slot=100), v]
    return _relink(blocks)


def test_oracle_future_slot_panics():
    from oracle import ref, replay
    with pytest.raises(ref.GoPanic):
        replay.replay(future_slot_chain(), 1024)


@pytest.mark.gpu
def test_gpu_future_slot_panics():
    from prysm_amd.blockchain import BeaconChain, ChainPanic
    with pytest.raises(ChainPanic):
        BeaconChain(1024).process_blocks(future_slot_chain())


@pytest.mark.gpu
def test_gpu_replay_rejections_and_missing_parents():
    from oracle import replay
    blocks = edited_chain()
    o_recs, o_roots = replay.replay(blocks, 1000)
    recs, roots = _product(1000, blocks)
    strip = lambda rs: [{**r, "atts": [a if "error" not in a else {"error": True} for a in r["atts"]]} for r in rs]  # noqa: E731
    assert strip(_hexrecs(recs)) == strip(_hexrecs(o_recs))
    for k in ("chain_active", "chain_crystallized", "cand_active", "cand_crystallized"):
        assert roots[k] == o_roots[k], k
    assert roots["vote_totals"] == o_roots["vote_totals"]


@pytest.mark.gpu
def test_gpu_replay_reproduces_reward_panic():
    from prysm_amd.blockchain import BeaconChain, ChainPanic
    g = golden()
    assert g["full_participation_panics_at"]
    ch = BeaconChain(g["nval"])
    # the deferred epoch is collected at the end of the call (block 69): the panic names the
    # transition's block and slot, after which the call's result rows are undefined
    with pytest.raises(ChainPanic, match=r"CalculateRewards.*stateRecalc of block \d+ of this call, slot 64"):
        ch.process_blocks(synth.chain_blocks(g["nval"], 70, seed=g["seed"], participation=(1.0,)))


def test_generator_shape():
    blocks = synth.chain_blocks(65536, 3, seed=6)
    assert [len(b.attestations) for b in blocks] == [5, 5, 5]
    k = [len(a.attester_bitfield) for a in blocks[0].attestations]
    assert k == [26, 26, 26, 26, 26]
    assert all(len(a.oblique_parent_hashes) == 1 for a in blocks[0].attestations)
    bf = np.frombuffer(blocks[0].attestations[0].attester_bitfield, np.uint8)
    assert bf[-1] & 0x0F == 0  # 204 members: the last 4 bits are padding


@pytest.mark.gpu
def test_gpu_state_bytes_match_oracle_encoding():
    """The persistence format (PersistActiveState / PersistCrystallizedState, core.go:161-177):
    the engine's state encodings are byte-identical to the protobuf runtime's marshal of the
    oracle's states, after genesis and after two cycle transitions, and they hash to the
    roots."""
    from oracle import ref
    from oracle import replay as oreplay
    from prysm_amd.blockchain import BeaconChain
    nval = 1024
    ch = BeaconChain(nval)
    _, _, ob = oreplay.replay([], nval, with_state_bytes=True)
    for k in ("chain_active", "chain_crystallized"):
        assert ch.state_bytes(k) == ob[k], k
    assert ch.state_bytes("cand_active") is None
    blocks = synth.chain_blocks(nval, 130, seed=1)
    ch.process_blocks(blocks)
    _, oroots, ob = oreplay.replay(blocks, nval, with_state_bytes=True)
    roots = ch.roots()
    for k in BeaconChain.STATES:
        b = ch.state_bytes(k)
        assert b == ob[k], k
        assert ref.hash32(b) == roots[k] == oroots[k], k


@pytest.mark.gpu
@pytest.mark.parametrize("nval", [32, 40])
def test_gpu_replay_empty_committees_vs_oracle(nval):
    """Fewer than 64 validators: splitBySlotShard leaves the slot-0 committee empty, so every
    pending attestation carries a zero-length bitfield (BitLength(0), core.go:377-394) and
    names an empty committee, whose 3*0 >= 2*0 qualifies it for the crosslink (core.go:549).
    No bitfield has a byte at the transitions, so the winner reset must not depend on the
    popcount pass finding any."""
    from oracle import replay
    blocks = synth.chain_blocks(nval, 130, seed=5)
    assert all(len(a.attester_bitfield) == 0 for b in blocks for a in b.attestations)
    o_recs, o_roots = replay.replay(blocks, nval)
    recs, roots = _product(nval, blocks)
    assert _hexrecs(recs) == _hexrecs(o_recs)
    assert sum(r["transition"] for r in recs) == 2
    for k in ("chain_active", "chain_crystallized", "cand_active", "cand_crystallized"):
        assert roots[k] == o_roots[k], k


@pytest.mark.gpu
def test_gpu_replay_configs4_full_chain_vs_c_port():
    """BASELINE configs[4] at full size: the 10,000-block, 156-transition chain of the bench
    (65,536 validators, seed 6) through the GPU engine and through the C restatement of the
    block pipeline (oracle/c/replay_ref.c, checker mode): every block digest, status and
    transition, every attestation status class, Key, Hash and message digest, the four state
    roots and every vote-cache total."""
    from prysm_amd.blockchain import BeaconChain, serialize_blocks
    from replay_port_helpers import mismatches, port_replay
    nval = 65536
    blocks = synth.chain_blocks(nval, 10000, seed=6)
    data, offs = serialize_blocks(blocks)
    ch = BeaconChain(nval)
    br, ar = ch.process_serialized(data, offs)
    assert int(br["transition"].sum()) == 156
    out, port_roots = port_replay(data, offs, nval, len(ar))
    assert mismatches(br, ar, ch.roots(), out, port_roots) == []


def _saved_from(recs):
    return [r["hash"] for r in recs if r["status"] in ("processed", "saved_not_candidate")]


@pytest.mark.gpu
@pytest.mark.parametrize("nval,k,total", [(1024, 129, 200), (1000, 70, 140), (65536, 65, 140)])
def test_gpu_resume_from_persisted_state_vs_oracle(nval, k, total):
    """f3 read side: NewBeaconChain over a database holding a CrystallizedState
    (blockchain/core.go:86-95).  The GPU chain runs k blocks; the persisted encoding of its
    CrystallizedState (what updateHead stores, core.go:170-177) and the saved block hashes
    seed a reloaded chain (genesis ActiveState, as the reference reloads), which runs the
    remaining blocks.  The oracle does the same from the same bytes; every record and root
    must agree."""
    from oracle import replay
    from prysm_amd.blockchain import BeaconChain
    blocks = synth.chain_blocks(nval, total, seed=11)
    ch = BeaconChain(nval)
    recs = ch.process_blocks(blocks[:k])
    cs_bytes = ch.state_bytes("chain_crystallized")
    saved = _saved_from(recs)
    o_chain = replay.Chain(nval)
    o_recs = [o_chain.process_block(replay.to_pb_block(b)) for b in blocks[:k]]
    assert _hexrecs(recs) == _hexrecs(o_recs) and set(saved) == o_chain.saved
    from oracle import ref
    assert cs_bytes == ref.marshal(o_chain.C)
    ch2 = BeaconChain.from_state(cs_bytes, saved)
    assert ch2.state_bytes("chain_crystallized") == cs_bytes
    recs2 = ch2.process_blocks(blocks[k:])
    o2 = replay.Chain.reload(cs_bytes, saved)
    o_recs2, o_roots2 = replay.replay_from(o2, blocks[k:])
    assert _hexrecs(recs2) == _hexrecs(o_recs2)
    assert sum(r["transition"] for r in recs2) >= 1
    roots2 = ch2.roots()
    for key in ("chain_active", "chain_crystallized", "cand_active", "cand_crystallized"):
        assert roots2[key] == o_roots2[key], key
    assert roots2["vote_totals"] == o_roots2["vote_totals"]


@pytest.mark.gpu
def test_gpu_reload_general_state_encoding():
    """A stored state with every ValidatorRecord field set (public key, withdrawal shard and
    address, RANDAO commitment), a dynasty seed, non-genesis crosslinks and committees: the
    reloaded chain re-encodes exactly the canonical bytes and hashes them like the oracle."""
    from oracle import ref
    from oracle import schema as pb
    _, cs = ref.new_genesis_states(1000)
    for i, v in enumerate(cs.validators):
        v.public_key = (i * 7919) % 1000 + 1
        v.withdrawal_shard = i % 3
        v.withdrawal_address = bytes([i & 0xFF]) * (i % 21)
        v.randao_commitment = bytes([(i * 3) & 0xFF]) * (i % 33)
        v.balance = 30 + i % 5
    cs.dynasty_seed = b"\x07" * 32
    cs.dynasty_seed_last_reset = 5
    cs.crosslink_records[3].CopyFrom(pb.CrosslinkRecord(dynasty=2, blockhash=b"\x09" * 32, slot=64))
    cs.last_state_recalc = 64
    cs.current_dynasty = 3
    b = ref.marshal(cs)
    from prysm_amd.blockchain import BeaconChain
    ch = BeaconChain.from_state(b, [])
    assert ch.state_bytes("chain_crystallized") == b
    assert ch.roots()["chain_crystallized"] == ref.crystallized_state_hash(cs)
    active, _ = ref.new_genesis_states(1)
    assert ch.roots()["chain_active"] == ref.active_state_hash(active)


@pytest.mark.gpu
def test_gpu_reload_rejects_undecodable_state():
    from prysm_amd import _lib
    from prysm_amd.blockchain import BeaconChain
    with pytest.raises(_lib.PzError) as ei:
        BeaconChain.from_state(b"\x0a\xff", [])
    assert ei.value.code == _lib.PZ_EINVAL


# ---- one chain over a communicator (the vote cache and the epoch sharded
# by validator range; on the one-GPU test box over the loopback communicator, every rank on
# cuda:0 with the same code RCCL drives) ---------------------------------------------------------
def _sharded(nval, blocks, world):
    from prysm_amd.blockchain import BeaconChain
    from prysm_amd.native import Comm
    comm = Comm.devices(1) if world == "rccl1" else Comm.loopback(world)
    ch = BeaconChain(nval, comm=comm)
    recs = ch.process_blocks(blocks)
    return recs, ch.roots()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3, 8, "rccl1"])
def test_gpu_sharded_chain_matches_golden(world):
    g = golden()
    recs, roots = _sharded(g["nval"], synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"]), world)
    _compare(recs, roots, g)


@pytest.mark.gpu
@pytest.mark.parametrize("ndev", [2, 8])
def test_gpu_sharded_chain_multi_device_matches_golden(ndev):
    """The golden chain over RCCL across ``ndev`` real GPUs of one process (pz_init_devices:
    each rank's device state, pinned queue mappings and streams on its own device); skipped
    where fewer GPUs are visible (the one-GPU test boxes; the 8-GPU node runs it)."""
    import torch
    if torch.cuda.device_count() < ndev:
        pytest.skip("needs %d GPUs" % ndev)
    from prysm_amd.blockchain import BeaconChain
    from prysm_amd.native import Comm
    g = golden()
    ch = BeaconChain(g["nval"], comm=Comm.devices(ndev))
    recs = ch.process_blocks(synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"]))
    _compare(recs, ch.roots(), g)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_sharded_chain_rejections_vs_oracle(world):
    from oracle import replay
    blocks = edited_chain()
    o_recs, o_roots = replay.replay(blocks, 1000)
    recs, roots = _sharded(1000, blocks, world)
    strip = lambda rs: [{**r, "atts": [a if "error" not in a else {"error": True} for a in r["atts"]]} for r in rs]  # noqa: E731
    assert strip(_hexrecs(recs)) == strip(_hexrecs(o_recs))
    for k in ("chain_active", "chain_crystallized", "cand_active", "cand_crystallized"):
        assert roots[k] == o_roots[k], k
    assert roots["vote_totals"] == o_roots["vote_totals"]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_sharded_chain_one_collective_per_transition(world):
    """The sharded transition's single collective: the justification totals, the
    epoch's partial sums and the previous epoch's next-cycle partial ride in ONE all-reduce, and
    the call's final flush carries the last next-cycle partial -- transitions + 1 collectives per
    call, two calls in a row (the pending partial crossing the call boundary), each matching
    the golden roots."""
    from prysm_amd.blockchain import BeaconChain
    from prysm_amd.native import Comm
    g = golden()
    blocks = synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"])
    comm = Comm.loopback(world)
    ch = BeaconChain(g["nval"], comm=comm)
    comm.set_timing(True)
    comm.collective_time()
    recs = ch.process_blocks(blocks[:70])
    _, n1 = comm.collective_time()
    recs += ch.process_blocks(blocks[70:])
    _, n2 = comm.collective_time()
    comm.set_timing(False)
    t1 = sum(r["transition"] for r in recs[:70])
    t2 = sum(r["transition"] for r in recs[70:])
    assert t1 + t2 == 2
    assert (n1, n2) == (t1 + 1, t2 + 1), (n1, n2, t1, t2)
    _compare(recs, ch.roots(), g)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_sharded_chain_reward_panic(world):
    from prysm_amd.blockchain import BeaconChain, ChainPanic
    from prysm_amd.native import Comm
    g = golden()
    ch = BeaconChain(g["nval"], comm=Comm.loopback(world))
    with pytest.raises(ChainPanic):
        ch.process_blocks(synth.chain_blocks(g["nval"], 70, seed=g["seed"], participation=(1.0,)))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_sharded_chain_configs4_full_vs_c_port(world):
    """BASELINE configs[4] as ONE chain over `world` ranks: the 10,000-block, 156-transition
    chain at 65,536 validators, every block, attestation, root and vote-cache total bit-exact
    against the C restatement of the block pipeline."""
    from prysm_amd.blockchain import BeaconChain, serialize_blocks
    from prysm_amd.native import Comm
    from replay_port_helpers import mismatches, port_replay
    nval = 65536
    blocks = synth.chain_blocks(nval, 10000, seed=6)
    data, offs = serialize_blocks(blocks)
    ch = BeaconChain(nval, comm=Comm.loopback(world))
    br, ar = ch.process_serialized(data, offs)
    assert int(br["transition"].sum()) == 156
    out, port_roots = port_replay(data, offs, nval, len(ar))
    assert mismatches(br, ar, ch.roots(), out, port_roots) == []


@pytest.mark.gpu
@pytest.mark.parametrize("groups", ["1", "0"])
@pytest.mark.parametrize("nval,ncomm", [(131072, 9), (262144, 17), (524288, 33)])
def test_gpu_replay_wide_committees_vs_c_port(nval, ncomm, groups):
    """Larger validator sets than configs[4]: 9, 17 and 33 slot-0 committees per block, each a
    group of the grouped tally (votes.h kVoteMaxGroups), of up to 249 members (every bitfield
    inline in the 64-B record), over 130 blocks (two transitions) against the C restatement;
    groups 0 runs the per-attestation form over the same chains (pz_chain_options.tally_forms)."""
    from prysm_amd import _lib
    from prysm_amd.blockchain import BeaconChain, serialize_blocks
    from replay_port_helpers import mismatches, port_replay
    sizes = synth.genesis_committee_sizes(nval)
    assert len(sizes) == ncomm and max(k for _, k in sizes) <= 256
    blocks = synth.chain_blocks(nval, 130, seed=11)
    data, offs = serialize_blocks(blocks)
    ch = BeaconChain(nval, tally_forms=0 if groups == "1" else _lib.TALLY_PER_ATTESTATION)
    br, ar = ch.process_serialized(data, offs)
    assert int(br["transition"].sum()) == 2
    out, port_roots = port_replay(data, offs, nval, len(ar))
    assert mismatches(br, ar, ch.roots(), out, port_roots) == []


def _vote_queue_chain(**opts):
    """2,000 blocks of the configs[4] chain in two calls (31 transitions, the two queues
    alternating, carried over a call boundary) against the C restatement."""
    from prysm_amd.blockchain import BeaconChain, serialize_blocks
    from replay_port_helpers import mismatches, port_replay
    nval = 65536
    blocks = synth.chain_blocks(nval, 2000, seed=6)
    data, offs = serialize_blocks(blocks)
    ch = BeaconChain(nval, **opts)
    br, ar = ch.process_serialized(data[: int(offs[1000])], offs[:1001])  # two calls: the queues
    br2, ar2 = ch.process_serialized(data, offs[1000:])                     # carry over a call
    br, ar = np.concatenate([br, br2]), np.concatenate([ar, ar2])
    out, port_roots = port_replay(data, offs, nval, len(ar))
    assert mismatches(br, ar, ch.roots(), out, port_roots) == []


@pytest.mark.gpu
@pytest.mark.parametrize("forms", [0, 1, 2, 4, 7])
def test_gpu_replay_vote_queue_forms_vs_c_port(forms):
    """Every record form of the vote queue (votes.h VoteRec: the bitfield inline or in the row
    array, TALLY_BITS_ROWS; the parents' ids as a run or an explicit row, TALLY_ID_ROWS) and both
    tally forms (grouped by committee -- the product when every record is a run with its
    bitfield inline --, or per attestation: TALLY_PER_ATTESTATION or any other form), forced by
    pz_chain_options.tally_forms, over the configs[4] chain against the C restatement."""
    _vote_queue_chain(tally_forms=forms)


@pytest.mark.gpu
@pytest.mark.ab
@pytest.mark.parametrize("path,epack,prep", [("segments", "copy", ""), ("packed", "copy", ""), ("direct", "direct", ""),
                                             ("direct", "direct", "merged"), ("direct", "copy", "merged")])
def test_ab_replay_vote_queue_paths_vs_c_port(path, epack, prep, monkeypatch):
    """The A/B library's measured-and-dropped ways a flush reaches the device (PZ_VOTE_PATH: the
    queue's arrays staged by one multi-segment copy, or round 3's packed arena), the
    transitions' epoch kernels reading their inputs in place (PZ_EPOCH_PACK=direct), and the
    stateRecalc's tally and epoch count blocks in one grid (PZ_EPOCH_PREP=merged:
    pz_vote_words_count_kernel)."""
    monkeypatch.setenv("PZ_VOTE_PATH", path)
    monkeypatch.setenv("PZ_EPOCH_PACK", epack)
    monkeypatch.setenv("PZ_EPOCH_PREP", prep)
    _vote_queue_chain()


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", ["0", pytest.param("1", marks=pytest.mark.ab)])
def test_gpu_malformed_block_ends_the_call_there(pipeline, monkeypatch):
    """A block that is not a canonical encoding ends the call there with PZ_EINVAL, the blocks
    before it processed (as the reference's sync service handles each block as it arrives), in
    the batch path and in the pipelined one (PZ_CHAIN_PIPELINE=1: calls of >= 1,024 blocks parse
    and hash a chunk ahead of the walk).  The chain is then exactly the chain of those blocks."""
    monkeypatch.setenv("PZ_CHAIN_PIPELINE", pipeline)
    from prysm_amd import _lib
    from prysm_amd.blockchain import BeaconChain, serialize_blocks
    blocks = synth.chain_blocks(1024, 1100, seed=3)
    data, offs = serialize_blocks(blocks)
    bad = 1050
    chunks = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in range(len(blocks))]
    chunks[bad] = b"\x10\x00" + chunks[bad]  # a zero scalar Marshal would omit: not canonical
    raw = b"".join(chunks)
    o2 = np.zeros(len(chunks) + 1, dtype=np.uint64)
    o2[1:] = np.cumsum([len(c) for c in chunks])
    ch = BeaconChain(1024)
    with pytest.raises(_lib.PzError) as e:
        ch.process_serialized(np.frombuffer(raw, dtype=np.uint8), o2)
    assert e.value.code == _lib.PZ_EINVAL and ("block %d " % bad) in str(e.value)
    ref = BeaconChain(1024)
    ref.process_serialized(*serialize_blocks(blocks[:bad]))
    assert ch.roots() == ref.roots()


@pytest.mark.gpu
def test_gpu_chain_options_fixed_after_first_call():
    """pz_chain_set_options: the tally forms shape the vote queue's records, so once
    a call has queued some, another form fails with PZ_EINVAL and the chain keeps its form (its
    next call still matches the C restatement); msg_batch may still change."""
    import ctypes

    from prysm_amd import _lib
    from prysm_amd.blockchain import BeaconChain, serialize_blocks
    from replay_port_helpers import mismatches, port_replay
    nval = 4096
    blocks = synth.chain_blocks(nval, 140, seed=3)
    data, offs = serialize_blocks(blocks)
    ch = BeaconChain(nval)
    br0, ar0 = ch.process_serialized(data[: int(offs[70])], offs[:71])
    with pytest.raises(_lib.PzError) as ei:
        _lib.lib.call("pz_chain_set_options", ch._h, ctypes.byref(_lib.ChainOptions(0, _lib.TALLY_BITS_ROWS)))
    assert ei.value.code == _lib.PZ_EINVAL
    _lib.lib.call("pz_chain_set_options", ch._h, ctypes.byref(_lib.ChainOptions(16, 0)))
    br1, ar1 = ch.process_serialized(data, offs[70:])
    br, ar = np.concatenate([br0, br1]), np.concatenate([ar0, ar1])
    out, port_roots = port_replay(data, offs, nval, len(ar))
    assert mismatches(br, ar, ch.roots(), out, port_roots) == []
