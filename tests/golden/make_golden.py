"""Generate tests/golden/*.json from the oracle (run in the build container:
``python tests/golden/make_golden.py``).  The fixtures are data only — inputs and expected
outputs — so the GPU box never needs the oracle's protobuf runtime or /root/reference.

Provenance of the expected values: BLAKE2b-512 = CPython hashlib (RFC 7693 reference C,
pinned by the RFC "abc" vector); proto3 bytes = Google protobuf over oracle/schema.py (pinned
to the descriptor embedded in the reference, oracle/check_schema_vs_reference.py); Go logic =
oracle/ref.py (pinned by every reference KAT, tests/test_oracle_kats.py).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ref  # noqa: E402
from oracle import schema as pb  # noqa: E402


def pattern(n, salt=7):
    return bytes((i * salt + (i >> 3)) & 0xFF for i in range(n))


def blake2b_vectors():
    return {
        "rfc7693_abc": ref.sum512(b"abc").hex(),
        "pattern_lengths": {str(n): ref.sum512(pattern(n)).hex() for n in range(0, 301)},
        "pattern_512": ref.sum512(pattern(512)).hex(),
        "pattern_28395": ref.sum512(pattern(28395)).hex(),
    }


def att(slot, shard, jslot, jbh, sbh, bf, obl, sig):
    return pb.AttestationRecord(slot=slot, shard_id=shard, justified_slot=jslot, justified_block_hash=jbh,
                                shard_block_hash=sbh, attester_bitfield=bf, oblique_parent_hashes=obl,
                                aggregate_sig=sig)


def attestation_vectors():
    cases = [
        att(0, 0, 0, b"", b"", b"", [], []),
        att(0, 0, 0, b"", b"", b"", [b""], []),                     # NewAttestation(nil) shape
        att(5, 3, 0, b"", b"\x00", b"", [], [0, 0]),                 # NewAttestationRecord shape
        att(300, 5, 2, b"J" * 32, b"S" * 32, b"\xff\x80", [b"A", b"B" * 40, b""], [1, 1 << 63]),
        att(1 << 40, 1023, 77, pattern(32), pattern(32, 3), pattern(26, 5),
            [pattern(32, 11) for _ in range(4)], [(1 << 64) - 1]),
    ]
    out = []
    for a in cases:
        enc = a.SerializeToString()
        kb = ref.attestation_key_bytes(a)
        out.append({
            "slot": a.slot, "shard_id": a.shard_id, "justified_slot": a.justified_slot,
            "justified_block_hash": a.justified_block_hash.hex(), "shard_block_hash": a.shard_block_hash.hex(),
            "attester_bitfield": a.attester_bitfield.hex(),
            "oblique_parent_hashes": [h.hex() for h in a.oblique_parent_hashes],
            "aggregate_sig": [str(x) for x in a.aggregate_sig],
            "encoding": enc.hex(), "hash": ref.hash32(enc).hex(),
            "key_bytes": kb.hex(), "key": ref.hash32(kb).hex(),
        })
    return out


def block_vectors():
    g = ref.new_genesis_block()
    b = pb.BeaconBlock(parent_hash=pattern(32), slot_number=9, randao_reveal=b"\x00",
                       pow_chain_ref=b"\x00", active_state_hash=bytes(32), crystallized_state_hash=bytes(32))
    b.timestamp.seconds = 72
    b.attestations.add().CopyFrom(att(8, 2, 0, b"", b"x", b"\xa0", [], []))
    neg = pb.BeaconBlock(slot_number=1)
    neg.timestamp.seconds = -1
    neg.timestamp.nanos = -5
    out = []
    for name, blk in (("genesis", g), ("slot9", b), ("negative_timestamp", neg)):
        enc = blk.SerializeToString()
        out.append({"name": name, "encoding": enc.hex(), "hash": ref.hash32(enc).hex()})
    return out


def genesis_vectors():
    out = {}
    for n in (1000, 1024):
        active, cs = ref.new_genesis_states(n)
        ae, ce = active.SerializeToString(), cs.SerializeToString()
        out[str(n)] = {"active_len": len(ae), "active_hash": ref.hash32(ae).hex(),
                       "crystallized_len": len(ce), "crystallized_hash": ref.hash32(ce).hex(),
                       "committees_slot0": [[sc.shard_id, list(sc.committee)]
                                            for sc in cs.shard_and_committees_for_slots[0].array_shard_and_committee]}
    return out


def shuffle_vectors():
    out = []
    for seed_name, seed in (("Hash{'A'}", b"A" + bytes(31)), ("BytesToHash('A')", ref.bytes_to_hash(b"A")),
                            ("zero", bytes(32))):
        for n in (0, 1, 2, 20, 100, 1000, 1024):
            out.append({"seed_name": seed_name, "seed": seed.hex(), "n": n,
                        "permutation": ref.shuffle_indices(seed, list(range(n)))})
    return out


def reward_vectors():
    rng = np.random.default_rng(40)
    cases = []
    # casper/incentives_test.go:9-43
    cases.append({"name": "incentives_test", "start": [1] * 40, "end": [10] * 40, "balance": [32] * 40,
                  "dynasty": 1, "total_deposit": 100, "bitfields": [bytes([200, 148, 146, 179, 49]).hex()]})
    for k in range(3):
        n = int(rng.integers(50, 400))
        start = rng.integers(0, 3, size=n).tolist()
        end = rng.integers(1, 5, size=n).tolist()
        bal = rng.integers(0, 40, size=n).tolist()
        bfs = [rng.integers(0, 256, size=int(rng.integers(1, 9)), dtype=np.uint8).tobytes().hex() for _ in range(3)]
        bfs.append(rng.integers(0, 256, size=(n + 7) // 8, dtype=np.uint8).tobytes().hex())
        cases.append({"name": "random%d" % k, "start": start, "end": end, "balance": bal, "dynasty": 2,
                      "total_deposit": [1, sum(bal), 1 << 63][k], "bitfields": bfs})
    for c in cases:
        vals = [pb.ValidatorRecord(start_dynasty=s, end_dynasty=e, balance=b)
                for s, e, b in zip(c["start"], c["end"], c["balance"])]
        atts = [pb.AttestationRecord(attester_bitfield=bytes.fromhex(h)) for h in c["bitfields"]]
        c["attesters_total_deposit"] = ref.get_attesters_total_deposit(atts)
        c["active"] = ref.active_validator_indices(vals, c["dynasty"])
        c["exited"] = ref.exited_validator_indices(vals, c["dynasty"])
        c["queued"] = ref.queued_validator_indices(vals, c["dynasty"])
        ref.calculate_rewards(atts, vals, c["dynasty"], c["total_deposit"])
        c["balance_after"] = [v.balance for v in vals]
        c["next_cycle_balance"] = sum(vals[i].balance for i in ref.active_validator_indices(vals, c["dynasty"])) & ref.M64
    return cases


def replay_vectors(nval=1024, nblocks=130, seed=1):
    """oracle/replay.py over prysm_amd.synth.chain_blocks (input generation: numpy + hashlib)."""
    import hashlib

    from oracle import replay
    from prysm_amd import synth
    blocks = synth.chain_blocks(nval, nblocks, seed=seed)
    pbs = [replay.to_pb_block(b) for b in blocks]
    recs, roots = replay.replay(blocks, nval)
    h = hashlib.sha256(b"".join(b.SerializeToString() for b in pbs)).hexdigest()
    out = {"nval": nval, "nblocks": nblocks, "seed": seed, "blocks_sha256": h,
           "records": [{"hash": r["hash"].hex(), "status": r["status"], "transition": r["transition"],
                        "atts": [{k: (v.hex() if isinstance(v, bytes) else v) for k, v in a.items()} for a in r["atts"]]}
                       for r in recs],
           "roots": {k: v.hex() for k, v in roots.items() if isinstance(v, bytes)},
           "vote_totals": {k.hex(): v for k, v in sorted(roots["vote_totals"].items())}}
    try:  # the same generator with full participation: CalculateRewards panics
        replay.replay(synth.chain_blocks(nval, 70, seed=seed, participation=(1.0,)), nval)
        out["full_participation_panics_at"] = None
    except ref.GoPanic as e:
        out["full_participation_panics_at"] = str(e)
    return out


def main():
    fixtures = {
        "replay_n1024.json": replay_vectors(),
        "blake2b.json": blake2b_vectors(),
        "attestations.json": attestation_vectors(),
        "blocks.json": block_vectors(),
        "genesis.json": genesis_vectors(),
        "shuffle.json": shuffle_vectors(),
        "rewards.json": reward_vectors(),
    }
    for name, data in fixtures.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, separators=(",", ":"))
        print("wrote", name, os.path.getsize(os.path.join(HERE, name)), "bytes")


if __name__ == "__main__":
    main()
