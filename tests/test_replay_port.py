"""The C restatement of the block pipeline (oracle/c/replay_ref.c: Go's data layout and
algorithms, the replay leg's CPU baseline and a whole-chain checker) against the scalar oracle
(oracle/replay.py) and the committed fixture.  CPU only."""
import json
import os

import numpy as np
import pytest

from oracle import cport
from oracle import replay as oreplay
from prysm_amd import synth
from prysm_amd.blockchain import serialize_blocks

from test_replay import edited_chain, future_slot_chain

HERE = os.path.dirname(os.path.abspath(__file__))


def _port(blocks, nval, bitmap=False):
    data, offs = serialize_blocks(blocks)
    r = cport.Replay(nval, bitmap_dedup=bitmap)
    try:
        out = r.process(data, offs, sum(len(b.attestations) for b in blocks))
        return out, r.roots()
    finally:
        r.close()


def _compare(blocks, nval, bitmap=False):
    out, roots = _port(blocks, nval, bitmap)
    recs, o_roots = oreplay.replay(blocks, nval)
    names = {"processed": 0, "no_parent": 1, "attestations_rejected": 2, "saved_not_candidate": 3}
    ai = 0
    for i, r in enumerate(recs):
        assert out["hash"][i].tobytes() == r["hash"], i
        assert out["status"][i] == names[r["status"]], i
        assert bool(out["transition"][i]) == r["transition"], i
        nb = len(blocks[i].attestations)
        if r["status"] == "no_parent":
            assert (out["att_status"][ai:ai + nb] == 1).all()
        else:
            for a in r["atts"]:
                if "error" in a:
                    assert out["att_status"][ai] == 2, (i, ai)
                else:
                    assert out["att_status"][ai] == 0
                    assert out["key"][ai].tobytes() == a["key"] and out["att_hash"][ai].tobytes() == a["hash"]
                    assert out["msg"][ai].tobytes() == a["msg"] and out["msg_len"][ai] == a["msg_len"]
                ai += 1
            continue
        ai += nb
    for k in ("chain_active", "chain_crystallized", "cand_active", "cand_crystallized", "vote_totals"):
        assert roots.get(k) == o_roots.get(k), k


def test_port_matches_golden_fixture():
    with open(os.path.join(HERE, "golden", "replay_n1024.json")) as f:
        g = json.load(f)
    blocks = synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"])
    out, roots = _port(blocks, g["nval"])
    for k, v in g["roots"].items():
        assert roots[k].hex() == v, k
    assert {k.hex(): v for k, v in roots["vote_totals"].items()} == g["vote_totals"]
    assert [out["hash"][i].tobytes().hex() for i in range(len(blocks))] == [r["hash"] for r in g["records"]]


@pytest.mark.parametrize("bitmap", [False, True])
@pytest.mark.parametrize("case", ["edited", "empty_committees", "n1000_200"])
def test_port_matches_scalar_oracle(case, bitmap):
    if case == "edited":
        _compare(edited_chain(), 1000, bitmap)
    elif case == "empty_committees":
        _compare(synth.chain_blocks(40, 130, seed=5), 40, bitmap)
    else:
        _compare(synth.chain_blocks(1000, 200, seed=8), 1000, bitmap)


def test_port_panics_where_go_panics():
    with pytest.raises(cport.OraclePanic):
        _port(future_slot_chain(), 1024)
    with pytest.raises(cport.OraclePanic):  # CalculateRewards' CheckBit by global index
        _port(synth.chain_blocks(1024, 70, seed=1, participation=(1.0,)), 1024)
