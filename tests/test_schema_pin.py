"""The oracle's proto3 schema (oracle/schema.py) is pinned to the descriptor embedded in the
reference's generated code (proto/beacon/p2p/v1/messages.pb.go:1099-).  Every digest fixture
rests on it.  Field numbers, wire types, labels and sub-message type names must agree; names
are not on the wire (the descriptor's stale field-12 name ``indices_for_slots`` is ignored)."""
import json
import os

import pytest

from oracle.schema import _MESSAGES, PKG

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "schema_descriptor.json")
REF = "/root/reference/proto/beacon/p2p/v1/messages.pb.go"


def _fixture():
    with open(FIXTURE) as f:
        return json.load(f)


def test_schema_matches_descriptor_fixture():
    d = _fixture()
    assert d["package"] == PKG
    for mname, fields in _MESSAGES.items():
        ref = {num: (ftype, label, tname) for num, ftype, label, tname in d["messages"][mname]}
        assert len(ref) == len(fields), mname
        for fname, num, ftype, label, tname in fields:
            assert num in ref, (mname, fname)
            rtype, rlabel, rtname = ref[num]
            assert (rtype, rlabel) == (ftype, label), (mname, fname)
            if tname:
                assert rtname == tname, (mname, fname)


@pytest.mark.skipif(not os.path.exists(REF), reason="reference tree absent (GPU box)")
def test_fixture_matches_reference_descriptor():
    from oracle.check_schema_vs_reference import main, reference_descriptor
    from oracle.dump_schema_fixture import descriptor_table
    assert descriptor_table(reference_descriptor()) == _fixture()
    assert main() == 0
