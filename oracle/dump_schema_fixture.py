"""ORACLE tool (container only; needs /root/reference) — write tests/golden/schema_descriptor.json.

The fixture is data: for every message of the descriptor that the reference's generated code
embeds (``proto/beacon/p2p/v1/messages.pb.go:1099-``), each field's number, type, label and
type name (no source text).  ``tests/test_schema_pin.py`` checks ``oracle/schema.py`` against
it, and against the live descriptor when /root/reference is present.
Run: ``python -m oracle.dump_schema_fixture``.
"""
import json
import os

from oracle.check_schema_vs_reference import reference_descriptor

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "schema_descriptor.json")


def descriptor_table(fdp):
    return {"package": fdp.package,
            "messages": {m.name: [[f.number, f.type, f.label, f.type_name] for f in m.field]
                         for m in fdp.message_type}}


if __name__ == "__main__":
    with open(OUT, "w") as f:
        json.dump(descriptor_table(reference_descriptor()), f, indent=1, sort_keys=True)
    print("wrote", OUT)
