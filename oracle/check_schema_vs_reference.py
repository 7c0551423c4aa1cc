"""ORACLE tool (container only; needs /root/reference) — pin oracle/schema.py.

Decodes the gzipped FileDescriptorProto that the reference's generated code embeds
(``/root/reference/proto/beacon/p2p/v1/messages.pb.go:1099-``) and checks that every
field of every hashed message in ``oracle/schema.py`` has the same number, type and
label.  The reference descriptor names field 12 of CrystallizedState
``indices_for_slots`` (stale vs messages.proto); names are not on the wire, so only
number/type/label/type_name are compared.  Run: ``python -m oracle.check_schema_vs_reference``.
"""
import gzip
import re
import sys

from google.protobuf import descriptor_pb2

from oracle.schema import _MESSAGES, PKG

REF = "/root/reference/proto/beacon/p2p/v1/messages.pb.go"


def reference_descriptor():
    src = open(REF).read()
    body = src[src.index("var fileDescriptor_messages"):]
    body = body[body.index("{") + 1: body.index("\n}")]
    raw = bytes(int(h, 16) for h in re.findall(r"0x([0-9a-f]{2})", body))
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.ParseFromString(gzip.decompress(raw))
    return fdp


def main():
    fdp = reference_descriptor()
    ref = {m.name: {f.number: f for f in m.field} for m in fdp.message_type}
    bad = 0
    for mname, fields in _MESSAGES.items():
        for fname, num, ftype, label, tname in fields:
            rf = ref[mname].get(num)
            ok = rf is not None and rf.type == ftype and rf.label == label
            if ok and tname:
                ok = rf.type_name == tname
            print("%-24s %2d %-32s %s" % (mname, num, fname, "ok" if ok else "MISMATCH"))
            bad += not ok
        if len(ref[mname]) != len(fields):
            print("%s: field count differs" % mname)
            bad += 1
    print("package", fdp.package, "==", PKG, fdp.package == PKG)
    return 1 if bad or fdp.package != PKG else 0


if __name__ == "__main__":
    sys.exit(main())
