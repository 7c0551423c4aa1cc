"""ORACLE (test infrastructure only) — proto3 schema of the hashed messages.

Restates ``/root/reference/proto/beacon/p2p/v1/messages.proto:37-125`` as a
FileDescriptorProto built field by field, so Google's protobuf runtime serves as an
encoder that is independent of the product's own (``prysm_amd/wire.py``, ``prysm_amd/csrc/wire.hip``).
Field numbers, types and packing match the golang struct tags in
``messages.pb.go:224-232`` (BeaconBlock), ``:432-444`` (CrystallizedState), ``:559``
(ShardAndCommitteeArray), ``:673-674`` (ShardAndCommittee, packed committee),
``:757-758`` (ActiveState), ``:803-809`` (ValidatorRecord), ``:889-896``
(AttestationRecord, packed aggregate_sig), ``:983-985`` (CrosslinkRecord).
"""
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory, timestamp_pb2

_F = descriptor_pb2.FieldDescriptorProto
U64, U32, BYTES, MSG, I64, I32 = (_F.TYPE_UINT64, _F.TYPE_UINT32, _F.TYPE_BYTES,
                                  _F.TYPE_MESSAGE, _F.TYPE_INT64, _F.TYPE_INT32)
OPT, REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

PKG = "ethereum.beacon.p2p.v1"

# name -> [(field name, number, type, label, message type name or None)]
_MESSAGES = {
    "BeaconBlock": [
        ("parent_hash", 1, BYTES, OPT, None),
        ("slot_number", 2, U64, OPT, None),
        ("randao_reveal", 3, BYTES, OPT, None),
        ("pow_chain_ref", 4, BYTES, OPT, None),
        ("active_state_hash", 5, BYTES, OPT, None),
        ("crystallized_state_hash", 6, BYTES, OPT, None),
        ("timestamp", 7, MSG, OPT, ".google.protobuf.Timestamp"),
        ("attestations", 8, MSG, REP, ".%s.AttestationRecord" % PKG),
    ],
    "CrystallizedState": [
        ("last_state_recalc", 1, U64, OPT, None),
        ("justified_streak", 2, U64, OPT, None),
        ("last_justified_slot", 3, U64, OPT, None),
        ("last_finalized_slot", 4, U64, OPT, None),
        ("current_dynasty", 5, U64, OPT, None),
        ("crosslinking_start_shard", 6, U64, OPT, None),
        ("total_deposits", 7, U64, OPT, None),
        ("dynasty_seed", 8, BYTES, OPT, None),
        ("dynasty_seed_last_reset", 9, U64, OPT, None),
        ("crosslink_records", 10, MSG, REP, ".%s.CrosslinkRecord" % PKG),
        ("validators", 11, MSG, REP, ".%s.ValidatorRecord" % PKG),
        ("shard_and_committees_for_slots", 12, MSG, REP, ".%s.ShardAndCommitteeArray" % PKG),
    ],
    "ShardAndCommitteeArray": [
        ("array_shard_and_committee", 1, MSG, REP, ".%s.ShardAndCommittee" % PKG),
    ],
    "ShardAndCommittee": [
        ("shard_id", 1, U64, OPT, None),
        ("committee", 2, U32, REP, None),
    ],
    "ActiveState": [
        ("pending_attestations", 1, MSG, REP, ".%s.AttestationRecord" % PKG),
        ("recent_block_hashes", 2, BYTES, REP, None),
    ],
    "ValidatorRecord": [
        ("public_key", 1, U64, OPT, None),
        ("withdrawal_shard", 2, U64, OPT, None),
        ("withdrawal_address", 3, BYTES, OPT, None),
        ("randao_commitment", 4, BYTES, OPT, None),
        ("balance", 5, U64, OPT, None),
        ("start_dynasty", 6, U64, OPT, None),
        ("end_dynasty", 7, U64, OPT, None),
    ],
    "AttestationRecord": [
        ("slot", 1, U64, OPT, None),
        ("shard_id", 2, U64, OPT, None),
        ("justified_slot", 3, U64, OPT, None),
        ("justified_block_hash", 4, BYTES, OPT, None),
        ("shard_block_hash", 5, BYTES, OPT, None),
        ("attester_bitfield", 6, BYTES, OPT, None),
        ("oblique_parent_hashes", 7, BYTES, REP, None),
        ("aggregate_sig", 8, U64, REP, None),
    ],
    "CrosslinkRecord": [
        ("dynasty", 1, U64, OPT, None),
        ("blockhash", 2, BYTES, OPT, None),
        ("slot", 3, U64, OPT, None),
    ],
}


def _build():
    pool = descriptor_pool.DescriptorPool()
    ts = descriptor_pb2.FileDescriptorProto()
    timestamp_pb2.DESCRIPTOR.CopyToProto(ts)
    pool.Add(ts)
    fdp = descriptor_pb2.FileDescriptorProto(name="oracle_messages.proto", package=PKG,
                                             syntax="proto3",
                                             dependency=["google/protobuf/timestamp.proto"])
    for mname, fields in _MESSAGES.items():
        m = fdp.message_type.add(name=mname)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
    pool.Add(fdp)
    classes = {}
    for mname in _MESSAGES:
        classes[mname] = message_factory.GetMessageClass(
            pool.FindMessageTypeByName("%s.%s" % (PKG, mname)))
    classes["Timestamp"] = message_factory.GetMessageClass(
        pool.FindMessageTypeByName("google.protobuf.Timestamp"))
    return classes


_CLASSES = _build()
BeaconBlock = _CLASSES["BeaconBlock"]
CrystallizedState = _CLASSES["CrystallizedState"]
ShardAndCommitteeArray = _CLASSES["ShardAndCommitteeArray"]
ShardAndCommittee = _CLASSES["ShardAndCommittee"]
ActiveState = _CLASSES["ActiveState"]
ValidatorRecord = _CLASSES["ValidatorRecord"]
AttestationRecord = _CLASSES["AttestationRecord"]
CrosslinkRecord = _CLASSES["CrosslinkRecord"]
Timestamp = _CLASSES["Timestamp"]
