"""Device proto3 encoder of AttestationRecord columns (prysm_amd/csrc/wire_att.hip) against
Google's protobuf runtime over the oracle schema (oracle/schema.py, pinned to
messages.pb.go:889-896) and the host encoder (prysm_amd/wire.py); and the config-2 records
(synth.attestation_records_512) rebuilt from their columns.  Byte-exact."""
import numpy as np
import pytest

from prysm_amd import _lib, pb, synth, wire
from test_wire import o_att, rand_att, rand_bytes, rand_u64

pytestmark = pytest.mark.gpu


def varint(x):
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


@pytest.mark.parametrize("n,seed", [(1, 1), (7, 2), (300, 3), (2000, 4)])
def test_bare_records_match_protobuf_runtime(n, seed):
    rng = np.random.default_rng(seed)
    atts = [rand_att(rng) for _ in range(n)]
    raw, offs = wire.attestations_device(wire.attestation_columns(atts), n, 0)
    assert offs[0] == 0 and offs[-1] == len(raw)
    for i, a in enumerate(atts):
        rec = raw[int(offs[i]):int(offs[i + 1])]
        assert rec == o_att(a).SerializeToString() == wire.attestation_record(a), i


@pytest.mark.parametrize("field_num", [8, 1, 16, (1 << 29) - 1])
def test_framed_records(field_num):
    rng = np.random.default_rng(field_num % 97)
    atts = [rand_att(rng) for _ in range(500)]
    raw, offs = wire.attestations_device(wire.attestation_columns(atts), len(atts), field_num)
    tag = varint((field_num << 3) | 2)
    want = b"".join(tag + varint(len(r)) + r for r in (wire.attestation_record(a) for a in atts))
    assert raw == want


def test_long_repeated_fields_and_empty_elements():
    """More than 64 oblique hashes / signature values (several wave chunks), empty elements
    (emitted as 3a 00), all-zero scalars, and records with nothing at all."""
    rng = np.random.default_rng(9)
    atts = [pb.AttestationRecord(slot=0, shard_id=0, justified_slot=0, justified_block_hash=b"", shard_block_hash=b"",
                                 attester_bitfield=b"", oblique_parent_hashes=[], aggregate_sig=[])]
    atts.append(pb.AttestationRecord(slot=5, shard_id=0, justified_slot=(1 << 64) - 1, justified_block_hash=b"x",
                                     shard_block_hash=b"", attester_bitfield=rand_bytes(rng, 300, 301),
                                     oblique_parent_hashes=[rand_bytes(rng, 0, 40) for _ in range(150)] + [b""],
                                     aggregate_sig=[rand_u64(rng) for _ in range(200)]))
    atts.append(pb.AttestationRecord(slot=1, shard_id=2, justified_slot=3, justified_block_hash=b"",
                                     shard_block_hash=b"", attester_bitfield=b"", oblique_parent_hashes=[b""] * 65,
                                     aggregate_sig=[0] * 70))
    raw, offs = wire.attestations_device(wire.attestation_columns(atts), len(atts), 0)
    for i, a in enumerate(atts):
        assert raw[int(offs[i]):int(offs[i + 1])] == o_att(a).SerializeToString(), i
    assert offs[1] == 0  # the empty record encodes to nothing


@pytest.mark.parametrize("field_num", [0, 1])
def test_half_wave_path_limits(field_num):
    """Records at and just past the row path's limits (wire_att.hip: 13 oblique elements,
    16 signature values, 64-byte segments, 768-byte records) next to each other, so both
    paths share waves, with segment sources at every alignment."""
    rng = np.random.default_rng(11 + field_num)
    atts = []
    for nob in (0, 1, 12, 13, 14, 33):
        for seg in (0, 1, 31, 32, 33, 63, 64, 65):
            for nsig in (0, 15, 16, 17):
                atts.append(pb.AttestationRecord(
                    slot=rand_u64(rng), shard_id=int(rng.integers(0, 3)), justified_slot=rand_u64(rng),
                    justified_block_hash=rand_bytes(rng, seg, seg + 1), shard_block_hash=rand_bytes(rng, 0, 66),
                    attester_bitfield=rand_bytes(rng, max(seg - 1, 0), seg + 2),
                    oblique_parent_hashes=[rand_bytes(rng, 0, min(seg, 24) + 1) for _ in range(nob)],
                    aggregate_sig=[rand_u64(rng) for _ in range(nsig)]))
    for extra in (0, 13, 14, 22):  # 13 elements of 55 bytes: records of 753, 768, 769 and 777 bytes
        atts.append(pb.AttestationRecord(slot=1, shard_id=1, justified_slot=1, justified_block_hash=b"",
                                         shard_block_hash=rand_bytes(rng, extra, extra + 1), attester_bitfield=b"x",
                                         oblique_parent_hashes=[rand_bytes(rng, 55, 56) for _ in range(13)],
                                         aggregate_sig=[7]))
    rng.shuffle(atts)
    raw, offs = wire.attestations_device(wire.attestation_columns(atts), len(atts), field_num)
    tag = varint((field_num << 3) | 2) if field_num else b""
    want = [wire.attestation_record(a) for a in atts]
    assert raw == b"".join((tag + varint(len(r)) + r) if field_num else r for r in want)
    assert any(len(r) > 768 for r in want) and any(len(r) <= 768 for r in want)


def test_mixed_paths_across_many_waves():
    """Row-path and whole-wave records of every size class shuffled over ~2,000 waves: each
    wave's output offset comes from the look-back over its predecessors (wire_att.hip)."""
    rng = np.random.default_rng(23)
    atts = []
    for _ in range(8000):
        kind = int(rng.integers(0, 4))
        nob = (0, 9, 14, 40)[kind]
        atts.append(pb.AttestationRecord(
            slot=rand_u64(rng), shard_id=int(rng.integers(0, 1 << 20)), justified_slot=int(rng.integers(0, 2)),
            justified_block_hash=rand_bytes(rng, 0, 33), shard_block_hash=rand_bytes(rng, 32, 33),
            attester_bitfield=rand_bytes(rng, 0, 70 if kind < 3 else 300),
            oblique_parent_hashes=[rand_bytes(rng, 0, 33) for _ in range(nob)],
            aggregate_sig=[rand_u64(rng) for _ in range(int(rng.integers(0, 18)))]))
    raw, offs = wire.attestations_device(wire.attestation_columns(atts), len(atts), 0)
    want = [wire.attestation_record(a) for a in atts]
    assert raw == b"".join(want)
    assert np.array_equal(np.diff(offs), [len(r) for r in want])


def test_empty_batch():
    raw, offs = wire.attestations_device(wire.attestation_columns([]), 0, 0)
    assert raw == b"" and list(offs) == [0]


def test_config2_records_rebuilt_from_columns():
    """synth.attestation_columns_512 encodes to exactly the 512-byte records the hash bench
    uses (BASELINE configs[1]), at 2^18 records."""
    n = 1 << 18
    cols = synth.attestation_columns_512(n, seed=2)
    raw, offs = wire.attestations_device(cols, n, 0)
    assert np.array_equal(offs, np.arange(n + 1, dtype=np.uint64) * 512)
    assert raw == synth.attestation_records_512(n, seed=2).tobytes()


def test_capacity_error():
    rng = np.random.default_rng(5)
    atts = [rand_att(rng) for _ in range(50)]
    cols = wire.attestation_columns(atts)
    c = _lib.AttestationCols(*[_lib.ptr(np.ascontiguousarray(cols[k])) for k in wire.ATT_COLS])
    out = np.empty(8, dtype=np.uint8)
    length = _lib.ctypes.c_uint64(0)
    with pytest.raises(_lib.PzError) as e:
        _lib.lib.call("pz_wire_attestations", _lib.ctypes.byref(c), 50, 0, _lib.ptr(out), 8, None,
                      _lib.ctypes.byref(length))
    assert e.value.code == _lib.PZ_ERANGE
    assert length.value == sum(len(wire.attestation_record(a)) for a in atts)
