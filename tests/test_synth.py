"""The synthetic 512-byte attestation records are canonical proto3 encodings."""
from oracle import schema as pb
from prysm_amd import synth


def test_records_are_canonical_attestations():
    recs = synth.attestation_records_512(300, seed=2)
    assert recs.shape == (300, 512)
    for i in range(0, 300, 7):
        raw = recs[i].tobytes()
        a = pb.AttestationRecord()
        a.ParseFromString(raw)
        assert len(a.oblique_parent_hashes) == synth.N_OBLIQUE
        assert len(a.attester_bitfield) == synth.BITFIELD_BYTES
        assert len(a.aggregate_sig) == 2
        assert a.SerializeToString() == raw
