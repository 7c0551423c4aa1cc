"""Synthetic, seeded inputs shaped like the BASELINE.json configs (plumbing for bench/tests).

``attestation_records_512`` builds N proto3-serialized AttestationRecords
(proto/beacon/p2p/v1/messages.proto:110-119) of exactly 512 bytes each, vectorised with
numpy: every record has the same field layout (fixed-width varints, 11 oblique parent
hashes, a 35-byte attester bitfield, two 10-byte-varint aggregate_sig words) and random
payload bytes.  ``tests/test_synth.py`` re-parses samples with the oracle's protobuf schema
and checks they re-serialize to the identical bytes, i.e. they are canonical encodings.
"""
import numpy as np

RECORD_BYTES = 512
N_OBLIQUE = 11
BITFIELD_BYTES = 35


def _varint_fixed(values, width):
    """Little-endian base-128 varint of ``values`` (uint64 array) occupying exactly ``width``
    bytes (caller guarantees the value range makes that the canonical length)."""
    out = np.empty((values.shape[0], width), dtype=np.uint8)
    v = values.astype(np.uint64).copy()
    for k in range(width):
        b = (v & np.uint64(0x7F)).astype(np.uint8)
        if k < width - 1:
            b |= 0x80
        out[:, k] = b
        v >>= np.uint64(7)
    return out


def attestation_records_512(n, seed=2):
    """(n, 512) uint8 array of canonical AttestationRecord encodings."""
    rng = np.random.default_rng(seed)
    rec = np.empty((n, RECORD_BYTES), dtype=np.uint8)
    col = 0

    def put(arr):
        nonlocal col
        w = arr.shape[1]
        rec[:, col:col + w] = arr
        col += w

    def const(*bs):
        put(np.tile(np.array(bs, dtype=np.uint8), (n, 1)))

    slot = rng.integers(1 << 14, 1 << 21, size=n, dtype=np.uint64)          # 3-byte varint
    shard = rng.integers(128, 1024, size=n, dtype=np.uint64)                # 2-byte varint
    jslot = rng.integers(1 << 14, 1 << 21, size=n, dtype=np.uint64)         # 3-byte varint
    const(0x08); put(_varint_fixed(slot, 3))                                # slot = 1
    const(0x10); put(_varint_fixed(shard, 2))                               # shard_id = 2
    const(0x18); put(_varint_fixed(jslot, 3))                               # justified_slot = 3
    const(0x22, 32); put(rng.integers(0, 256, size=(n, 32), dtype=np.uint8))  # justified_block_hash
    const(0x2A, 32); put(rng.integers(0, 256, size=(n, 32), dtype=np.uint8))  # shard_block_hash
    bf = rng.integers(0, 256, size=(n, BITFIELD_BYTES), dtype=np.uint8)
    const(0x32, BITFIELD_BYTES); put(bf)                                    # attester_bitfield
    for _ in range(N_OBLIQUE):                                              # oblique_parent_hashes
        const(0x3A, 32); put(rng.integers(0, 256, size=(n, 32), dtype=np.uint8))
    sig = rng.integers(1 << 63, (1 << 64) - 1, size=(n, 2), dtype=np.uint64, endpoint=True)
    const(0x42, 20); put(_varint_fixed(sig[:, 0], 10)); put(_varint_fixed(sig[:, 1], 10))
    assert col == RECORD_BYTES, col
    return rec
