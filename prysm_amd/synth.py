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


def committees_csr(shuffled, crosslink_start_shard=0):
    """casper/sharding.go:27-53 on a shuffled index list -> (committee uint32, coffs uint64,
    slot_of uint32, shard_of uint32) with committees ordered slot-major."""
    from prysm_amd.casper import split_by_slot_shard
    members, offs, slots, shards = [], [0], [], []
    for s, arr in enumerate(split_by_slot_shard(list(shuffled), crosslink_start_shard)):
        for shard, c in arr:
            members.append(np.asarray(c, dtype=np.uint32))
            offs.append(offs[-1] + len(c))
            slots.append(s)
            shards.append(shard)
    return (np.concatenate(members) if members else np.zeros(0, np.uint32), np.array(offs, dtype=np.uint64),
            np.array(slots, dtype=np.uint32), np.array(shards, dtype=np.uint32))


def epoch_batch(nval, ninst, seed=3, shuffled=None, density=0.75, last_bits=None):
    """Synthetic epoch instances shaped like BASELINE configs[2]/[3]:
    all validators active (start 0, end DefaultEndDynasty), balances 32 +- jitter in
    [16, 48], one attestation per committee (~75% (density 0.75) or ~50% bits set, trailing bits zero) plus a
    final attestation whose bitfield has ``nval`` bits (the incentives_test.go:24-25 shape),
    TotalDeposits = sum(balance), CurrentDynasty 1, crosslink records at dynasty 0.
    ``shuffled`` is the shuffled active index list (ShuffleIndices(Hash{'A'}, 0..N-1)); the
    committees are shared by all instances."""
    from prysm_amd.params import DEFAULT_END_DYNASTY
    rng = np.random.default_rng(seed)
    if shuffled is None:
        shuffled = np.arange(nval, dtype=np.uint32)
    committee, coffs, c_slot, c_shard = committees_csr(shuffled)
    ncomm = len(coffs) - 1
    natt = ncomm + 1
    sizes = np.diff(coffs).astype(np.int64)
    start = np.zeros((ninst, nval), dtype=np.uint64)
    end = np.full((ninst, nval), DEFAULT_END_DYNASTY, dtype=np.uint64)
    balance = rng.integers(16, 49, size=(ninst, nval), dtype=np.uint64)
    kfinal = last_bits if last_bits is not None else nval
    blens = np.concatenate([(sizes + 7) // 8, [(kfinal + 7) // 8]])
    per_inst = int(blens.sum())
    boffs = np.zeros(ninst * natt + 1, dtype=np.uint64)
    boffs[1:] = np.cumsum(np.tile(blens, ninst))
    # ~75% of bits set (OR of two uniform bytes), then the trailing pad bits of every
    # bitfield cleared (validateAttesterBitfields, core.go:384-392)
    bits = rng.integers(0, 256, size=ninst * per_inst, dtype=np.uint8)
    if density >= 0.75:
        bits |= rng.integers(0, 256, size=ninst * per_inst, dtype=np.uint8)
    kbits = np.concatenate([sizes, [kfinal]])
    tail = (kbits % 8).astype(np.uint8)
    last_byte = np.tile(np.cumsum(blens) - 1, ninst) + np.repeat(np.arange(ninst) * per_inst, natt)
    keep = np.tile(np.where(tail == 0, 0xFF, (0xFF << (8 - tail)) & 0xFF).astype(np.uint8), ninst)
    bits[last_byte] &= keep
    att_comm = np.tile(np.concatenate([np.arange(ncomm), [ncomm - 1]]).astype(np.uint32), ninst)
    att_shard = np.tile(np.concatenate([c_shard, [c_shard[-1]]]).astype(np.uint32), ninst)
    att_slot = np.tile(np.concatenate([c_slot, [c_slot[-1]]]).astype(np.uint64), ninst)
    with np.errstate(over="ignore"):
        total = balance.sum(axis=1, dtype=np.uint64)
    return dict(nval=nval, ninst=ninst, natt=natt, start=start, end=end, balance=balance,
                dynasty=np.ones(ninst, dtype=np.uint64), total_deposit=total, bits=bits, boffs=boffs,
                committee=committee, coffs=coffs, att_comm=att_comm, att_shard=att_shard,
                att_slot=att_slot, rec_dynasty=np.zeros((ninst, 1024), dtype=np.uint64),
                max_inst_bytes=per_inst)


def epoch_instances(inst, k):
    """The first ``k`` instances of an ``epoch_batch`` (every instance's bitfields have the
    same layout, so instance i's CSR range is i * max_inst_bytes onward)."""
    natt, per = int(inst["natt"]), int(inst["max_inst_bytes"])
    out = dict(inst)
    out["ninst"] = k
    for key in ("start", "end", "balance", "dynasty", "total_deposit", "rec_dynasty"):
        out[key] = inst[key][:k].copy()
    for key in ("att_comm", "att_shard", "att_slot"):
        out[key] = inst[key][:k * natt].copy()
    out["bits"] = inst["bits"][:k * per].copy()
    out["boffs"] = inst["boffs"][:k * natt + 1].copy()
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


def attestation_columns_512(n, seed=2):
    """The SoA columns of ``attestation_records_512(n, seed)`` (same random draws), in the CSR
    layout of ``pz_attestation_cols``: encoding them gives exactly those 512-byte records."""
    rng = np.random.default_rng(seed)
    u64 = np.uint64
    slot = rng.integers(1 << 14, 1 << 21, size=n, dtype=u64)
    shard = rng.integers(128, 1024, size=n, dtype=u64)
    jslot = rng.integers(1 << 14, 1 << 21, size=n, dtype=u64)
    jbh = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sbh = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    bf = rng.integers(0, 256, size=(n, BITFIELD_BYTES), dtype=np.uint8)
    obl = np.stack([rng.integers(0, 256, size=(n, 32), dtype=np.uint8) for _ in range(N_OBLIQUE)], axis=1)
    sig = rng.integers(1 << 63, (1 << 64) - 1, size=(n, 2), dtype=u64, endpoint=True)

    def fixed(width, count):
        return np.arange(count + 1, dtype=u64) * u64(width)

    return dict(slot=slot, shard_id=shard, justified_slot=jslot,
                justified_block_hash=jbh.reshape(-1), justified_block_hash_offs=fixed(32, n),
                shard_block_hash=sbh.reshape(-1), shard_block_hash_offs=fixed(32, n),
                attester_bitfield=bf.reshape(-1), attester_bitfield_offs=fixed(BITFIELD_BYTES, n),
                oblique_parent_hashes=obl.reshape(-1), oblique_offs=fixed(32, n * N_OBLIQUE),
                oblique_first=fixed(N_OBLIQUE, n), aggregate_sig=sig.reshape(-1), aggregate_sig_first=fixed(2, n))


def genesis_committee_sizes(nval):
    """Shard ids and member counts of the slot-0 committees of the genesis shuffle
    (types/state.go:68-78 -> casper/sharding.go:27-53).  Sizes depend only on the validator
    count, so no shuffle is needed to shape attestations for them."""
    from prysm_amd.casper import split_by_slot_shard
    slot0 = split_by_slot_shard(list(range(nval)), 0)[0]
    return [(int(shard), int(len(c))) for shard, c in slot0]


def chain_blocks(nval, nblocks, seed=1, participation=(1.0, 0.25), n_oblique=1, committees=None):
    """A synthetic chain of ``nblocks`` blocks (slots 1..nblocks) that the reference's
    ChainService.blockProcessing (blockchain/service.go:229-363) processes end to end.

    Each block carries one AttestationRecord per slot-0 committee (``committees`` limits the
    count).  Its slot is ``64 * (s // 64)`` for block slot ``s``: the only choice that never
    makes the reference index ShardAndCommitteesForSlots with a wrapped-around
    ``Slot - LastStateRecalc`` (core.go:367), neither in processAttestation nor in the
    stateRecalc after next (pending attestations survive one recalc, core.go:445-450).
    Bitfields have BitLength(k) bytes with clear trailing bits (core.go:377-394); committee
    j of block s sets each bit with probability ``participation[(s + j) % len(participation)]``.
    The default mix keeps the attester popcount under 2/3 of the deposits, so
    CalculateRewards does not run into its CheckBit-by-global-index panic (SURVEY.md §0 fact
    2); ``participation=(1.0,)`` reproduces that panic at the first cycle transition.

    Timestamps are 8 s per slot (Timestamp{8*s, 0}); the parent of block 1 is the genesis
    block.  Parent digests are computed here with hashlib (input generation only: the
    replay under test recomputes every digest on the GPU and checks parents against them).
    Returns the list of ``pb.BeaconBlock``."""
    import hashlib

    from prysm_amd import pb, wire
    from prysm_amd.params import CYCLE_LENGTH

    rng = np.random.default_rng(seed)
    comms = genesis_committee_sizes(nval)
    if committees is not None:
        comms = comms[:committees]
    parent = hashlib.blake2b(wire.beacon_block(pb.BeaconBlock(timestamp=pb.Timestamp())), digest_size=64).digest()[:32]
    out = []
    for s in range(1, nblocks + 1):
        a_slot = CYCLE_LENGTH * (s // CYCLE_LENGTH)
        atts = []
        for j, (shard, k) in enumerate(comms):
            p = participation[(s + j) % len(participation)]
            nb = (k + 7) // 8
            bits = (rng.random(8 * nb) < p)
            bits[k:] = False
            atts.append(pb.AttestationRecord(
                slot=a_slot, shard_id=shard, justified_slot=0,
                justified_block_hash=rng.bytes(32), shard_block_hash=rng.bytes(32),
                attester_bitfield=np.packbits(bits).tobytes(),
                oblique_parent_hashes=[rng.bytes(32) for _ in range(n_oblique)],
                aggregate_sig=[int(x) for x in rng.integers(0, 1 << 63, size=2, dtype=np.uint64)]))
        blk = pb.BeaconBlock(parent_hash=parent, slot_number=s, randao_reveal=rng.bytes(32),
                             pow_chain_ref=rng.bytes(32), active_state_hash=rng.bytes(32),
                             crystallized_state_hash=rng.bytes(32), timestamp=pb.Timestamp(8 * s, 0),
                             attestations=atts)
        out.append(blk)
        parent = hashlib.blake2b(wire.beacon_block(blk), digest_size=64).digest()[:32]
    return out
