"""ORACLE (test infrastructure only) — scalar CPU restatement of the reference hot path.

Every function cites the Go source it restates (paths relative to
``/root/reference/beacon-chain``).  Go ``uint64`` wrap-around is reproduced with ``& M64``;
Go index-out-of-range panics are reproduced as ``GoPanic``.  State objects are the
protobuf messages of ``oracle.schema`` (mutable, like the Go ``*pb.X`` pointers).
"""
import hashlib

from oracle import schema as pb

M64 = (1 << 64) - 1

# params/config.go:4-26
ATTESTER_REWARD = 1
CYCLE_LENGTH = 64
SHARD_COUNT = 1024
DEFAULT_BALANCE = 32
MAX_VALIDATORS = 4194304
MIN_COMMITTEE_SIZE = 128
DEFAULT_END_DYNASTY = 9999999999999999999
BOOTSTRAPPED_VALIDATORS_COUNT = 1000


class GoPanic(Exception):
    """A Go runtime panic (index out of range) in the reference."""


class GoError(Exception):
    """A Go ``error`` return in the reference."""


# --- BLAKE2b (golang.org/x/crypto/blake2b @ a49355c, RFC 7693) ----------------------------
def sum512(data):
    return hashlib.blake2b(bytes(data), digest_size=64).digest()


def hash32(data):
    """``h := blake2b.Sum512(data); copy(hash[:], h[:32])`` (types/block.go:73-76)."""
    return sum512(data)[:32]


# --- go-ethereum common helpers ----------------------------------------------------------
def bytes_to_hash(b):
    """common.BytesToHash: keep the last 32 bytes, right-align (go-ethereum @ c169d4b)."""
    b = bytes(b)
    if len(b) > 32:
        b = b[len(b) - 32:]
    return bytes(32 - len(b)) + b


def copy32(b):
    """``var h [32]byte; copy(h[:], b)``: left-align, truncate (types/block.go:80-84)."""
    b = bytes(b)[:32]
    return b + bytes(32 - len(b))


def put_uvarint(buf, off, x):
    """encoding/binary.PutUvarint into ``buf[off:]`` (mutates ``buf``); returns length."""
    i = 0
    while x >= 0x80:
        buf[off + i] = (x & 0x7F) | 0x80
        x >>= 7
        i += 1
    buf[off + i] = x
    return i + 1


# --- utils/checkbit.go -------------------------------------------------------------------
def check_bit(bitfield, index):
    """utils/checkbit.go:4-15 (MSB-first); panics when the byte is out of range."""
    chunk = (index + 1) // 8
    loc = (index + 1) % 8
    if loc == 0:
        loc = 8
    else:
        chunk += 1
    if index < -1 or chunk - 1 >= len(bitfield) or chunk - 1 < 0:
        raise GoPanic("CheckBit index %d out of range for %d-byte bitfield" % (index, len(bitfield)))
    return (bitfield[chunk - 1] >> (8 - loc)) % 2 != 0


def bit_set_count(v):
    """utils/checkbit.go:19-23 (SWAR byte popcount)."""
    v = (v & 0x55) + ((v >> 1) & 0x55)
    v = (v & 0x33) + ((v >> 2) & 0x33)
    return (v + (v >> 4)) & 0xF


def bit_length(b):
    """utils/checkbit.go:26-28."""
    return (b + 7) // 8


# --- utils/shuffle.go --------------------------------------------------------------------
def shuffle_indices(seed32, validator_list):
    """utils/shuffle.go:14-33: in place; the 64-byte seed stream is never re-hashed and the
    3-byte sum wraps as a byte (``int(hashSeed[j] + hashSeed[j+1] + hashSeed[j+2])``)."""
    if len(validator_list) > MAX_VALIDATORS:
        raise GoError("Validator count has exceeded MaxValidator Count")
    hs = sum512(seed32)
    n = len(validator_list)
    sw = [(hs[j] + hs[j + 1] + hs[j + 2]) & 0xFF for j in range(0, 61, 3)]
    lst = validator_list
    for i in range(n - 1):
        rem = n - i
        for s in sw:
            p = s % rem + i
            lst[i], lst[p] = lst[p], lst[i]
    return lst


def split_indices(l, n):
    """utils/shuffle.go:36-44."""
    return [l[len(l) * i // n: len(l) * (i + 1) // n] for i in range(n)]


# --- casper/sharding.go ------------------------------------------------------------------
def get_committee_params(num_validators):
    """casper/sharding.go:60-73."""
    if num_validators >= CYCLE_LENGTH * MIN_COMMITTEE_SIZE:
        return num_validators // (CYCLE_LENGTH * MIN_COMMITTEE_SIZE * 2) + 1, 1
    spc = 1
    while num_validators * spc < MIN_COMMITTEE_SIZE * CYCLE_LENGTH and spc < CYCLE_LENGTH:
        spc *= 2
    return 1, spc


def split_by_slot_shard(shuffled, crosslink_start_shard):
    """casper/sharding.go:27-53 -> list of 64 ShardAndCommitteeArray."""
    cps, spc = get_committee_params(len(shuffled))
    out = []
    for i, vs in enumerate(split_indices(shuffled, CYCLE_LENGTH)):
        arr = pb.ShardAndCommitteeArray()
        shard_start = crosslink_start_shard + i * cps // spc
        for j, committee in enumerate(split_indices(vs, cps)):
            sc = arr.array_shard_and_committee.add()
            sc.shard_id = (shard_start + j) % SHARD_COUNT
            sc.committee.extend(committee)
        out.append(arr)
    return out


def shuffle_validators_to_committees(seed32, validators, dynasty, crosslink_start_shard):
    """casper/sharding.go:11-21."""
    indices = active_validator_indices(validators, dynasty)
    shuffled = shuffle_indices(seed32, indices)
    return split_by_slot_shard(shuffled, crosslink_start_shard)


# --- casper/validator.go -----------------------------------------------------------------
def active_validator_indices(validators, dynasty):
    """casper/validator.go:45-53."""
    return [i for i, v in enumerate(validators) if v.start_dynasty <= dynasty < v.end_dynasty]


def exited_validator_indices(validators, dynasty):
    """casper/validator.go:57-65."""
    return [i for i, v in enumerate(validators) if v.start_dynasty < dynasty and v.end_dynasty <= dynasty]


def queued_validator_indices(validators, dynasty):
    """casper/validator.go:69-77."""
    return [i for i, v in enumerate(validators) if v.start_dynasty > dynasty]


def get_attesters_total_deposit(attestations):
    """casper/validator.go:93-102."""
    bits = sum(bit_set_count(b) for a in attestations for b in a.attester_bitfield)
    return (bits * DEFAULT_BALANCE) & M64


def rotate_validator_set(validators, dynasty):
    """casper/validator.go:17-41."""
    upper = len(active_validator_indices(validators, dynasty)) // 30 + 1
    for idx in active_validator_indices(validators, dynasty):
        if validators[idx].balance < DEFAULT_BALANCE // 2:
            validators[idx].end_dynasty = dynasty
    induct = upper
    queued = queued_validator_indices(validators, dynasty)
    if len(queued) < induct:
        induct = len(queued)
    for idx in queued_validator_indices(validators, dynasty):
        validators[idx].start_dynasty = dynasty
        induct -= 1
        if induct == 0:
            break
    return validators


# --- casper/incentives.go ----------------------------------------------------------------
def calculate_rewards(attestations, validators, dynasty, total_deposit):
    """casper/incentives.go:14-32: target is ``validators[i]`` (rank i in the active list),
    the bit tested is ``a[i]`` of the LAST attestation's bitfield."""
    active = active_validator_indices(validators, dynasty)
    deposits = get_attesters_total_deposit(attestations)
    if (deposits * 3) & M64 >= (total_deposit * 2) & M64:
        for i, a in enumerate(active):
            if not attestations:
                raise GoPanic("index out of range [-1]")
            voted = check_bit(attestations[-1].attester_bitfield, a)
            v = validators[i]
            v.balance = (v.balance + ATTESTER_REWARD) & M64 if voted else (v.balance - ATTESTER_REWARD) & M64
    return validators


# --- types -------------------------------------------------------------------------------
def marshal(msg):
    return msg.SerializeToString()


def block_hash(block):
    """types/block.go:67-77."""
    return hash32(marshal(block))


def attestation_hash(att):
    """types/attestation.go:49-59."""
    return hash32(marshal(att))


def attestation_key_bytes(att):
    """types/attestation.go:61-77: both varints are written at offset 0 of a 10-byte buffer
    (the shard id overwrites the slot), then the raw shard block hash, then each oblique
    parent hash left-aligned to 32 bytes."""
    key = bytearray(10)
    put_uvarint(key, 0, att.slot)
    put_uvarint(key, 0, att.shard_id)
    key += bytes(att.shard_block_hash)
    for h in att.oblique_parent_hashes:
        key += copy32(h)
    return bytes(key)


def attestation_key(att):
    return hash32(attestation_key_bytes(att))


def active_state_hash(astate):
    """types/state.go:138-149."""
    return hash32(marshal(astate))


def crystallized_state_hash(cstate):
    """types/state.go:237-248."""
    return hash32(marshal(cstate))


def new_genesis_states(num_validators=BOOTSTRAPPED_VALIDATORS_COUNT):
    """types/state.go:44-112 (``BootstrappedValidatorsCount`` made a parameter)."""
    active = pb.ActiveState()
    for _ in range(2 * CYCLE_LENGTH):
        active.recent_block_hashes.append(b"")
    cs = pb.CrystallizedState()
    for _ in range(num_validators):
        v = cs.validators.add()
        v.start_dynasty = 0
        v.end_dynasty = DEFAULT_END_DYNASTY
        v.balance = DEFAULT_BALANCE
    committees = shuffle_validators_to_committees(bytes_to_hash(b""), cs.validators, 1, 0)
    committees = committees + committees
    for arr in committees + committees:
        cs.shard_and_committees_for_slots.add().CopyFrom(arr)
    for _ in range(SHARD_COUNT):
        cs.crosslink_records.add()
    cs.current_dynasty = 1
    cs.total_deposits = (num_validators * DEFAULT_BALANCE) & M64
    return active, cs


def new_genesis_block():
    """types/block.go:43-55: Timestamp{0,0} is a non-nil empty message (``3a 00``)."""
    b = pb.BeaconBlock()
    b.timestamp.SetInParent()
    return b


# --- blockchain/core.go ------------------------------------------------------------------
def recent_block_hashes(astate):
    """types/state.go:189-195 (right-aligned via BytesToHash)."""
    return [bytes_to_hash(h) for h in astate.recent_block_hashes]


def get_attester_indices(cstate, att):
    """blockchain/core.go:363-374."""
    idx = (att.slot - cstate.last_state_recalc) & M64
    arrs = cstate.shard_and_committees_for_slots
    if idx >= len(arrs):
        raise GoPanic("ShardAndCommitteesForSlots index out of range")
    for sc in arrs[idx].array_shard_and_committee:
        if sc.shard_id == att.shard_id:
            return list(sc.committee)
    raise GoError("unable to find attestation based on slot: %d, shardID: %d" % (att.slot, att.shard_id))


def get_signed_parent_hashes(astate, block_slot, att):
    """blockchain/core.go:348-360.  Slicing beyond len (allowed by Go up to cap) raises."""
    start = (block_slot - att.slot) & M64
    end = (block_slot - att.slot - len(att.oblique_parent_hashes) + CYCLE_LENGTH) & M64
    recent = recent_block_hashes(astate)
    if start > end or end > len(recent):
        raise GoPanic("slice bounds out of range [%d:%d] with length %d" % (start, end, len(recent)))
    return recent[start:end] + [bytes_to_hash(h) for h in att.oblique_parent_hashes]


def validate_attester_bitfields(att, attester_indices):
    """blockchain/core.go:377-394."""
    if bit_length(len(attester_indices)) != len(att.attester_bitfield):
        raise GoError("attestation has incorrect bitfield length")
    last = len(attester_indices)
    if last % 8 != 0:
        for i in range(8 - last % 8):
            if check_bit(att.attester_bitfield, last + i):
                raise GoError("attestation has non-zero trailing bits")


def process_attestation_message(att, parent_hashes):
    """blockchain/core.go:277-290: both varints land at offset 0 (shard id overwrites slot%64)."""
    msg = bytearray(10)
    signed = b"".join(h + b" " for h in parent_hashes)
    put_uvarint(msg, 0, att.slot % CYCLE_LENGTH)
    msg += signed
    put_uvarint(msg, 0, att.shard_id)
    msg += bytes(att.shard_block_hash)
    return bytes(msg)


def process_attestation(cstate, astate, block_slot, att):
    """blockchain/core.go:240-297 -> (message bytes, Sum512 of it)."""
    if att.slot > block_slot:
        raise GoError("attestation slot number can't be higher than block slot number")
    if att.slot < block_slot - CYCLE_LENGTH:
        raise GoError("attestation slot number can't be lower than block slot number by one CycleLength")
    if att.justified_slot != cstate.last_justified_slot:
        raise GoError("attestation's last justified slot has to match")
    parents = get_signed_parent_hashes(astate, block_slot, att)
    indices = get_attester_indices(cstate, att)
    validate_attester_bitfields(att, indices)
    msg = process_attestation_message(att, parents)
    return msg, sum512(msg)


def calculate_block_vote_cache(cstate, astate, cache, block_slot, att):
    """blockchain/core.go:300-345.  ``cache`` maps 32-byte hash -> [VoterIndices, total].
    VoterIndices is an insertion-ordered dict (the Go slice's append order; the linear
    membership scan of core.go:333-337 becomes a dict lookup, same answer)."""
    parents = get_signed_parent_hashes(astate, block_slot, att)
    committee = get_attester_indices(cstate, att)
    obliques = [bytes(o) for o in att.oblique_parent_hashes]
    for h in parents:
        if any(h == o for o in obliques):
            continue
        if h not in cache:
            cache[h] = [{}, 0]
        entry = cache[h]
        for i, v in enumerate(committee):
            if not check_bit(att.attester_bitfield, i):
                continue
            if v not in entry[0]:
                entry[0][v] = None
                entry[1] = (entry[1] + cstate.validators[v].balance) & M64
    return cache


def process_crosslinks(cstate, records, validators, pending, dynasty, slot):
    """blockchain/core.go:502-558: in order; the first qualifying attestation per shard wins
    for a given dynasty because the record is replaced in place."""
    for att in pending:
        indices = get_attester_indices(cstate, att)
        total = 0
        for a in indices:
            total = (total + validators[a].balance) & M64
        vote = 0
        for i, a in enumerate(indices):
            if check_bit(att.attester_bitfield, i):
                vote = (vote + validators[a].balance) & M64
        # Go's && short-circuits: crosslinkRecords[ShardId] is indexed (and panics when out of
        # range) only once the 2/3 test holds (core.go:549)
        if (3 * vote) & M64 < (2 * total) & M64:
            continue
        if att.shard_id >= len(records):
            raise GoPanic("crosslink record index out of range")
        if dynasty > records[att.shard_id].dynasty:
            rec = pb.CrosslinkRecord(dynasty=dynasty, blockhash=bytes(att.shard_block_hash), slot=slot)
            records[att.shard_id].CopyFrom(rec)
    return records


def state_recalc(cstate, astate, cache, block_slot):
    """blockchain/core.go:398-497.  Returns (new cstate, new astate).  Mutates
    ``cstate``'s crosslink records and validator balances in place, like the reference.
    Committee lookups use ``cstate`` (== ``b.CrystallizedState()`` on the service path)."""
    streak = cstate.justified_streak
    justified = cstate.last_justified_slot
    finalized = cstate.last_finalized_slot
    lsr = cstate.last_state_recalc
    recent = recent_block_hashes(astate)
    for i in range(CYCLE_LENGTH):
        slot = (lsr - CYCLE_LENGTH + i) & M64
        bh = recent[i]
        bal = cache[bh][1] if bh in cache else 0
        if (3 * bal) & M64 >= (2 * cstate.total_deposits) & M64:
            if slot > justified:
                justified = slot
            streak = (streak + 1) & M64
        else:
            streak = 0
        if streak >= CYCLE_LENGTH + 1 and ((slot - CYCLE_LENGTH) & M64) > finalized:
            finalized = (slot - CYCLE_LENGTH) & M64

    pending = list(astate.pending_attestations)
    process_crosslinks(cstate, cstate.crosslink_records, cstate.validators, pending,
                       cstate.current_dynasty, block_slot)
    new_pending = [a for a in pending if a.slot > lsr]
    calculate_rewards(pending, cstate.validators, cstate.current_dynasty, cstate.total_deposits)
    nxt = 0
    for idx in active_validator_indices(cstate.validators, cstate.current_dynasty):
        nxt = (nxt + cstate.validators[idx].balance) & M64

    nc = pb.CrystallizedState()
    nc.validators.extend(cstate.validators)
    nc.last_state_recalc = (lsr + CYCLE_LENGTH) & M64
    nc.shard_and_committees_for_slots.extend(cstate.shard_and_committees_for_slots)
    nc.last_justified_slot = justified
    nc.justified_streak = streak
    nc.last_finalized_slot = finalized
    nc.crosslinking_start_shard = 0
    nc.crosslink_records.extend(cstate.crosslink_records)
    nc.dynasty_seed_last_reset = cstate.dynasty_seed_last_reset
    nc.total_deposits = nxt

    hashes = []
    for h in recent:
        hashes.append(h)
        while len(hashes) > 2 * CYCLE_LENGTH:
            hashes = hashes[1:]
    na = pb.ActiveState()
    na.pending_attestations.extend(new_pending)
    na.recent_block_hashes.extend(hashes)
    return nc, na


def compute_new_active_state(astate, attestations, block_hash32):
    """blockchain/core.go:223-237 (vote cache handled by the caller)."""
    astate.pending_attestations.extend(attestations)
    hashes = recent_block_hashes(astate) + [bytes(block_hash32)]
    while len(hashes) > 2 * CYCLE_LENGTH:
        hashes = hashes[1:]
    del astate.recent_block_hashes[:]
    astate.recent_block_hashes.extend(hashes)
    return astate
