"""ORACLE (test infrastructure only) — numpy restatement of the epoch T/R path for large N.

Vectorised twins of ``oracle.ref`` (checked against it at small N in
tests/test_oracle_np.py).  SoA inputs: ``start``, ``end``, ``balance`` uint64 arrays;
pending attestations as CSR bitfields ``bits`` (uint8) / ``boffs`` (uint64[natt+1]).
uint64 numpy arithmetic wraps exactly like Go's uint64.
"""
import numpy as np

from oracle.ref import DEFAULT_BALANCE, GoPanic

U64 = np.uint64


def indices(start, end, dynasty, kind):
    """casper/validator.go:45-77 (kind 0 active, 1 exited, 2 queued)."""
    d = U64(dynasty)
    if kind == 0:
        m = (start <= d) & (d < end)
    elif kind == 1:
        m = (start < d) & (end <= d)
    else:
        m = start > d
    return np.nonzero(m)[0].astype(np.uint32)


def bit_count(bits):
    return int(np.unpackbits(np.asarray(bits, dtype=np.uint8)).sum())


def attesters_total_deposit(bits):
    """casper/validator.go:93-102."""
    return (bit_count(bits) * DEFAULT_BALANCE) & ((1 << 64) - 1)


def check_bits(bf, idx):
    """Vectorised utils.CheckBit (MSB-first); GoPanic if any index is out of range."""
    bf = np.asarray(bf, dtype=np.uint8)
    idx = np.asarray(idx, dtype=np.int64)
    if idx.size and (idx.max() >> 3) >= bf.size:
        raise GoPanic("CheckBit index out of range")
    return ((bf[idx >> 3] >> (7 - (idx & 7)).astype(np.uint8)) & 1).astype(bool)


def calculate_rewards(balance, start, end, dynasty, total_deposit, bits, boffs):
    """casper/incentives.go:14-32 on a copy; returns (new balance, applied)."""
    bal = balance.copy()
    active = indices(start, end, dynasty, 0)
    dep = U64(attesters_total_deposit(bits[boffs[0]:boffs[-1]] if len(boffs) else bits[:0]))
    with np.errstate(over="ignore"):
        applied = dep * U64(3) >= U64(total_deposit) * U64(2)
    if applied and active.size:
        if len(boffs) < 2:
            raise GoPanic("index out of range [-1]")
        last = bits[int(boffs[-2]):int(boffs[-1])]
        voted = check_bits(last, active)
        ranks = np.arange(active.size)
        with np.errstate(over="ignore"):
            bal[ranks] = np.where(voted, bal[ranks] + U64(1), bal[ranks] - U64(1))
    return bal, bool(applied)


def active_balance_sum(balance, start, end, dynasty):
    """blockchain/core.go:459-464."""
    a = indices(start, end, dynasty, 0)
    with np.errstate(over="ignore"):
        return int(balance[a].sum(dtype=U64))


def crosslink_tallies(committee, coffs, att_comm, bits, boffs, balance):
    """blockchain/core.go:533-545 -> (vote[natt], total[natt]) uint64."""
    natt = len(att_comm)
    vote = np.zeros(natt, dtype=U64)
    total = np.zeros(natt, dtype=U64)
    for a in range(natt):
        c = int(att_comm[a])
        mem = committee[int(coffs[c]):int(coffs[c + 1])].astype(np.int64)
        if mem.size and mem.max() >= balance.size:
            raise GoPanic("validators index out of range")
        bf = bits[int(boffs[a]):int(boffs[a + 1])]
        b = balance[mem]
        with np.errstate(over="ignore"):
            total[a] = b.sum(dtype=U64)
            voted = check_bits(bf, np.arange(mem.size))
            vote[a] = b[voted].sum(dtype=U64)
    return vote, total


def crosslink_winners(vote, total, att_shard, rec_dynasty, dynasty):
    """blockchain/core.go:547-555 in attestation order -> winner[nrec] (uint32, 0xFFFFFFFF none)."""
    rec = np.array(rec_dynasty, dtype=U64).copy()
    win = np.full(rec.size, 0xFFFFFFFF, dtype=np.uint32)
    with np.errstate(over="ignore"):
        for a in range(len(vote)):
            if U64(3) * vote[a] >= U64(2) * total[a]:
                s = int(att_shard[a])
                if s >= rec.size:
                    raise GoPanic("crosslink record index out of range")
                if U64(dynasty) > rec[s]:
                    rec[s] = U64(dynasty)
                    win[s] = a
    return win
