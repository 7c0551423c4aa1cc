"""TEST DOUBLE (test infrastructure only): a numpy model of ONE rank of the sharded one-pass
epoch step (prysm_amd/csrc/epoch_state.hip step_sharded_fused; kernels epoch.hip
pz_epoch_pre_kernel / fused_body / pz_epoch_fwin_kernel), so that its collective protocol
runs under ``gloo`` on CPU with no GPU:

* the rank holds committee-order positions [lo, hi) from ``pz_epoch_plan`` (the library's
  own host planner: committee-aligned, so no committee straddles two ranks);
* it classifies, tallies every attestation of the committees it holds on the PRE-reward
  balances, rewards (bit ``co_index[p]`` of the last bitfield, blockchain/core.go:433-441 ->
  casper/incentives.go:14-32) and sums the post-reward balances (core.go:459-464);
* it proposes crosslink winners (core.go:547-555) only for the attestations whose committee
  it owns (the committee's first position in [lo, hi); the last rank for an empty committee
  at the end);
* one u64 SUM of the scalars and one u32 MIN of the winners combine the ranks; a second SUM
  completes vote/total (``pz_epoch_state_tallies``).

It is never used by the product; tests/test_onepass_multirank.py checks it bit-exact against
the oracle on every rank.
"""
import numpy as np

from oracle.epoch_np import check_bits as _bit
from prysm_amd.params import DEFAULT_BALANCE

U64 = np.uint64
NONE = 0xFFFFFFFF


def rank_step(inst, b, rank, lo, hi):
    """Rank ``rank``'s partial results for instance ``b`` over positions [lo, hi):
    (new balances of co[lo:hi], partial scal {pop, applied, next_bal}, vote, total, proposed
    winners).  Panics are outside the one-pass step's scope (the host keeps the two-pass step
    for a shard panic; bitfield panics are covered by the GPU tests)."""
    N, natt = int(inst["nval"]), int(inst["natt"])
    co = np.asarray(inst["committee"], dtype=np.int64)   # committee order == co_index
    coffs = np.asarray(inst["coffs"], dtype=np.int64)
    bo = np.asarray(inst["boffs"][b * natt:(b + 1) * natt + 1], dtype=np.int64)
    bits = inst["bits"]
    ac = np.asarray(inst["att_comm"][b * natt:(b + 1) * natt], dtype=np.int64)
    ash = np.asarray(inst["att_shard"][b * natt:(b + 1) * natt], dtype=np.int64)
    bal = inst["balance"][b].astype(U64)[co[lo:hi]]  # this rank's rows, in storage order
    dyn, tdep = int(inst["dynasty"][b]), int(inst["total_deposit"][b])
    nrec = inst["rec_dynasty"].shape[-1]
    rec_dyn = np.asarray(inst["rec_dynasty"]).reshape(-1, nrec)[b]

    # pre: bit count of every bitfield (every rank needs it; rank 0 reports it)
    pop = int(np.unpackbits(bits[bo[0]:bo[-1]]).sum())
    # fused: tallies of the committees this rank holds, on the pre-reward balances
    vote = np.zeros(natt, dtype=U64)
    total = np.zeros(natt, dtype=U64)
    with np.errstate(over="ignore"):
        for a in range(natt):
            c0, c1 = coffs[ac[a]], coffs[ac[a] + 1]
            p0, p1 = max(c0, lo), min(c1, hi)
            if p0 >= p1:
                continue
            seg = bal[p0 - lo:p1 - lo]
            total[a] = seg.sum(dtype=U64)
            vote[a] = seg[_bit(bits[bo[a]:bo[a + 1]], np.arange(p0 - c0, p1 - c0))].sum(dtype=U64)
        dep = U64((pop * DEFAULT_BALANCE) & ((1 << 64) - 1))  # casper/validator.go:93-102
        applied = dep * U64(3) >= U64(tdep) * U64(2)
        if applied:  # every validator is active: rank i == index i
            last = bits[bo[-2]:bo[-1]]
            voted = _bit(last, co[lo:hi])
            bal = np.where(voted, bal + U64(1), bal - U64(1))
        nxt = int(bal.sum(dtype=U64))
    # fwin: first qualifying attestation per shard, among those whose committee this rank owns
    win = np.full(nrec, NONE, dtype=np.int64)
    for a in range(natt):
        cb = coffs[ac[a]]
        if not ((lo <= cb < hi) or (cb == N and hi == N)):
            continue
        s = int(ash[a])
        with np.errstate(over="ignore"):
            q = vote[a] * U64(3) >= total[a] * U64(2)
        if q and int(rec_dyn[s]) < dyn and win[s] == NONE:
            win[s] = a
    r0 = rank == 0  # the per-instance scalars the SUM must not multiply
    return bal, pop if r0 else 0, int(applied) if r0 else 0, nxt, vote, total, win
