"""The library's own multi-GPU layer (include/prysm_hip.h "multi-GPU"): pz_epoch_state stepped
inside the C ABI, sharded by validator range over a pz_comm, bit-exact against the oracle.

On a one-GPU box the sharded path runs over the loopback communicator (every rank on cuda:0,
collectives by device copies + a sum kernel): the shard ranges, local committees with their
bitfield positions, the two-part pipeline, the active-mask all-gather and the next-cycle
all-reduce are the same code RCCL drives.  RCCL itself is exercised at world 1
(pz_init_devices(1)); the multi-process RCCL form is what bench.py --gpus N runs."""
import hashlib

import numpy as np
import pytest

from oracle import epoch_np as onp
from oracle import ref
from prysm_amd import _lib, casper, synth
from prysm_amd.native import Comm, NativeEpoch

from epoch_ref_helpers import oracle_epoch

pytestmark = pytest.mark.gpu


def _inst(n, B, inactive, seed=5, **kw):
    shuffled = casper.shuffle_indices(ref.bytes_to_hash(b"A"), np.arange(n, dtype=np.uint32))
    inst = synth.epoch_batch(n, B, seed=seed, shuffled=shuffled, **kw)
    if inactive:  # rank != index: the compaction / gathered-mask path
        rng = np.random.default_rng(1)
        inst["start"][:, rng.random(n) < 0.1] = 7
        inst["end"][:, rng.random(n) < 0.1] = 1
    return inst


def _check(ne, inst, steps=1):
    for _ in range(steps):
        ne.step()
        ne.sync()
        ne.tallies()  # sharded one-pass: vote/total complete on every rank (no-op otherwise)
        want = [oracle_epoch(inst, b) for b in range(inst["ninst"])]
        held = []
        for local in range(ne.nlocal):
            idx = ne.validators(local)
            held.append(idx)
            bal, scal, vote, total, win = ne.results(local)
            for b, (nb, applied, nxt, v, t, w) in enumerate(want):
                assert bool(scal[b, _lib.SCAL_APPLIED]) == applied, (local, b)
                np.testing.assert_array_equal(bal[b], nb[idx])
                assert int(scal[b, _lib.SCAL_NEXT_BAL]) == nxt, (local, b)
                np.testing.assert_array_equal(vote[b], v)
                np.testing.assert_array_equal(total[b], t)
                np.testing.assert_array_equal(win[b], w)
        if ne.comm is None or ne.nlocal == ne.comm.world:  # every validator held exactly once
            np.testing.assert_array_equal(np.sort(np.concatenate(held)), np.arange(inst["nval"]))
        for b, (nb, *_rest) in enumerate(want):
            inst["balance"][b] = nb


LAYOUTS = ["auto", "twopass", "index"]


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("n,B,inactive", [(65536, 3, False), (5000, 2, True), (4096, 9, False), (3000, 5, True),
                                          (4097, 2, False), (1000, 3, False), (130, 2, False), (1 << 20, 2, False)])
def test_native_epoch_single_device(n, B, inactive, layout):
    inst = _inst(n, B, inactive)
    ne = NativeEpoch(inst, device=0, layout=layout)
    # committee order whenever every validator is active (the synthetic committees partition);
    # the one-pass step on it when every shard id is in range
    assert ne.committee_order == (layout != "index" and not inactive)
    assert ne.one_pass == (layout == "auto" and not inactive)
    _check(ne, inst, steps=2)


@pytest.mark.parametrize("n", [65536, 32768, 16385, 4096, 4097, 1000, 130])
@pytest.mark.parametrize("density", [0.5, 0.75])
def test_native_epoch_single_launch(n, density):
    """One instance on one device, three steps in a row (tickets, the winners' ping-pong and
    the next step's tallies are reset in-kernel), bit-exact: the single-launch step
    (pz_epoch_one_kernel) when every attested committee is one piece, else the window pass (32,768
    validators give 256-member committees, some of them two pieces)."""
    inst = _inst(n, 1, False, density=density)
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass
    _check(ne, inst, steps=3)


def _rebits(inst, seed=9):
    """New random bitfields sized to the (changed) committees: attestation g < ncomm covers
    committee g, the final one all N validators; trailing bits clear (core.go:384-392)."""
    rng = np.random.default_rng(seed)
    B, natt, N = inst["ninst"], inst["natt"], inst["nval"]
    sizes = np.diff(inst["coffs"].astype(np.int64))
    kb = np.concatenate([sizes, [N]])
    blobs, offs = [], [0]
    for b in range(B):
        for g in range(natt):
            k = int(kb[g])
            nb = (k + 7) // 8
            x = (rng.integers(0, 256, size=nb, dtype=np.uint8) | rng.integers(0, 256, size=nb, dtype=np.uint8))
            if k % 8:
                x[-1] &= (0xFF << (8 - k % 8)) & 0xFF
            blobs.append(x)
            offs.append(offs[-1] + nb)
    inst["bits"] = np.concatenate(blobs)
    inst["boffs"] = np.array(offs, dtype=np.uint64)
    inst["max_inst_bytes"] = int(max(offs[(b + 1) * natt] - offs[b * natt] for b in range(B)))
    return inst


def _widen(inst, bal=False, dyn=None):
    """Data that selects the window pass's other column forms: balances 2^30 apart (the u64
    column), a CurrentDynasty at or past 0xFFFF (the 32-bit bounds) or 2^32 - 1 (the u64 bounds)."""
    if bal:
        inst["balance"][:, :3] = np.array([1, 1 << 31, 1 << 40], dtype=np.uint64)
    if dyn is not None:
        inst["dynasty"] = np.full(inst["ninst"], dyn, dtype=np.uint64)
    return inst


@pytest.mark.parametrize("bal", [False, True])
@pytest.mark.parametrize("dyn,db", [(None, 4), (0xFFFF, 8), ((1 << 32) + 3, 16)])
@pytest.mark.parametrize("n,B", [(65536, 5), (32768, 9), (4097, 3), (1000, 2)])
def test_native_epoch_window_forms(n, B, bal, dyn, db):
    """The window pass's six column forms, each selected by the data: balances as u32 offsets or
    u64 (a spread of 2^30 or more), {start, end} at 16, 32 or 64 bits (by CurrentDynasty); three
    steps each, bit-exact against the oracle."""
    inst = _widen(_inst(n, B, False), bal=bal, dyn=dyn)
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass and (ne.balance_bytes, ne.dynasty_bytes) == (8 if bal else 4, db)
    _check(ne, inst, steps=3)


@pytest.mark.parametrize("n,B,last_bits", [(65536, 3, 1 << 21), (4097, 2, 1 << 21), (1 << 20, 2, (1 << 20) + 8)])
def test_native_epoch_window_reward_bits_from_l2(n, B, last_bits):
    """A last bitfield longer than the block's LDS can hold next to its tables (256 KiB here;
    CalculateRewards reads only its first N bits): the window pass looks the reward bits up in
    L2 instead (the kernels' _g form); at 1M validators with a 128 KiB bitfield, the LDS form
    beside it.  Bit-exact over two steps."""
    inst = _inst(n, B, False, last_bits=last_bits)
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass
    _check(ne, inst, steps=2)


@pytest.mark.parametrize("n,B,density", [(65536, 5, 0.75), (1 << 20, 2, 0.75), (4097, 3, 0.5), (1000, 2, 0.75)])
def test_native_epoch_bal32_offsets(n, B, density):
    """The product's multi-instance layout: balances as u32 offsets from a per-instance u64 base
    (pz_epoch_state_columns reports 4 B), three steps against the oracle."""
    inst = _inst(n, B, False, density=density)
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass and (ne.balance_bytes, ne.dynasty_bytes) == (4, 4)
    _check(ne, inst, steps=3)


def test_native_epoch_bal32_rebase():
    """The offsets re-based every 2 steps (pz_epoch_options.rebase_period; 2^29 in the
    product): five steps, each compared with the oracle."""
    inst = _inst(65536, 3, False)
    ne = NativeEpoch(inst, device=0, rebase_period=2)
    assert ne.balance_bytes == 4
    _check(ne, inst, steps=5)


def test_native_epoch_bal32_wide_spread():
    """An instance whose balances span 2^30 or more keeps the u64 column (the widest part is
    reported); the instances beside it are unaffected; bit-exact."""
    inst = _inst(4096, 3, False)
    inst["balance"][1, :7] = np.array([1, 1 << 30, 5, 1 << 40, 2, 3, 9999999999999999999], dtype=np.uint64)
    ne = NativeEpoch(inst, device=0)
    assert ne.balance_bytes == 8
    _check(ne, inst, steps=2)


def test_native_epoch_bal32_wrap_below_zero():
    """Balances of 0 and 1 under penalties wrap below zero as Go's uint64 does (2^64 - 1):
    exact in the offsets (mod 2^64); the re-base after the wrap finds the spread too wide and
    the state returns to the u64 column; three steps against the oracle."""
    inst = _inst(4096, 3, False, density=0.75)
    rng = np.random.default_rng(4)
    inst["balance"][:] = rng.integers(0, 2, size=inst["balance"].shape, dtype=np.uint64)
    ne = NativeEpoch(inst, device=0, rebase_period=1)
    assert ne.balance_bytes == 4
    _check(ne, inst, steps=3)
    assert (inst["balance"] > (1 << 63)).any()  # some balance wrapped


@pytest.mark.parametrize("case", ["reward_panic", "short_bitfield", "many_atts"])
def test_native_epoch_single_launch_edges(case):
    """The single-launch step's panics (CheckBit(last, N-1), a bitfield shorter than its
    committee: scal flags, balances untouched) and a committee with two attestations (the
    per-attestation atomics), against the oracle or the three-launch step."""
    n = 4096
    inst = _inst(n, 1, False, last_bits=n - 8 if case == "reward_panic" else None)
    if case == "short_bitfield":
        bo = inst["boffs"].astype(np.int64)
        inst["bits"] = np.delete(inst["bits"], int(bo[3]) - 1)
        bo[3:] -= 1
        inst["boffs"] = bo.astype(np.uint64)
    if case == "many_atts":  # the final (N-bit) attestation names committee 0 too
        inst["att_comm"] = inst["att_comm"].copy()
        inst["att_comm"][-1] = 0
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass
    if case == "many_atts":
        _check(ne, inst, steps=2)
        return
    ne.step()
    bal, scal, vote, total, _ = ne.results()
    assert scal[0, _lib.SCAL_APPLIED] == 0
    np.testing.assert_array_equal(bal[0], inst["balance"][0][ne.validators()])
    if case == "reward_panic":
        assert scal[0, _lib.SCAL_ERR_RWD] != 0
    else:
        assert int(scal[0, _lib.SCAL_ERR_XL]) == 2  # PZ_XLERR_BITFIELD


@pytest.mark.parametrize("n", [65536, 4096])
def test_native_epoch_single_launch_matches_window_pass(n):
    """The same instance stepped by the single launch (pz_epoch_one_kernel) and by the window
    pass (pz_epoch_options.window_only): identical balances, scalars, tallies and winners over
    two steps."""
    inst = _inst(n, 1, False)
    outs = []
    for wo in (False, True):
        k = {key: (val.copy() if isinstance(val, np.ndarray) else val) for key, val in inst.items()}
        ne = NativeEpoch(k, device=0, window_only=wo)
        for _ in range(2):
            ne.step()
        outs.append(ne.results())
        ne.free()
    for x, y in zip(*outs):
        np.testing.assert_array_equal(x, y)


@pytest.mark.ab
@pytest.mark.parametrize("abl", [16, 48, 8192, 32])
@pytest.mark.parametrize("n,B,short", [(65536, 5, False), (1 << 20, 2, False), (4096, 3, True)])
def test_native_epoch_window_meeting_fallbacks(abl, n, B, short):
    """The A/B meeting of an instance's R blocks (each counts 1/R of the bitfields, epoch_window.hip
    WinArgs.pacc; 16) and its fallback (48: the wait bound at zero, so a block that arrives
    before its partners counts the whole instance itself); the whole count before the loop
    (8192, no speculation); the speculating product's post-loop fallback count taken every
    time (32); each exact.  Two steps against the oracle; or one with a short committee bitfield in
    instance 0 (its flags, its balances untouched)."""
    dll = _lib.lib.dll
    old = dll.pz_debug_set_window_ablation(abl)
    try:
        inst = _inst(n, B, False)
        if short:
            bo = inst["boffs"].astype(np.int64)
            inst["bits"] = np.delete(inst["bits"], int(bo[3]) - 1)
            bo[3:] -= 1
            inst["boffs"] = bo.astype(np.uint64)
        ne = NativeEpoch(inst, device=0)
        assert ne.one_pass and (ne.balance_bytes, ne.dynasty_bytes) == (4, 4)
        if not short:
            _check(ne, inst, steps=2)
            return
        ne.step()
        bal, scal, _, _, _ = ne.results()
        assert scal[0, _lib.SCAL_APPLIED] == 0 and int(scal[0, _lib.SCAL_ERR_XL]) == 2
        np.testing.assert_array_equal(bal[0], inst["balance"][0][ne.validators()])
        for b in range(1, B):
            nb, applied, nxt, v, t, w = oracle_epoch(inst, b)
            assert bool(scal[b, _lib.SCAL_APPLIED]) == applied
    finally:
        dll.pz_debug_set_window_ablation(old)


@pytest.mark.parametrize("case", ["ok", "threshold", "short_bitfield", "reward_panic"])
def test_native_epoch_window_one_range(case):
    """256 instances (one block each, R = 1, the bench's configs[2] geometry): the whole count
    before the loop, no meeting; the threshold missed (half the bits set), a short committee
    bitfield in instance 0 and the CheckBit(last, N-1) panic.  Two steps against the oracle, or
    the flags and untouched balances."""
    n, B = 1024, 256
    inst = _inst(n, B, False, density=0.5 if case == "threshold" else 0.75,
                 last_bits=n - 8 if case == "reward_panic" else None)
    if case == "short_bitfield":
        bo = inst["boffs"].astype(np.int64)
        inst["bits"] = np.delete(inst["bits"], int(bo[3]) - 1)
        bo[3:] -= 1
        inst["boffs"] = bo.astype(np.uint64)
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass
    if case in ("ok", "threshold"):
        _check(ne, inst, steps=2)
        return
    ne.step()
    bal, scal, _, _, _ = ne.results()
    for b in range(B if case == "reward_panic" else 1):
        assert scal[b, _lib.SCAL_APPLIED] == 0
        np.testing.assert_array_equal(bal[b], inst["balance"][b][ne.validators()])
    if case == "short_bitfield":
        assert int(scal[0, _lib.SCAL_ERR_XL]) == 2
        for b in range(1, 4):
            nb, applied, nxt, v, t, w = oracle_epoch(inst, b)
            assert bool(scal[b, _lib.SCAL_APPLIED]) == applied
            np.testing.assert_array_equal(bal[b], nb[ne.validators()])


@pytest.mark.parametrize("case", ["many_atts", "short_bitfield", "reward_panic", "empty_committees"])
@pytest.mark.parametrize("B", [1, 3])
def test_native_epoch_window_edges(case, B):
    """The window pass on the single-launch edge cases and more: a committee with two
    attestations besides the final one (the per-attestation path), a bitfield shorter than its
    committee and the CheckBit(last, N-1) panic (flags, balances untouched), and empty
    committees (an attestation with nobody to count: total 0 qualifies under 3 * 0 >= 2 * 0);
    against the oracle."""
    n = 4096
    inst = _inst(n, B, False, last_bits=n - 8 if case == "reward_panic" else None)
    natt = inst["natt"]
    if case == "many_atts":  # each instance's final (N-bit) attestation names committee 0 too
        inst["att_comm"] = inst["att_comm"].copy()
        inst["att_comm"][natt - 1::natt] = 0
    if case == "short_bitfield":
        bo = inst["boffs"].astype(np.int64)
        inst["bits"] = np.delete(inst["bits"], int(bo[3]) - 1)
        bo[3:] -= 1
        inst["boffs"] = bo.astype(np.uint64)
    if case == "empty_committees":  # committees 5 and 9 emptied into their predecessors
        coffs = inst["coffs"].astype(np.int64)
        coffs[5] = coffs[6]
        coffs[9] = coffs[10]
        inst["coffs"] = coffs.astype(np.uint64)
        _rebits(inst)
    ne = NativeEpoch(inst, device=0, window_only=True)
    assert ne.one_pass
    if case in ("many_atts", "empty_committees"):
        _check(ne, inst, steps=2)
        return
    ne.step()
    bal, scal, vote, total, _ = ne.results()
    for b in range(B if case == "reward_panic" else 1):  # (short_bitfield: instance 0's)
        assert scal[b, _lib.SCAL_APPLIED] == 0
        np.testing.assert_array_equal(bal[b], inst["balance"][b][ne.validators()])
        if case == "reward_panic":
            assert scal[b, _lib.SCAL_ERR_RWD] != 0
        else:
            assert int(scal[b, _lib.SCAL_ERR_XL]) == 2  # PZ_XLERR_BITFIELD


@pytest.mark.parametrize("B", [1, 3])
def test_native_epoch_one_pass_dynasty_past_32_bits(B):
    """A CurrentDynasty of 2^32 - 1 or more: the state keeps the 64-bit {start, end} stream (the
    packed 32-bit column classifies exactly only below it); same results as the oracle, on the
    single launch (B = 1) and the pre + fused + mid step."""
    inst = _inst(4096, B, False)
    inst["dynasty"] = np.full(B, (1 << 32) + 3, dtype=np.uint64)
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass
    _check(ne, inst, steps=2)


def _record_dynasties(d):
    """Crosslink record dynasties around CurrentDynasty d (core.go:549, dynasty > record.Dynasty):
    d - 1 and 0 (beaten), d and d + 1 (not), 0xFFFFFFFF and 2^32 + k with k's low word below
    d's (the window pass's 32-bit saturated compare and its high-word table), 2^33 + 1."""
    c = [0, d - 1, d, d + 1, 0xFFFFFFFF, (1 << 32) + 1, (1 << 33) + 1]
    return np.array(sorted(set(x for x in c if 0 <= x < (1 << 64))), dtype=np.uint64)


@pytest.mark.parametrize("window_only", [True, False])
@pytest.mark.parametrize("B", [1, 3])
@pytest.mark.parametrize("d", [5, 0xFFFFFFFE, (1 << 32) + 3])
def test_native_epoch_record_dynasties(d, B, window_only):
    """The winner rule's dynasty compare against nonzero crosslink records: each
    instance's records drawn from values just below, at and above CurrentDynasty and around the
    32-bit saturation point, so some qualifying attestations beat their shard's record and some
    do not; the window pass (window_only, and B = 3) and the single launch (B = 1), two steps
    against oracle/epoch_np.crosslink_winners."""
    inst = _inst(4096, B, False)
    rng = np.random.default_rng(11)
    inst["dynasty"] = np.full(B, d, dtype=np.uint64)
    inst["rec_dynasty"] = rng.choice(_record_dynasties(d), size=inst["rec_dynasty"].shape)
    ne = NativeEpoch(inst, device=0, window_only=window_only)
    assert ne.one_pass
    want = [oracle_epoch(inst, b) for b in range(B)]
    # the draw must leave both outcomes: a qualifying attestation that wins and one its record blocks
    natt = inst["natt"]
    won = sum(int((w != 0xFFFFFFFF).sum()) for *_r, w in want)
    blocked = 0
    for b, (_nb, _a, _n, v, t, w) in enumerate(want):
        q = 3 * v.astype(object) >= 2 * t.astype(object)
        sh = inst["att_shard"][b * natt:(b + 1) * natt]
        blocked += int(sum(1 for g in np.nonzero(q)[0] if not d > int(inst["rec_dynasty"][b][sh[g]])))
    assert won > 0 and blocked > 0, (won, blocked)
    _check(ne, inst, steps=2)


@pytest.mark.parametrize("B", [1, 3])
@pytest.mark.parametrize("d", [0xFFFE, 0xFFFF, 0xFFFFFFFE])
def test_native_epoch_one_pass_saturated_bounds(B, d):
    """The stream's narrow {start, end} columns classify exactly at their limits: CurrentDynasty
    just below 0xFFFF (the 16-bit saturated column), at 0xFFFF and just below 2^32 - 1 (the 32-bit
    one), with start and end drawn around both saturation values (start <= d < end everywhere, so
    the committee order and the one-pass step hold), on the single launch and on pre + fused +
    mid, two steps against the oracle."""
    inst = _inst(4096, B, False)
    rng = np.random.default_rng(2)
    inst["dynasty"] = np.full(B, d, dtype=np.uint64)
    inst["start"] = rng.choice(np.array([0, 1, d - 1, d], dtype=np.uint64), size=inst["start"].shape)
    ends = np.array([d + 1, 0xFFFF, 0x10000, 0xFFFFFFFF, 1 << 32, 1 << 40, 9999999999999999999], dtype=np.uint64)
    inst["end"] = rng.choice(ends[ends > d], size=inst["end"].shape)
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass
    _check(ne, inst, steps=2)


@pytest.mark.parametrize("density", [0.5, 0.75])
def test_native_epoch_one_pass_threshold(density):
    """Half the bits set: GetAttestersTotalDeposit stays under 2/3 of TotalDeposits, so no
    reward is applied (incentives.go:18-20) while the tallies and winners still form."""
    inst = _inst(8192, 4, False, density=density)
    ne = NativeEpoch(inst, device=0)
    assert ne.one_pass
    _check(ne, inst, steps=2)


def test_native_epoch_one_pass_reward_panic():
    """The last bitfield shorter than the validator set with the threshold met: CheckBit(last,
    N-1) panics in CalculateRewards (incentives.go:23): PZ_SCAL_ERR_RWD, balances untouched, in
    every layout."""
    n = 4096
    inst = _inst(n, 3, False, last_bits=n - 8)
    for layout in LAYOUTS:
        k = {key: (v.copy() if isinstance(v, np.ndarray) else v) for key, v in inst.items()}
        ne = NativeEpoch(k, device=0, layout=layout)
        assert ne.one_pass == (layout == "auto")
        ne.step()
        bal, scal, vote, total, _ = ne.results()
        for b in range(3):
            assert scal[b, _lib.SCAL_ERR_RWD] != 0, (layout, b)
            assert scal[b, _lib.SCAL_APPLIED] == 0, (layout, b)
            np.testing.assert_array_equal(bal[b], k["balance"][b][ne.validators()])
            natt = k["natt"]  # the tallies are formed before the panic
            v, t = onp.crosslink_tallies(k["committee"], k["coffs"], k["att_comm"][b * natt:(b + 1) * natt],
                                         k["bits"], k["boffs"][b * natt:(b + 1) * natt + 1], k["balance"][b])
            np.testing.assert_array_equal(vote[b], v)
            np.testing.assert_array_equal(total[b], t)


def test_native_epoch_shard_out_of_range_two_pass():
    """An attestation naming a shard >= nrec: that processCrosslinks panic depends on the
    tallies (core.go:549), so the state keeps the two-pass step; with the vote under 2/3 there
    is no panic and the step is bit-exact."""
    inst = _inst(4096, 2, False)
    inst["att_shard"] = inst["att_shard"].copy()
    inst["att_shard"][0] = 5000  # > nrec (1024); its committee's vote must fail the threshold
    natt = inst["natt"]
    bo = inst["boffs"]
    inst["bits"] = inst["bits"].copy()
    inst["bits"][int(bo[0]):int(bo[1])] = 0
    ne = NativeEpoch(inst, device=0)
    assert ne.committee_order and not ne.one_pass
    _check(ne, inst)
    assert natt > 1


def test_native_epoch_committee_order_fallback():
    """A validator in two committees (the committees no longer partition the set): index order,
    still bit-exact."""
    inst = _inst(4096, 2, False)
    inst["committee"] = inst["committee"].copy()
    inst["committee"][7] = inst["committee"][8]
    ne = NativeEpoch(inst, device=0)
    assert not ne.committee_order
    _check(ne, inst)


def test_native_epoch_committee_order_short_bitfield():
    """Committee order with a bitfield one byte short of its committee: the bitfield panic
    (core.go:538, PZ_XLERR_BITFIELD) is raised and no balance changes, as in index order."""
    inst = _inst(4096, 2, False)
    for layout in LAYOUTS:
        k = {key: (v.copy() if isinstance(v, np.ndarray) else v) for key, v in inst.items()}
        bo = k["boffs"].astype(np.int64)
        cut = int(bo[3]) - 1  # drop the last byte of attestation 2 of instance 0
        k["bits"] = np.delete(k["bits"], cut)
        bo[3:] -= 1
        k["boffs"] = bo.astype(np.uint64)
        ne = NativeEpoch(k, device=0, layout=layout)
        assert ne.committee_order == (layout != "index")
        assert ne.one_pass == (layout == "auto")
        ne.step()
        bal, scal, *_ = ne.results()
        assert scal[0, _lib.SCAL_ERR_XL] & 2, layout  # PZ_XLERR_BITFIELD
        assert scal[0, _lib.SCAL_APPLIED] == 0
        np.testing.assert_array_equal(bal[0], k["balance"][0][ne.validators()])


@pytest.mark.parametrize("ndev", [2, 8])
def test_native_epoch_sharded_multi_device(ndev):
    """configs[3]-shaped instances sharded over RCCL across ``ndev`` real GPUs of one process
    (pz_init_devices), two steps against the oracle; skipped where fewer GPUs are visible."""
    import torch
    if torch.cuda.device_count() < ndev:
        pytest.skip("needs %d GPUs" % ndev)
    inst = _inst(1 << 20, 2, False)
    ne = NativeEpoch(inst, device=0, comm=Comm.devices(ndev))
    _check(ne, inst, steps=2)


def test_native_epoch_rccl_world1():
    comm = Comm.devices(1)
    assert (comm.world, comm.nlocal) == (1, 1)
    inst = _inst(8192, 4, True)
    _check(NativeEpoch(inst, comm=comm), inst, steps=2)


@pytest.mark.parametrize("world,n,B,inactive", [(2, 65536, 3, False), (2, 20000, 2, True), (3, 5000, 4, True),
                                                (8, 20000, 1, True), (5, 3000, 7, False), (3, 4099, 4, False),
                                                (7, 1001, 3, False)])
@pytest.mark.parametrize("layout", LAYOUTS)
def test_native_epoch_sharded_loopback(world, n, B, inactive, layout):
    comm = Comm.loopback(world)
    inst = _inst(n, B, inactive)
    _check(NativeEpoch(inst, comm=comm, layout=layout), inst, steps=2)


@pytest.mark.parametrize("inactive,layout", [(False, "auto"), (False, "twopass"), (False, "index"), (True, "auto")])
def test_native_epoch_configs3_world8_loopback(inactive, layout):
    """BASELINE configs[3]: 1,048,576 validators over 8 ranks (131,072 each), 65 committees per
    slot, through the library's sharded step."""
    inst = _inst(1 << 20, 2, inactive)
    _check(NativeEpoch(inst, comm=Comm.loopback(8), layout=layout), inst)


@pytest.mark.parametrize("world", [2, 3])
def test_native_epoch_one_pass_bitfield_panic_sharded(world):
    """A short bitfield under the sharded one-pass step: the flag (raised once, by rank 0's
    pre pass) survives the all-reduce and no rank changes a balance."""
    inst = _inst(4096, 3, False)
    bo = inst["boffs"].astype(np.int64)
    natt = inst["natt"]
    cut = int(bo[natt + 4]) - 1  # instance 1, attestation 3
    inst["bits"] = np.delete(inst["bits"], cut)
    bo[natt + 4:] -= 1
    inst["boffs"] = bo.astype(np.uint64)
    ne = NativeEpoch(inst, comm=Comm.loopback(world))
    assert ne.one_pass
    ne.step()
    for local in range(world):
        bal, scal, *_ = ne.results(local)
        assert int(scal[1, _lib.SCAL_ERR_XL]) == 2  # PZ_XLERR_BITFIELD, once
        assert scal[1, _lib.SCAL_APPLIED] == 0
        np.testing.assert_array_equal(bal[1], inst["balance"][1][ne.validators(local)])
        for b in (0, 2):
            nb, applied, nxt, *_ = oracle_epoch(inst, b)
            assert bool(scal[b, _lib.SCAL_APPLIED]) == applied and int(scal[b, _lib.SCAL_NEXT_BAL]) == nxt
            np.testing.assert_array_equal(bal[b], nb[ne.validators(local)])


def test_native_epoch_panic_flags_sharded():
    """A committee member beyond the validator set: Go panics in processCrosslinks
    (core.go:535); rank 0 keeps the out-of-range member, the flag survives the all-reduce and
    no balance changes on any rank."""
    inst = _inst(4096, 2, False)
    inst["committee"] = inst["committee"].copy()
    inst["committee"][5] = 4096 + 17
    ne = NativeEpoch(inst, comm=Comm.loopback(3))
    ne.step()
    for local in range(3):
        lo, hi, _, _ = ne.shard(local)
        bal, scal, *_ = ne.results(local)
        assert ((scal[:, _lib.SCAL_ERR_XL] & 1) == 1).all()  # PZ_XLERR_MEMBER
        assert scal[:, _lib.SCAL_APPLIED].sum() == 0
        np.testing.assert_array_equal(bal, inst["balance"][:, lo:hi])


@pytest.mark.parametrize("world", [1, 3])
def test_comm_hash_batch_loopback(world):
    rng = np.random.default_rng(world)
    lens = rng.integers(0, 700, size=1001)
    msgs = [rng.bytes(int(k)) for k in lens]
    offs = np.zeros(len(msgs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    data = np.frombuffer(b"".join(msgs) + bytes(16), dtype=np.uint8)
    got = Comm.loopback(world).hash_batch(data, offs, 32)
    for i, m in enumerate(msgs):
        assert got[i].tobytes() == hashlib.blake2b(m).digest()[:32], i


def test_comm_hash_batch_rccl_world1():
    msgs = [bytes([i & 255]) * (i * 7) for i in range(300)]
    offs = np.zeros(len(msgs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(m) for m in msgs])
    data = np.frombuffer(b"".join(msgs) + bytes(16), dtype=np.uint8)
    got = Comm.devices(1).hash_batch(data, offs, 64)
    assert [g.tobytes() for g in got] == [hashlib.blake2b(m).digest() for m in msgs]


def test_unique_id_and_shutdown():
    """ncclCommInitRank through the C ABI, then pz_shutdown (in a child process: it frees the
    library's device contexts, which other tests' live objects may still hold)."""
    import subprocess
    import sys
    code = r"""
import hashlib, sys
sys.path.insert(0, %r)
from prysm_amd import _lib
from prysm_amd.native import Comm
uid = Comm.unique_id()
assert len(uid) == 128
c = Comm.rank(uid, 1, 0, 0)
assert (c.world, c.nlocal, c.first_rank) == (1, 1, 0)
c.free()
assert _lib.blake2b512_batch([b"abc"], 64)[0] == hashlib.blake2b(b"abc").digest()
_lib.lib.dll.pz_shutdown()
assert _lib.blake2b512_batch([b"abcd"], 64)[0] == hashlib.blake2b(b"abcd").digest()
print("ok")
""" % (_lib.HERE.rsplit("/", 1)[0],)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stderr[-2000:]


def test_max_active_index_scalar():
    """PZ_SCAL_MAXIDX1 (1 + the largest active index) with the maximum at a block edge, in
    the last block, inside a block, and with no active validator."""
    n = 10000
    inst = _inst(n, 4, False)
    d = 1
    inst["start"][1, 2048:] = 7          # last active = 2047, the last validator of block 0
    rng = np.random.default_rng(3)
    inst["end"][2, rng.random(n) < 0.3] = 1
    inst["end"][2, 9000:] = 1            # last active inside block 4
    inst["start"][3, :] = 9              # nothing active
    ne = NativeEpoch(inst, device=0)
    ne.step()
    _, scal, *_ = ne.results()
    for b in range(4):
        act = np.nonzero((inst["start"][b] <= d) & (d < inst["end"][b]))[0]
        assert int(scal[b, _lib.SCAL_MAXIDX1]) == (int(act[-1]) + 1 if act.size else 0), b
        assert int(scal[b, _lib.SCAL_NACT]) == act.size


@pytest.mark.parametrize("world", [2, 3])
def test_native_epoch_tallies_twice_is_idempotent(world):
    """pz_epoch_state_tallies sums the owner ranks' vote/total once per step; a second
    call in the same step returns the same (complete) tallies, not world x them, and the next
    step's call sums that step's tallies again."""
    inst = _inst(20000, 2, False)
    ne = NativeEpoch(inst, comm=Comm.loopback(world))
    assert ne.one_pass
    for _ in range(2):
        ne.step()
        ne.tallies()
        ne.tallies()
        want = [oracle_epoch(inst, b) for b in range(2)]
        for local in range(world):
            _, _, vote, total, _ = ne.results(local)
            for b, (nb, _a, _n, v, t, _w) in enumerate(want):
                np.testing.assert_array_equal(vote[b], v)
                np.testing.assert_array_equal(total[b], t)
        for b, (nb, *_rest) in enumerate(want):
            inst["balance"][b] = nb


def test_native_epoch_sharded_ranges_are_committee_aligned():
    """The sharded one-pass step splits the committee-order positions at committee starts: no
    committee straddles two ranks, and without pz_epoch_state_tallies a rank's vote/total are
    complete exactly for the attestations whose committee it holds (zero elsewhere)."""
    inst = _inst(20000, 2, False)
    world = 3
    ne = NativeEpoch(inst, comm=Comm.loopback(world))
    assert ne.one_pass
    coffs = inst["coffs"].astype(np.int64)
    starts = []
    for local in range(world):
        lo, hi, _, _ = ne.shard(local)
        starts.append(lo)
        assert lo in set(coffs.tolist()) and hi in set(coffs.tolist())
    ne.step()
    ne.sync()
    natt = inst["natt"]
    for local in range(world):
        lo, hi, _, _ = ne.shard(local)
        _, _, vote, total, win = ne.results(local)
        for b in range(2):
            _, _, _, v, t, w = oracle_epoch(inst, b)
            cb = coffs[inst["att_comm"][b * natt:(b + 1) * natt]]
            own = (cb >= lo) & ((cb < hi) | ((cb == 20000) & (hi == 20000)))
            np.testing.assert_array_equal(vote[b][own], v[own])
            np.testing.assert_array_equal(total[b][own], t[own])
            np.testing.assert_array_equal(np.where(own, 0, vote[b]), 0)
            np.testing.assert_array_equal(win[b], w)  # winners exact on every rank
