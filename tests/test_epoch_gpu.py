"""T/R parity: casper filters, attester deposit, rewards, crosslinks, shuffle and the batched
device-resident epoch — HIP path through the C ABI vs the oracle.  Bit-exact (integers)."""
import numpy as np
import pytest

from oracle import epoch_np as onp
from oracle import ref
from oracle import schema as pb
from prysm_amd import _lib, casper, synth
from prysm_amd.params import DEFAULT_END_DYNASTY

from epoch_ref_helpers import oracle_epoch

pytestmark = pytest.mark.gpu
U64 = np.uint64


def _soa(recs):
    return (np.array([r["start"] for r in recs], dtype=U64), np.array([r["end"] for r in recs], dtype=U64),
            np.array([r.get("balance", 0) for r in recs], dtype=U64))


# ---- reference KATs through the GPU -------------------------------------------------------
def test_compute_rewards_kat_gpu():
    # casper/incentives_test.go:9-43
    start = np.ones(40, dtype=U64)
    end = np.full(40, 10, dtype=U64)
    bal = np.full(40, 32, dtype=U64)
    bits = np.array([200, 148, 146, 179, 49], dtype=np.uint8)
    applied = casper.calculate_rewards(bal, start, end, 1, 100, bits, np.array([0, 5], dtype=U64))
    assert applied
    assert bal[0] == 33 and bal[7] == 31 and bal[29] == 31


def test_validator_indices_kat_gpu():
    # casper/validator_test.go:94-141
    inf = 1 << 63
    s, e, _ = _soa([dict(start=0, end=2), dict(start=0, end=2), dict(start=1, end=2), dict(start=0, end=2),
                    dict(start=0, end=3), dict(start=2, end=inf)])
    assert casper.active_validator_indices(s, e, 1).tolist() == [0, 1, 2, 3, 4]
    assert casper.queued_validator_indices(s, e, 1).tolist() == [5]
    assert casper.exited_validator_indices(s, e, 1).tolist() == []
    s, e, _ = _soa([dict(start=1, end=inf), dict(start=2, end=inf), dict(start=6, end=inf), dict(start=7, end=inf),
                    dict(start=1, end=2), dict(start=1, end=3)])
    assert casper.active_validator_indices(s, e, 5).tolist() == [0, 1]
    assert casper.queued_validator_indices(s, e, 5).tolist() == [2, 3]
    assert casper.exited_validator_indices(s, e, 5).tolist() == [4, 5]


def test_rotate_validator_set_kat_gpu():
    # casper/validator_test.go:13-66
    E = DEFAULT_END_DYNASTY
    for specs, act in [([(10, 0), (15, 1), (20, 2), (25, 3), (30, 4), (30, 15)], [2, 3, 4, 5]),
                       ([(10, 0), (15, 1), (20, 2), (25, 3), (30, 4)], [2, 3, 4])]:
        bal = np.array([b for b, _ in specs], dtype=U64)
        start = np.array([s for _, s in specs], dtype=U64)
        end = np.full(len(specs), E, dtype=U64)
        casper.rotate_validator_set(bal, start, end, 10)
        assert casper.active_validator_indices(start, end, 10).tolist() == act
        assert casper.queued_validator_indices(start, end, 10).tolist() == []
        assert casper.exited_validator_indices(start, end, 10).tolist() == [0, 1]


def test_process_crosslinks_kat_gpu():
    # blockchain/core_test.go:979-1024 (genesis chain committees, 100 attestations to shard 0)
    _, cs = ref.new_genesis_states()
    comm = list(cs.shard_and_committees_for_slots[0].array_shard_and_committee[0].committee)
    committee = np.array(comm, dtype=np.uint32)
    coffs = np.array([0, len(comm)], dtype=U64)
    natt = 100
    bits = np.frombuffer(b"zz" * natt, dtype=np.uint8).copy()
    boffs = np.arange(natt + 1, dtype=U64) * 2
    bal = np.full(1024 * 128, 10000, dtype=U64)
    win, vote, total = _lib_process_crosslinks(committee, coffs, np.zeros(natt, np.uint32), np.zeros(natt, np.uint32),
                                               bits, boffs, bal, np.ones(1024, dtype=U64), 5)
    assert win[0] == 0  # record 0 -> {Dynasty 5, Blockhash 'a', Slot 50}


@pytest.mark.parametrize("bitfield,panics", [(b"\x00\x00", False), (b"zz", True)])
def test_process_crosslinks_shard_out_of_range_gpu(bitfield, panics):
    # blockchain/core.go:549: crosslinkRecords[ShardId] is indexed only when the 2/3 test holds,
    # so a shard beyond the records panics (PZ_EINDEX) only for a qualifying attestation
    _, cs = ref.new_genesis_states()
    comm = list(cs.shard_and_committees_for_slots[0].array_shard_and_committee[0].committee)
    committee = np.array(comm, dtype=np.uint32)
    coffs = np.array([0, len(comm)], dtype=U64)
    bits = np.frombuffer(bitfield, dtype=np.uint8).copy()
    boffs = np.array([0, len(bitfield)], dtype=U64)
    bal = np.full(1000, 10000, dtype=U64)
    args = (committee, coffs, np.zeros(1, np.uint32), np.full(1, 1024, np.uint32), bits, boffs, bal,
            np.ones(1024, dtype=U64), 5)
    if panics:
        with pytest.raises(_lib.PzError) as ei:
            _lib_process_crosslinks(*args)
        assert ei.value.code == _lib.PZ_EINDEX
    else:
        win, vote, total = _lib_process_crosslinks(*args)
        assert (win == 0xFFFFFFFF).all() and vote[0] == 0 and total[0] == 10000 * len(comm)


def _lib_process_crosslinks(committee, coffs, att_comm, att_shard, bits, boffs, bal, rec_dyn, dynasty):
    import ctypes
    natt = len(att_comm)
    win = np.empty(len(rec_dyn), dtype=np.uint32)
    vote = np.empty(natt, dtype=U64)
    total = np.empty(natt, dtype=U64)
    p = _lib.ptr
    _lib.lib.call("pz_process_crosslinks", p(committee), p(coffs), len(coffs) - 1, p(att_comm), p(att_shard),
                  p(bits), p(boffs), natt, p(bal), len(bal), p(rec_dyn), len(rec_dyn), dynasty, p(win), p(vote),
                  p(total))
    return win, vote, total


# ---- filters / deposit / rewards vs the oracle ---------------------------------------------
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 2047, 2048, 2049, 100003])
def test_indices_random(n):
    rng = np.random.default_rng(n)
    start = rng.integers(0, 8, size=n, dtype=U64)
    end = rng.integers(0, 12, size=n, dtype=U64)
    for d in (0, 3, 7, 20):
        for kind, f in ((0, casper.active_validator_indices), (1, casper.exited_validator_indices),
                        (2, casper.queued_validator_indices)):
            np.testing.assert_array_equal(f(start, end, d), onp.indices(start, end, d, kind))


@pytest.mark.parametrize("nbytes", [1, 15, 16, 17, 1000, 16384, 16385, 100001])
def test_attesters_total_deposit(nbytes):
    bits = np.random.default_rng(nbytes).integers(0, 256, size=nbytes, dtype=np.uint8)
    assert casper.get_attesters_total_deposit(bits) == onp.attesters_total_deposit(bits)
    # the scalar oracle agrees (casper/validator.go:93-102)
    a = pb.AttestationRecord(attester_bitfield=bits.tobytes())
    assert casper.get_attesters_total_deposit(bits) == ref.get_attesters_total_deposit([a])


def _random_rewards_case(rng, n, frac_active, natt, total_deposit=None):
    start = np.where(rng.random(n) < frac_active, 0, 5).astype(U64)
    end = np.where(rng.random(n) < 0.95, DEFAULT_END_DYNASTY, 1).astype(U64)
    bal = rng.integers(0, 64, size=n, dtype=U64)
    lens = rng.integers(1, 40, size=max(natt - 1, 0)).tolist() + [(n + 7) // 8] if natt else []
    boffs = np.zeros(len(lens) + 1, dtype=U64)
    boffs[1:] = np.cumsum(lens)
    bits = rng.integers(0, 256, size=int(boffs[-1]), dtype=np.uint8)
    td = int(bal.sum()) if total_deposit is None else total_deposit
    return bal, start, end, bits, boffs, td


@pytest.mark.parametrize("n,frac", [(1, 1.0), (40, 1.0), (2048, 0.5), (5000, 0.9), (70001, 1.0), (70001, 0.7)])
def test_calculate_rewards_random(n, frac):
    rng = np.random.default_rng(n + int(frac * 10))
    bal, start, end, bits, boffs, td = _random_rewards_case(rng, n, frac, 6, total_deposit=1)
    want, applied = onp.calculate_rewards(bal, start, end, 1, td, bits, boffs)
    got = bal.copy()
    assert casper.calculate_rewards(got, start, end, 1, td, bits, boffs) == applied
    assert applied
    np.testing.assert_array_equal(got, want)


def test_calculate_rewards_threshold_not_met_and_wrap():
    n = 3000
    rng = np.random.default_rng(9)
    bal, start, end, bits, boffs, _ = _random_rewards_case(rng, n, 1.0, 3)
    got = bal.copy()
    assert not casper.calculate_rewards(got, start, end, 1, (1 << 63) - 1, bits, boffs)
    np.testing.assert_array_equal(got, bal)
    # uint64 wrap: balance 0 penalised -> 2^64-1; 3*dep and 2*total wrap too
    bal0 = np.zeros(n, dtype=U64)
    want, applied = onp.calculate_rewards(bal0, start, end, 1, 1 << 63, bits, boffs)
    got = bal0.copy()
    assert casper.calculate_rewards(got, start, end, 1, 1 << 63, bits, boffs) == applied
    np.testing.assert_array_equal(got, want)


def test_calculate_rewards_panics_map_to_eindex():
    n = 100
    start = np.zeros(n, dtype=U64)
    end = np.full(n, DEFAULT_END_DYNASTY, dtype=U64)
    bal = np.full(n, 32, dtype=U64)
    bits = np.full(5, 0xFF, dtype=np.uint8)  # 40 bits < 100 active validators
    before = bal.copy()
    with pytest.raises(_lib.PzError) as ei:
        casper.calculate_rewards(bal, start, end, 1, 1, bits, np.array([0, 5], dtype=U64))
    assert ei.value.code == _lib.PZ_EINDEX
    np.testing.assert_array_equal(bal, before)
    with pytest.raises(_lib.PzError) as ei:  # no attestations, total 0 -> attestations[-1]
        casper.calculate_rewards(bal, start, end, 1, 0, np.zeros(0, np.uint8), np.zeros(1, dtype=U64))
    assert ei.value.code == _lib.PZ_EINDEX


# ---- shuffle ------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [0, 1, 2, 20, 100, 256, 257, 258, 1000, 1024, 20000, 65536, 1 << 20])
def test_shuffle_bit_exact(n):
    """utils/shuffle.go:14-33 at every size up to configs[3]'s 1,048,576: the scalar oracle
    (n <= 1024) and the C restatement (any n).  Hash{} (the genesis seed) has a zero swap
    number (a self-swap), which the division-free window path must skip."""
    from oracle import cport
    for seed in (ref.bytes_to_hash(b"A"), ref.bytes_to_hash(b""), bytes(range(32))):
        got = casper.shuffle_indices(seed, np.arange(n, dtype=np.uint32))
        if n <= 1024:
            assert got.tolist() == ref.shuffle_indices(seed, list(range(n)))
        np.testing.assert_array_equal(got, cport.shuffle_indices(seed, np.arange(n, dtype=np.uint32)))


def test_shuffle_max_validators():
    with pytest.raises(_lib.PzError) as ei:
        casper.shuffle_indices(bytes(32), np.zeros(ref.MAX_VALIDATORS + 1, dtype=np.uint32))
    assert ei.value.code == _lib.PZ_ETOOMANY


def test_committees_match_oracle():
    for n in (20, 1000, 1024, 9000):
        s = np.zeros(n, dtype=U64)
        e = np.full(n, DEFAULT_END_DYNASTY, dtype=U64)
        got = casper.shuffle_validators_to_committees(ref.bytes_to_hash(b"A"), s, e, 1, 0)
        vals = [pb.ValidatorRecord(start_dynasty=0, end_dynasty=DEFAULT_END_DYNASTY) for _ in range(n)]
        want = ref.shuffle_validators_to_committees(ref.bytes_to_hash(b"A"), vals, 1, 0)
        assert len(got) == len(want) == 64
        for g, w in zip(got, want):
            assert [(sh, c.tolist()) for sh, c in g] == [(sc.shard_id, list(sc.committee))
                                                         for sc in w.array_shard_and_committee]


# ---- crosslinks ----------------------------------------------------------------------------
def test_crosslinks_vs_oracle_synthetic():
    n = 65536
    shuffled = casper.shuffle_indices(ref.bytes_to_hash(b"A"), np.arange(n, dtype=np.uint32))
    inst = synth.epoch_batch(n, 1, seed=4, shuffled=shuffled)
    bal = inst["balance"][0]
    rec = np.zeros(1024, dtype=U64)
    rec[::3] = 1  # some shards already at the current dynasty: they must not be replaced
    win, vote, total = _lib_process_crosslinks(inst["committee"], inst["coffs"], inst["att_comm"], inst["att_shard"],
                                               inst["bits"], inst["boffs"], bal, rec, 1)
    v2, t2 = onp.crosslink_tallies(inst["committee"], inst["coffs"], inst["att_comm"], inst["bits"], inst["boffs"], bal)
    np.testing.assert_array_equal(vote, v2)
    np.testing.assert_array_equal(total, t2)
    np.testing.assert_array_equal(win, onp.crosslink_winners(v2, t2, inst["att_shard"], rec, 1))


def test_crosslink_short_bitfield_panics():
    committee = np.arange(20, dtype=np.uint32)
    coffs = np.array([0, 20], dtype=U64)
    bits = np.full(2, 0xFF, dtype=np.uint8)  # 16 bits for a 20-member committee
    with pytest.raises(_lib.PzError) as ei:
        _lib_process_crosslinks(committee, coffs, np.zeros(1, np.uint32), np.zeros(1, np.uint32), bits,
                                np.array([0, 2], dtype=U64), np.full(20, 5, dtype=U64), np.zeros(1024, dtype=U64), 1)
    assert ei.value.code == _lib.PZ_EINDEX


# ---- device-resident batched epoch ---------------------------------------------------------
_oracle_epoch = oracle_epoch


@pytest.mark.parametrize("n,B,inactive", [(65536, 3, False), (5000, 2, True), (20000, 1, True), (4096, 9, False),
                                          (3000, 17, True)])
def test_device_epoch_vs_oracle(n, B, inactive):
    import torch

    from torch_epoch import DeviceEpoch
    shuffled = casper.shuffle_indices(ref.bytes_to_hash(b"A"), np.arange(n, dtype=np.uint32))
    inst = synth.epoch_batch(n, B, seed=5, shuffled=shuffled)
    if inactive:  # general rank path: some validators exited/queued, rank != index
        rng = np.random.default_rng(1)
        inst["start"][:, rng.random(n) < 0.1] = 7
        inst["end"][:, rng.random(n) < 0.1] = 1
    dev = torch.device("cuda", 0)
    de = DeviceEpoch(inst, dev)
    de.step()
    torch.cuda.synchronize()
    bal, scal, vote, total, win = de.results()
    for b in range(B):
        nb, applied, nxt, v, t, w = _oracle_epoch(inst, b)
        assert bool(scal[b, _lib.SCAL_APPLIED]) == applied
        assert scal[b, _lib.SCAL_ERR_XL] == 0 and (not applied or scal[b, _lib.SCAL_ERR_RWD] == 0)
        np.testing.assert_array_equal(bal[b], nb)
        assert int(scal[b, _lib.SCAL_NEXT_BAL]) == nxt
        np.testing.assert_array_equal(vote[b], v)
        np.testing.assert_array_equal(total[b], t)
        np.testing.assert_array_equal(win[b], w)


def test_device_epoch_configs3_size_vs_oracle():
    """BASELINE configs[3]'s instance size on one GPU: 1,048,576 validators, the real 1M shuffle
    (Hash{'A'}), 65 committees per slot (4,160 of 252-253 members) + the final N-bit
    attestation.  Instance 0 is all active (rank == index, the bench's fast path); instance 1
    has queued and exited validators (rank != index: the compaction path).  Bit-exact against
    the numpy oracle on every balance, tally, winner and the next-cycle total."""
    import torch

    from torch_epoch import DeviceEpoch
    n, B = 1 << 20, 2
    shuffled = casper.shuffle_indices(ref.bytes_to_hash(b"A"), np.arange(n, dtype=np.uint32))
    inst = synth.epoch_batch(n, B, seed=5, shuffled=shuffled)
    sizes = np.diff(inst["coffs"]).astype(np.int64)
    assert inst["natt"] == 4161 and sizes.size == 64 * 65 and set(sizes.tolist()) == {252, 253}
    rng = np.random.default_rng(2)
    inst["start"][1, rng.random(n) < 0.1] = 7   # queued at dynasty 1
    inst["end"][1, rng.random(n) < 0.05] = 1    # exited at dynasty 1
    de = DeviceEpoch(inst, torch.device("cuda", 0))
    de.step()
    torch.cuda.synchronize()
    bal, scal, vote, total, win = de.results()
    for b in range(B):
        nb, applied, nxt, v, t, w = _oracle_epoch(inst, b)
        assert applied and bool(scal[b, _lib.SCAL_APPLIED])
        assert int(scal[b, _lib.SCAL_NACT]) == int(onp.indices(inst["start"][b], inst["end"][b], 1, 0).size)
        np.testing.assert_array_equal(bal[b], nb)
        assert int(scal[b, _lib.SCAL_NEXT_BAL]) == nxt
        np.testing.assert_array_equal(vote[b], v)
        np.testing.assert_array_equal(total[b], t)
        np.testing.assert_array_equal(win[b], w)
    assert int(scal[1, _lib.SCAL_NACT]) < n


def test_device_epoch_repeated_steps_ping_pong():
    """Consecutive steps (ping-pong scal buffers, in-kernel winner reset) equal the oracle
    applied step after step."""
    import torch

    from torch_epoch import DeviceEpoch
    n, B = 8192, 8
    shuffled = casper.shuffle_indices(ref.bytes_to_hash(b"A"), np.arange(n, dtype=np.uint32))
    inst = synth.epoch_batch(n, B, seed=21, shuffled=shuffled)
    de = DeviceEpoch(inst, torch.device("cuda", 0))
    for step in range(3):
        de.step()
        torch.cuda.synchronize()
        bal, scal, vote, total, win = de.results()
        for b in range(B):
            nb, applied, nxt, v, t, w = _oracle_epoch(inst, b)
            np.testing.assert_array_equal(bal[b], nb)
            assert int(scal[b, _lib.SCAL_NEXT_BAL]) == nxt and bool(scal[b, _lib.SCAL_APPLIED]) == applied
            np.testing.assert_array_equal(win[b], w)
            inst["balance"][b] = nb  # the oracle's next step starts from the new balances


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed", [(1, 1), (100, 2), (5000, 3), (70000, 4)])
def test_rotate_validator_set_vs_oracle(n, seed):
    """pz_rotate_validator_set against the oracle on mixed sets: active / queued / exited,
    balances around the 16 cut, and more queued validators than len(active)/30 + 1."""
    rng = np.random.default_rng(seed)
    dyn = 50
    start = rng.choice([0, 10, 49, 50, 51, 80], size=n).astype(U64)
    end = rng.choice([20, 50, 51, 200, DEFAULT_END_DYNASTY], size=n).astype(U64)
    bal = rng.integers(10, 40, size=n).astype(U64)
    vals = [pb.ValidatorRecord(balance=int(b), start_dynasty=int(s), end_dynasty=int(e))
            for b, s, e in zip(bal, start, end)]
    ref.rotate_validator_set(vals, dyn)
    s2, e2 = start.copy(), end.copy()
    casper.rotate_validator_set(bal, s2, e2, dyn)
    assert s2.tolist() == [v.start_dynasty for v in vals]
    assert e2.tolist() == [v.end_dynasty for v in vals]


@pytest.mark.gpu
def test_committees_partial_active_and_start_shard():
    n = 20000
    rng = np.random.default_rng(8)
    s = rng.choice([0, 0, 0, 7], size=n).astype(U64)
    e = rng.choice([DEFAULT_END_DYNASTY, DEFAULT_END_DYNASTY, 2], size=n).astype(U64)
    got = casper.shuffle_validators_to_committees(ref.bytes_to_hash(b"B"), s, e, 3, 1000)
    vals = [pb.ValidatorRecord(start_dynasty=int(a), end_dynasty=int(b)) for a, b in zip(s, e)]
    want = ref.shuffle_validators_to_committees(ref.bytes_to_hash(b"B"), vals, 3, 1000)
    for g, w in zip(got, want):
        assert [(sh, c.tolist()) for sh, c in g] == [(sc.shard_id, list(sc.committee))
                                                     for sc in w.array_shard_and_committee]
