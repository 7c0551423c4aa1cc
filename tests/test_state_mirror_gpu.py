"""pz_state (the device-resident validator mirror, SURVEY.md §8b "Ownership"): the casper
drop-ins on HBM-resident balances give the reference's results, bit-exact against the oracle,
across repeated calls with no re-upload in between."""
import numpy as np
import pytest

from oracle import epoch_np as onp
from prysm_amd import _lib, casper
from prysm_amd.params import DEFAULT_END_DYNASTY

pytestmark = pytest.mark.gpu
U64 = np.uint64


def test_mirror_rewards_kat():
    # casper/incentives_test.go:9-43
    m = casper.ValidatorMirror(40)
    m.upload(np.full(40, 32, U64), np.ones(40, U64), np.full(40, 10, U64))
    assert m.calculate_rewards(1, 100, np.array([200, 148, 146, 179, 49], np.uint8), np.array([0, 5], U64))
    bal, start, end = m.download()
    assert bal[0] == 33 and bal[7] == 31 and bal[29] == 31
    assert (start == 1).all() and (end == 10).all()


@pytest.mark.parametrize("n", [1, 63, 2048, 2049, 70001])
def test_mirror_repeated_calls_vs_oracle(n):
    """Three epochs of rewards on the resident balances (uploaded once), with the filters and
    the next-cycle total after each, against the numpy oracle."""
    rng = np.random.default_rng(n)
    start = np.where(rng.random(n) < 0.85, 0, 5).astype(U64)
    end = np.where(rng.random(n) < 0.95, DEFAULT_END_DYNASTY, 1).astype(U64)
    bal = rng.integers(0, 64, size=n, dtype=U64)
    m = casper.ValidatorMirror(n)
    m.upload(bal, start, end)
    for step in range(3):
        lens = rng.integers(1, 40, size=3).tolist() + [(n + 7) // 8]
        boffs = np.zeros(len(lens) + 1, dtype=U64)
        boffs[1:] = np.cumsum(lens)
        bits = rng.integers(0, 256, size=int(boffs[-1]), dtype=np.uint8)
        tdep = int(rng.integers(0, 200)) * n // 8
        want, applied = onp.calculate_rewards(bal, start, end, 1, tdep, bits, boffs)
        assert m.calculate_rewards(1, tdep, bits, boffs) == applied
        bal = want
        for kind in (0, 1, 2):
            np.testing.assert_array_equal(m.indices(1, kind), onp.indices(start, end, 1, kind))
        assert m.active_balance(1) == onp.active_balance_sum(bal, start, end, 1)
    np.testing.assert_array_equal(m.download()[0], bal)


def test_mirror_panic_leaves_balances():
    """The last bitfield too short for the largest active index: CalculateRewards panics
    (incentives.go:23) -> PZ_EINDEX, balances untouched."""
    n = 100
    m = casper.ValidatorMirror(n)
    bal = np.full(n, 32, U64)
    m.upload(bal, np.zeros(n, U64), np.full(n, DEFAULT_END_DYNASTY, U64))
    with pytest.raises(_lib.PzError) as ei:
        m.calculate_rewards(1, 1, np.full(4, 0xFF, np.uint8), np.array([0, 4], U64))
    assert ei.value.code == _lib.PZ_EINDEX
    np.testing.assert_array_equal(m.download()[0], bal)
