"""Host-side mirror of the reference's ``beacon-chain/casper`` package over the HIP C ABI.

Validators are SoA numpy arrays (``start``, ``end``, ``balance``: uint64) — the packing a
cgo shim does from ``[]*pb.ValidatorRecord``.  Pending attestations are CSR bitfields
(``bits``: uint8 bytes, ``boffs``: uint64 offsets[natt+1]).  Errors mirror Go: a panic in
the reference raises ``PzError`` with code ``PZ_EINDEX``.

Functions that are sequential by nature (``ShuffleIndices``, committee splitting) run on the
host by design (BASELINE.json north_star); everything data-parallel runs on the GPU.
"""
import ctypes

import numpy as np

from prysm_amd import _lib
from prysm_amd._lib import KIND_ACTIVE, KIND_EXITED, KIND_QUEUED, lib, ptr
from prysm_amd.params import CYCLE_LENGTH, MIN_COMMITTEE_SIZE, SHARD_COUNT

_u64 = np.uint64


def _arr(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _indices(start, end, dynasty, kind):
    start, end = _arr(start, _u64), _arr(end, _u64)
    n = start.shape[0]
    out = np.empty(max(n, 1), dtype=np.uint32)
    cnt = ctypes.c_uint64(0)
    lib.call("pz_validator_indices", ptr(start), ptr(end), n, int(dynasty), kind, ptr(out), ctypes.byref(cnt))
    return out[:cnt.value].copy()


def active_validator_indices(start, end, dynasty):
    """casper/validator.go:45-53 (empty array where Go returns nil)."""
    return _indices(start, end, dynasty, KIND_ACTIVE)


def exited_validator_indices(start, end, dynasty):
    """casper/validator.go:57-65."""
    return _indices(start, end, dynasty, KIND_EXITED)


def queued_validator_indices(start, end, dynasty):
    """casper/validator.go:69-77."""
    return _indices(start, end, dynasty, KIND_QUEUED)


def get_attesters_total_deposit(bits):
    """casper/validator.go:93-102 over the concatenated bitfield bytes of all attestations."""
    bits = _arr(bits, np.uint8)
    out = ctypes.c_uint64(0)
    lib.call("pz_attesters_total_deposit", ptr(bits), bits.size, ctypes.byref(out))
    return out.value


def calculate_rewards(balance, start, end, dynasty, total_deposit, bits, boffs):
    """casper/incentives.go:14-32.  ``balance`` (uint64, C-contiguous) is updated in place,
    like the reference mutating ``validators[i].Balance``.  Returns True when the 2/3
    threshold held (rewards applied)."""
    assert isinstance(balance, np.ndarray) and balance.dtype == _u64 and balance.flags["C_CONTIGUOUS"]
    start, end = _arr(start, _u64), _arr(end, _u64)
    bits, boffs = _arr(bits, np.uint8), _arr(boffs, _u64)
    natt = max(boffs.shape[0] - 1, 0)
    applied = ctypes.c_int(0)
    lib.call("pz_calculate_rewards", ptr(balance), ptr(start), ptr(end), balance.shape[0], int(dynasty),
             int(total_deposit), ptr(bits), ptr(boffs) if natt else None, natt, ctypes.byref(applied))
    return bool(applied.value)


def shuffle_indices(seed32, validator_list):
    """utils/shuffle.go:14-33 through pz_shuffle_indices (host swap chain; the 32-byte seed's
    BLAKE2b is a small batch, hashed on the calling thread).  In place on a uint32 array;
    returns it."""
    lst = validator_list if isinstance(validator_list, np.ndarray) else np.array(validator_list, dtype=np.uint32)
    assert lst.dtype == np.uint32 and lst.flags["C_CONTIGUOUS"]
    seed = np.frombuffer(bytes(seed32).ljust(32, b"\0")[:32], dtype=np.uint8).copy()
    lib.call("pz_shuffle_indices", ptr(seed), ptr(lst), lst.shape[0])
    return lst


def split_indices(l, n):
    """utils/shuffle.go:36-44."""
    return [l[len(l) * i // n: len(l) * (i + 1) // n] for i in range(n)]


def get_committee_params(num_validators):
    """casper/sharding.go:60-73."""
    if num_validators >= CYCLE_LENGTH * MIN_COMMITTEE_SIZE:
        return num_validators // (CYCLE_LENGTH * MIN_COMMITTEE_SIZE * 2) + 1, 1
    spc = 1
    while num_validators * spc < MIN_COMMITTEE_SIZE * CYCLE_LENGTH and spc < CYCLE_LENGTH:
        spc *= 2
    return 1, spc


def split_by_slot_shard(shuffled, crosslink_start_shard):
    """casper/sharding.go:27-53 -> [slot][(shard_id, committee uint32 array)]."""
    cps, spc = get_committee_params(len(shuffled))
    out = []
    for i, vs in enumerate(split_indices(shuffled, CYCLE_LENGTH)):
        shard_start = crosslink_start_shard + i * cps // spc
        out.append([((shard_start + j) % SHARD_COUNT, np.asarray(c, dtype=np.uint32))
                    for j, c in enumerate(split_indices(vs, cps))])
    return out


def shuffle_validators_to_committees(seed32, start, end, dynasty, crosslink_start_shard):
    """casper/sharding.go:11-21 through pz_shuffle_validators_to_committees (device filter,
    host swap chain and split) -> [slot][(shard_id, committee uint32 array)]."""
    start, end = _arr(start, _u64), _arr(end, _u64)
    n = start.shape[0]
    seed = np.frombuffer(bytes(seed32).ljust(32, b"\0")[:32], dtype=np.uint8).copy()
    cap = CYCLE_LENGTH * (n // (CYCLE_LENGTH * MIN_COMMITTEE_SIZE * 2) + 1)
    members = np.empty(max(n, 1), dtype=np.uint32)
    coffs = np.empty(cap + 1, dtype=_u64)
    shard = np.empty(cap, dtype=_u64)
    slot_offs = np.empty(CYCLE_LENGTH + 1, dtype=_u64)
    ncomm = ctypes.c_uint64(0)
    lib.call("pz_shuffle_validators_to_committees", ptr(seed), ptr(start), ptr(end), n, int(dynasty),
             int(crosslink_start_shard), ptr(members), ptr(coffs), ptr(shard), ptr(slot_offs), cap,
             ctypes.byref(ncomm))
    return [[(int(shard[c]), members[int(coffs[c]):int(coffs[c + 1])].copy())
             for c in range(int(slot_offs[s]), int(slot_offs[s + 1]))] for s in range(CYCLE_LENGTH)]


def rotate_validator_set(balance, start, end, dynasty):
    """casper/validator.go:17-41 through pz_rotate_validator_set (device filters), in place on
    ``start`` / ``end`` (uint64 arrays); returns them."""
    balance = _arr(balance, _u64)
    for a in (start, end):
        assert isinstance(a, np.ndarray) and a.dtype == _u64 and a.flags["C_CONTIGUOUS"]
    lib.call("pz_rotate_validator_set", ptr(balance), ptr(start), ptr(end), start.shape[0], int(dynasty))
    return start, end


class ValidatorMirror:
    """pz_state: one CrystallizedState's validator set resident in HBM (SURVEY.md §8b
    "Ownership"); the casper functions on it copy only the attestation bitfields per call.
    ``upload`` / ``download`` are the explicit sync points with the host records."""

    def __init__(self, n, device=0):
        self.n = int(n)
        self.h = ctypes.c_void_p()
        lib.call("pz_state_new", self.n, device, ctypes.byref(self.h))

    def upload(self, balance=None, start=None, end=None):
        cols = [None if c is None else _arr(c, _u64) for c in (balance, start, end)]
        for c in cols:
            assert c is None or c.shape == (self.n,)
        lib.call("pz_state_upload", self.h, *[ptr(c) if c is not None else None for c in cols])

    def download(self):
        """-> (balance, start, end) uint64 arrays."""
        out = [np.empty(self.n, dtype=_u64) for _ in range(3)]
        lib.call("pz_state_download", self.h, *[ptr(c) for c in out])
        return tuple(out)

    def indices(self, dynasty, kind=_lib.KIND_ACTIVE):
        out = np.empty(max(self.n, 1), dtype=np.uint32)
        cnt = ctypes.c_uint64(0)
        lib.call("pz_state_validator_indices", self.h, int(dynasty), kind, ptr(out), ctypes.byref(cnt))
        return out[:cnt.value].copy()

    def calculate_rewards(self, dynasty, total_deposit, bits, boffs):
        """casper/incentives.go:14-32 on the resident balances -> applied."""
        bits = _arr(bits, np.uint8)
        boffs = _arr(boffs, _u64)
        applied = ctypes.c_int(0)
        lib.call("pz_state_calculate_rewards", self.h, int(dynasty), int(total_deposit), ptr(bits), ptr(boffs),
                 max(len(boffs) - 1, 0), ctypes.byref(applied))
        return bool(applied.value)

    def active_balance(self, dynasty):
        tot = ctypes.c_uint64(0)
        lib.call("pz_state_active_balance", self.h, int(dynasty), ctypes.byref(tot))
        return tot.value

    def free(self):
        if self.h:
            lib.dll.pz_state_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # pragma: no cover
            pass
