"""Device proto3 encoder of ValidatorRecord columns (prysm_amd/csrc/wire.hip) against Google's
protobuf runtime over the oracle schema (oracle/schema.py, pinned to messages.pb.go:803-809)
and, at full size, against the host encoder (prysm_amd/wire.py, itself pinned to the runtime
by tests/test_wire.py).  Byte-exact."""
import ctypes

import numpy as np
import pytest

from oracle import schema as opb
from prysm_amd import _lib, pb, wire

pytestmark = pytest.mark.gpu


def varint(x):
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def rand_cols(rng, n, with_bytes):
    mags = np.array([0, 1, 127, 128, 16383, 16384, (1 << 32) - 1, (1 << 63), (1 << 64) - 1], dtype=np.uint64)

    def col():
        pick = rng.integers(0, len(mags) + 1, size=n)
        x = rng.integers(0, 1 << 62, size=n, dtype=np.uint64) * np.uint64(4) + np.uint64(3)
        return np.where(pick < len(mags), mags[np.minimum(pick, len(mags) - 1)], x).astype(np.uint64)

    def blobs():
        if not with_bytes:
            return None
        lens = rng.choice([0, 0, 1, 20, 32, 127, 128, 300], size=n)
        return [rng.integers(0, 256, size=int(k), dtype=np.uint8).tobytes() for k in lens]

    return pb.Validators(n, public_key=col(), withdrawal_shard=col(), withdrawal_address=blobs(),
                         randao_commitment=blobs(), balance=col(), start_dynasty=col(), end_dynasty=col())


def oracle_record(v, i):
    return opb.ValidatorRecord(
        public_key=int(v.public_key[i]), withdrawal_shard=int(v.withdrawal_shard[i]),
        withdrawal_address=v.withdrawal_address[i] if v.withdrawal_address is not None else b"",
        randao_commitment=v.randao_commitment[i] if v.randao_commitment is not None else b"",
        balance=int(v.balance[i]), start_dynasty=int(v.start_dynasty[i]),
        end_dynasty=int(v.end_dynasty[i])).SerializeToString()


def oracle_framed(v, field_num):
    tag = varint((field_num << 3) | 2)
    return b"".join(tag + varint(len(r)) + r for r in (oracle_record(v, i) for i in range(len(v))))


@pytest.mark.parametrize("n", [1, 63, 255, 256, 257, 1000, 3000])
@pytest.mark.parametrize("with_bytes", [False, True])
def test_validators_match_protobuf_runtime(n, with_bytes):
    v = rand_cols(np.random.default_rng(n * 2 + with_bytes), n, with_bytes)
    got = wire.validators_device(v, 11)
    assert got == oracle_framed(v, 11)
    # the CrystallizedState framing is exactly the runtime's repeated field 11
    o = opb.CrystallizedState()
    for i in range(n):
        o.validators.add().ParseFromString(oracle_record(v, i))
    assert got == o.SerializeToString()


@pytest.mark.parametrize("field_num", [1, 15, 16, 2047, 2048, (1 << 29) - 1])
def test_framing_field_numbers(field_num):
    v = rand_cols(np.random.default_rng(field_num % 1000), 600, False)
    assert wire.validators_device(v, field_num) == oracle_framed(v, field_num)


@pytest.mark.parametrize("with_bytes", [False, True])
def test_bare_records_with_offsets(with_bytes):
    n = 777
    v = rand_cols(np.random.default_rng(5), n, with_bytes)
    raw, offs = wire.validators_device(v, 0, with_offsets=True)
    assert offs[0] == 0 and offs[-1] == len(raw)
    for i in range(n):
        assert raw[int(offs[i]):int(offs[i + 1])] == oracle_record(v, i), i


def test_all_zero_records_and_empty():
    v = pb.Validators(300)
    assert wire.validators_device(v, 11) == b"\x5a\x00" * 300
    raw, offs = wire.validators_device(v, 0, with_offsets=True)  # bare empty records: all offsets 0
    assert raw == b"" and not offs.any()
    assert wire.validators_device(pb.Validators(0), 11) == b""


def test_genesis_validators_full_size():
    """MaxValidators (4,194,304) genesis-style records vs the host encoder, plus 1M random."""
    n = 1 << 22
    v = pb.Validators(n, balance=np.full(n, 32, np.uint64),
                      end_dynasty=np.full(n, 9999999999999999999, np.uint64))
    got = wire.validators_device(v, 11)
    assert got == wire.validators(v)
    assert len(got) == n * 15
    v = rand_cols(np.random.default_rng(9), 1 << 20, False)
    assert wire.validators_device(v, 11) == wire.validators(v)


def test_capacity_error():
    v = rand_cols(np.random.default_rng(3), 100, False)
    cols = _lib.ValidatorCols(None, None, None, None, None, None, _lib.ptr(v.balance), None, None)
    out = np.empty(10, dtype=np.uint8)
    length = ctypes.c_uint64(0)
    with pytest.raises(_lib.PzError) as e:
        _lib.lib.call("pz_wire_validators", ctypes.byref(cols), 100, 11, _lib.ptr(out), 10, None,
                      ctypes.byref(length))
    assert e.value.code == _lib.PZ_ERANGE
    assert length.value == len(wire.validators(pb.Validators(100, balance=v.balance)))


def test_device_entry_point_null_columns():
    """pz_dev_wire_validators on device-resident columns (torch tensors, torch's stream), with
    NULL columns for the fields that are zero, as the chain engine calls it."""
    import torch

    n = 100_003
    rng = np.random.default_rng(11)
    bal = rng.integers(16, 48, size=n, dtype=np.uint64)
    end = np.full(n, 9999999999999999999, np.uint64)
    d_bal = torch.from_numpy(bal.view(np.int64)).cuda()
    d_end = torch.from_numpy(end.view(np.int64)).cuda()
    bound = _lib.lib.dll.pz_wire_validators_bound(n, 0)
    d_out = torch.zeros(bound, dtype=torch.uint8, device="cuda")
    d_offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    d_scr = torch.zeros(_lib.lib.dll.pz_wire_scratch_bytes(n) // 8, dtype=torch.int64, device="cuda")
    d_tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    cols = _lib.ValidatorCols(None, None, None, None, None, None, d_bal.data_ptr(), None, d_end.data_ptr())
    _lib.lib.call("pz_dev_wire_validators", ctypes.byref(cols), n, 11, d_out.data_ptr(), d_offs.data_ptr(),
                  d_scr.data_ptr(), d_tot.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    total = int(d_tot.item())
    want = wire.validators(pb.Validators(n, balance=bal, end_dynasty=end))
    assert total == len(want) == int(d_offs[-1].item())
    assert d_out[:total].cpu().numpy().tobytes() == want


def _scalar_cols(rng, n, which):
    """Random scalar columns for the fields in `which`, the rest NULL; magnitudes mixed so
    varints take 1-10 bytes and some 4,096-record tiles outgrow the 64 KiB LDS stage."""
    out = {}
    for k in which:
        mags = rng.integers(0, 64, size=n)
        out[k] = (rng.integers(0, 1 << 63, size=n, dtype=np.uint64) >> mags.astype(np.uint64)).astype(np.uint64)
        out[k][rng.random(n) < 0.1] = 0
    return pb.Validators(n, **out)


@pytest.mark.parametrize("which", [("balance",), ("balance", "end_dynasty"), ("balance", "start_dynasty", "end_dynasty"),
                                   ("public_key", "balance", "end_dynasty")])
@pytest.mark.parametrize("offsets", [False, True])
def test_scalar_columns_many_tiles(which, offsets):
    """The scalar-only kernel with 1-3 non-NULL columns over 12 tiles of 4,096 records (the
    look-back across tiles, a ragged last tile), framed against the host encoder and bare with
    record offsets against the protobuf runtime record by record."""
    n = 4096 * 11 + 1234
    v = _scalar_cols(np.random.default_rng(len(which) * 10 + offsets), n, which)
    if offsets:
        raw, offs = wire.validators_device(v, 0, with_offsets=True)
        assert offs[0] == 0 and offs[-1] == len(raw)
        assert raw == b"".join(oracle_record(v, i) for i in range(n))
    else:
        assert wire.validators_device(v, 11) == wire.validators(v)


@pytest.mark.ab
@pytest.mark.parametrize("variant", [16384])
def test_lookback_multi_window(variant):
    """The wave-reduced look-back over several windows (the A/B library's test path): with no
    inclusive prefix published (wire.hip variant bit 14) every tile sums aggregates window after
    window back to tile 0.  3,000 tiles: up to 2 windows per tile.
    The bytes must equal the product kernel's, which must equal the host encoder's."""
    import torch

    n = 4096 * 3000 - 77
    rng = np.random.default_rng(21)
    bal = rng.integers(16, 49, size=n, dtype=np.uint64)
    end = np.full(n, 9999999999999999999, np.uint64)
    start = (rng.integers(0, 3, size=n).astype(np.uint64) * rng.integers(0, 1 << 40, size=n, dtype=np.uint64))
    cols_t = [torch.from_numpy(a.view(np.int64)).cuda() for a in (bal, start, end)]
    dll = _lib.lib.dll
    bound = int(dll.pz_wire_validators_bound(n, 0))
    d_scr = torch.zeros(int(dll.pz_wire_scratch_bytes(n)) // 8, dtype=torch.int64, device="cuda")
    d_tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    cols = _lib.ValidatorCols(None, None, None, None, None, None, *[t.data_ptr() for t in cols_t])
    sh = torch.cuda.current_stream().cuda_stream

    def encode(v):
        out = torch.zeros(bound, dtype=torch.uint8, device="cuda")
        old = dll.pz_debug_set_wire_variant(v)
        try:
            _lib.lib.call("pz_dev_wire_validators", ctypes.byref(cols), n, 11, out.data_ptr(), None, d_scr.data_ptr(),
                          d_tot.data_ptr(), sh)
            torch.cuda.synchronize()
        finally:
            dll.pz_debug_set_wire_variant(old)
        return out[:int(d_tot.item())]

    ref = encode(0)
    assert torch.equal(encode(variant), ref)
    k = 50_000  # the host encoder on a prefix (the framing is per record, so prefixes agree)
    want = wire.validators(pb.Validators(k, balance=bal[:k], start_dynasty=start[:k], end_dynasty=end[:k]))
    assert ref[:len(want)].cpu().numpy().tobytes() == want


