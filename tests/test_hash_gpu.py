"""BLAKE2b-512 batch kernels vs the oracle (hashlib, RFC 7693).  Bit-exact."""
import numpy as np
import pytest

from oracle import ref
from prysm_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu_route():
    """These tests pin the GPU kernels: every batch, however small, goes to the device."""
    with _lib.small_batch_threshold(0):
        yield


def test_small_batch_host_route_matches_oracle():
    """Drop-in Hash() calls (one message, types/block.go:67-77) below the small-batch
    threshold are hashed on the calling thread; same digests as the oracle, at every block
    boundary, and a batch just above the threshold takes the GPU route with the same result."""
    with _lib.small_batch_threshold(_lib.SMALL_BATCH_DEFAULT):
        for n in list(range(0, 600)) + [8191, 8192]:
            m = bytes((i * 31 + n) & 0xFF for i in range(n))
            assert _lib.blake2b512_batch([m], 64)[0] == ref.sum512(m), n
        msgs = [bytes([k]) * 512 for k in range(65)]  # 65 x 4 compressions > 256: the GPU route
        assert _lib.blake2b512_batch(msgs, 32) == [ref.sum512(m)[:32] for m in msgs]


def test_rfc7693_abc_gpu():
    d = _lib.blake2b512_batch([b"abc"], out_bytes=64)[0]
    assert d == ref.sum512(b"abc")


def test_lengths_0_to_600():
    # every block boundary, empty message, partial dwords
    msgs = [bytes((i * 7 + j) & 0xFF for j in range(i)) for i in range(0, 601)]
    for ob in (32, 64):
        got = _lib.blake2b512_batch(msgs, out_bytes=ob)
        for m, g in zip(msgs, got):
            assert g == ref.sum512(m)[:ob], len(m)


def test_fixed_512_records_uniform_path():
    rng = np.random.default_rng(2)
    n = 5000  # not a multiple of 64 or 256: exercises the tail wave
    data = rng.integers(0, 256, size=n * 512, dtype=np.uint8)
    offs = np.arange(n + 1, dtype=np.uint64) * 512
    got = _lib.blake2b512_csr(data, offs)
    raw = data.tobytes()
    for i in range(0, n, 37):
        assert got[i].tobytes() == ref.hash32(raw[i * 512:(i + 1) * 512])
    assert got[n - 1].tobytes() == ref.hash32(raw[(n - 1) * 512:])


@pytest.mark.parametrize("rec", [16, 112, 128, 144, 256, 400])
def test_fixed_other_lengths(rec):
    rng = np.random.default_rng(rec)
    n = 300
    data = rng.integers(0, 256, size=n * rec, dtype=np.uint8)
    offs = np.arange(n + 1, dtype=np.uint64) * rec
    got = _lib.blake2b512_csr(data, offs, out_bytes=64)
    raw = data.tobytes()
    for i in range(n):
        assert got[i].tobytes() == ref.sum512(raw[i * rec:(i + 1) * rec])


def test_ragged_unaligned_csr():
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 700, size=777)
    msgs = [rng.integers(0, 256, size=int(l), dtype=np.uint8).tobytes() for l in lens]
    got = _lib.blake2b512_batch(msgs)
    for m, g in zip(msgs, got):
        assert g == ref.hash32(m)


def test_fixed_kernel_paths_match_oracle():
    """Both fixed-length kernels, each reached by the shape that selects it: the persistent
    LDS-DMA kernel takes the 64-aligned bulk when the stride holds whole 128-B blocks (512, 384 B
    records) and the plain grid takes the tail (n not a multiple of 64) and tight strides (500 B
    records: 4 blocks in a 500 B stride).  Every digest is checked against hashlib."""
    import hashlib
    rng = np.random.default_rng(77)
    for rec, n in ((512, 70001), (384, 6400), (500, 3000)):
        data = rng.integers(0, 256, size=n * rec, dtype=np.uint8)
        offs = np.arange(n + 1, dtype=np.uint64) * rec
        got = _lib.blake2b512_csr(data, offs)
        raw = data.tobytes()
        want = np.frombuffer(b"".join(hashlib.blake2b(raw[i * rec:(i + 1) * rec], digest_size=64).digest()[:32]
                                      for i in range(n)), dtype=np.uint8).reshape(n, 32)
        np.testing.assert_array_equal(got[:, :32], want)


@pytest.mark.parametrize("thr", [1000, _lib.SERIAL_ON_GPU])
def test_long_messages_host_route_and_gpu_route_agree(thr):
    """Messages at or above the serial threshold are hashed on host threads while the GPU
    hashes the rest of the batch; both routes are bit-exact with hashlib, and
    the digest order is kept when long and short messages interleave."""
    rng = np.random.default_rng(5)
    lens = [0, 999, 1000, 1001, 5, 70000, 128, 1000, 3, 131072, 0]
    msgs = [rng.integers(0, 256, size=l, dtype=np.uint8).tobytes() for l in lens]
    with _lib.serial_threshold(thr):
        for ob in (32, 64):
            got = _lib.blake2b512_batch(msgs, out_bytes=ob)
            assert got == [ref.sum512(m)[:ob] for m in msgs]
        only_long = [m for m in msgs if len(m) >= 1000]
        assert _lib.blake2b512_batch(only_long, 64) == [ref.sum512(m) for m in only_long]


def test_batch_api_thread_safe():
    """The host-pointer C ABI is thread-safe (per-device mutex, library stream): eight Python
    threads (ctypes releases the GIL) hash different batches concurrently, mixing the GPU
    route and the host serial route; every digest is still right."""
    import threading

    rng = np.random.default_rng(11)
    batches = []
    for t in range(8):
        lens = rng.integers(0, 3000, size=200).tolist() + ([70000] if t % 2 else [])
        batches.append([rng.integers(0, 256, size=l, dtype=np.uint8).tobytes() for l in lens])
    out = [None] * len(batches)
    errs = []

    def work(i):
        try:
            for _ in range(3):
                out[i] = _lib.blake2b512_batch(batches[i], out_bytes=64)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(batches))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for msgs, got in zip(batches, out):
        assert got == [ref.sum512(m) for m in msgs]
