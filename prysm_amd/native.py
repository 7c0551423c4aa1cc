"""Python face of the library's own multi-GPU layer (include/prysm_hip.h, "multi-GPU").

``Comm`` wraps a ``pz_comm`` (RCCL over xGMI, or the in-process loopback used to run the
sharded path on one GPU); ``NativeEpoch`` wraps a ``pz_epoch_state``: B epoch instances
resident in HBM, sharded by validator range over the communicator's ranks, stepped entirely
inside the C ABI (kernels and RCCL collectives on the library's streams).  This is the path a
cgo caller links; ``prysm_amd.epoch.DeviceEpoch`` (torch.distributed collectives) is kept as
the test double of the same orchestration.
"""
import ctypes

import numpy as np

from prysm_amd import _lib
from prysm_amd._lib import EpochHost, EpochOptions, SCAL_COUNT, lib, ptr

COMM_ID_BYTES = 128


class Comm:
    """A ``pz_comm``.  Use the constructors below; ``free()`` (or garbage collection) releases it."""

    def __init__(self, handle):
        self.h = handle
        w, nl, r0 = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        lib.call("pz_comm_size", self.h, ctypes.byref(w), ctypes.byref(nl), ctypes.byref(r0))
        self.world, self.nlocal, self.first_rank = w.value, nl.value, r0.value

    @staticmethod
    def unique_id():
        buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
        lib.call("pz_comm_unique_id", buf)
        return bytes(buf)

    @classmethod
    def rank(cls, uid, world, rank, device):
        """One process per GPU: RCCL rank ``rank`` of ``world`` (``uid`` from rank 0's
        ``unique_id()``)."""
        h = ctypes.c_void_p()
        lib.call("pz_comm_init_rank", (ctypes.c_uint8 * COMM_ID_BYTES)(*uid), world, rank, device, ctypes.byref(h))
        return cls(h)

    @classmethod
    def devices(cls, ndev, devices=None):
        """One process driving ``ndev`` GPUs (ncclCommInitAll)."""
        h = ctypes.c_void_p()
        arr = (ctypes.c_int * ndev)(*devices) if devices is not None else None
        lib.call("pz_init_devices", ndev, arr, ctypes.byref(h))
        return cls(h)

    @classmethod
    def loopback(cls, world, device=0):
        """``world`` ranks in this process on one device (collectives without RCCL)."""
        h = ctypes.c_void_p()
        lib.call("pz_comm_init_loopback", world, device, ctypes.byref(h))
        return cls(h)

    @classmethod
    def shm(cls, name, world, rank, device=0, timeout_ms=60000):
        """One process per rank, ranks free to share a device: collectives staged through host
        memory and the POSIX shared-memory group ``name`` (every rank passes the same name;
        rank 0 creates it).  Checks that all ranks issue the same collective sequence."""
        h = ctypes.c_void_p()
        lib.call("pz_comm_init_shm", name.encode(), world, rank, device, timeout_ms, ctypes.byref(h))
        return cls(h)

    def set_timing(self, on=True):
        """Bracket every collective with HIP events on the communicator's streams."""
        lib.call("pz_comm_set_timing", self.h, 1 if on else 0)

    def collective_time(self):
        """(ms, count): the summed device time of the collectives since the last call (max over
        this process's local ranks per collective) and how many there were."""
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        lib.call("pz_comm_collective_time", self.h, ctypes.byref(ms), ctypes.byref(n))
        return ms.value, n.value

    def hash_batch(self, data, offsets, out_bytes=32):
        """pz_comm_blake2b512_batch: this process's ranks' slices of the CSR batch; rows of
        other processes' slices are left zero."""
        n = len(offsets) - 1
        out = np.zeros((max(n, 0), out_bytes), dtype=np.uint8)
        if n > 0:
            data = np.ascontiguousarray(data, dtype=np.uint8)
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            lib.call("pz_comm_blake2b512_batch", self.h, ptr(data), ptr(offsets), n, ptr(out), out_bytes)
        return out

    def free(self):
        if self.h:
            lib.dll.pz_comm_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # pragma: no cover - interpreter teardown
            pass


def _epoch_host(inst, layout="auto"):
    """(``pz_epoch_host`` over a ``synth.epoch_batch``-shaped dict, the arrays it points into)."""
    u64 = lambda a: np.ascontiguousarray(a, dtype=np.uint64)  # noqa: E731
    u32 = lambda a: np.ascontiguousarray(a, dtype=np.uint32)  # noqa: E731
    k = dict(balance=u64(inst["balance"]), start=u64(inst["start"]), end=u64(inst["end"]),
             dynasty=u64(inst["dynasty"]), total_deposit=u64(inst["total_deposit"]),
             bits=np.ascontiguousarray(inst["bits"], dtype=np.uint8), boffs=u64(inst["boffs"]),
             committee=u32(inst["committee"]), coffs=u64(inst["coffs"]),
             att_comm=u32(inst["att_comm"]), att_shard=u32(inst["att_shard"]),
             rec_dynasty=u64(inst["rec_dynasty"]))
    h = EpochHost()
    h.ninst, h.nval, h.natt = int(inst["ninst"]), int(inst["nval"]), int(inst["natt"])
    h.balance, h.start, h.end = ptr(k["balance"]), ptr(k["start"]), ptr(k["end"])
    h.dynasty, h.total_deposit = ptr(k["dynasty"]), ptr(k["total_deposit"])
    h.bits, h.boffs = ptr(k["bits"]), ptr(k["boffs"])
    h.committee, h.coffs, h.ncomm = ptr(k["committee"]), ptr(k["coffs"]), len(k["coffs"]) - 1
    h.att_comm, h.att_shard = ptr(k["att_comm"]), ptr(k["att_shard"])
    h.nrec = int(k["rec_dynasty"].shape[1]) if k["rec_dynasty"].ndim == 2 else int(k["rec_dynasty"].size)
    h.rec_dynasty = ptr(k["rec_dynasty"])
    h.layout = {"auto": 0, "index": 1, "twopass": 2}[layout]
    return h, k


def epoch_plan(inst, world, rank, layout="auto"):
    """``pz_epoch_plan`` (host only, no device): (lo, hi, layout code) of global rank ``rank``
    -- the storage positions a ``NativeEpoch`` rank of that world would hold and whether its
    step is index order (0), committee order (1) or the one-pass step (2)."""
    h, keep = _epoch_host(inst, layout)
    lo, hi, co = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    lib.call("pz_epoch_plan", ctypes.byref(h), world, rank, ctypes.byref(lo), ctypes.byref(hi), ctypes.byref(co))
    del keep
    return lo.value, hi.value, co.value


class NativeEpoch:
    """``pz_epoch_state``: the same inputs as ``prysm_amd.epoch.DeviceEpoch`` (a
    ``synth.epoch_batch``-shaped dict over all validators)."""

    def __init__(self, inst, device=0, comm=None, layout="auto", rebase_period=0, window_only=False):
        """``layout``: "auto" (committee order when every validator is active and the
        committees partition the set, with the one-pass step when no attestation names a
        shard >= nrec), "twopass" (the same layout, two-pass step) or "index".
        ``rebase_period`` / ``window_only``: pz_epoch_options (tests: the u32 offsets re-based
        every k steps; one instance through the window pass instead of pz_epoch_one_kernel)."""
        h, self._keep = _epoch_host(inst, layout)
        self.B, self.N, self.natt, self.nrec = int(h.ninst), int(h.nval), int(h.natt), int(h.nrec)
        self.comm = comm
        self.st = ctypes.c_void_p()
        opts = EpochOptions(int(rebase_period), 1 if window_only else 0)
        lib.call("pz_epoch_state_new_opts", comm.h if comm is not None else None, device, ctypes.byref(h),
                 ctypes.byref(opts), ctypes.byref(self.st))
        self._keep = None  # the library copied everything it needs
        self.nlocal = comm.nlocal if comm is not None else 1
        co = ctypes.c_int(0)
        lib.call("pz_epoch_state_layout", self.st, ctypes.byref(co))
        self.committee_order = bool(co.value)
        self.one_pass = co.value == 2
        bb, db = ctypes.c_uint32(), ctypes.c_uint32()
        lib.call("pz_epoch_state_columns", self.st, ctypes.byref(bb), ctypes.byref(db))
        # bytes the one-pass stream reads per validator-epoch: balance (u32 offsets or u64) and
        # the {start, end} column (16-bit, 32-bit saturated or u64)
        self.balance_bytes, self.dynasty_bytes = int(bb.value), int(db.value)

    def step(self):
        lib.call("pz_epoch_state_step", self.st)

    def sync(self):
        lib.call("pz_epoch_state_sync", self.st)

    def bind_stream(self, stream_handle, local=0):
        """Enqueue local rank ``local``'s steps on the caller's stream (a ``hipStream_t``
        handle; None: the state's own stream) -- pz_epoch_state_bind_stream."""
        lib.call("pz_epoch_state_bind_stream", self.st, local,
                 ctypes.c_void_p(stream_handle) if stream_handle else None)

    def shard(self, local=0):
        """(lo, hi, device, stream handle) of local rank ``local``."""
        lo, hi, dev, s = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int(), ctypes.c_void_p()
        lib.call("pz_epoch_state_shard", self.st, local, ctypes.byref(lo), ctypes.byref(hi), ctypes.byref(dev),
                 ctypes.byref(s))
        return lo.value, hi.value, dev.value, s.value

    def tallies(self):
        """Complete every attestation's vote/total on every rank after a sharded one-pass
        step (a collective; a no-op otherwise)."""
        lib.call("pz_epoch_state_tallies", self.st)

    def validators(self, local=0):
        """The validator index of each balance column ``results(local)`` returns."""
        lo, hi, _, _ = self.shard(local)
        idx = np.empty(hi - lo, dtype=np.uint32)
        lib.call("pz_epoch_state_validators", self.st, local, ptr(idx))
        return idx

    def results(self, local=0):
        """Host copies after the last step: (balance [B][hi-lo] of the validators
        ``validators(local)`` names, scal [B][8], vote, total, winner)."""
        lo, hi, _, _ = self.shard(local)
        bal = np.empty((self.B, hi - lo), dtype=np.uint64)
        scal = np.empty((self.B, SCAL_COUNT), dtype=np.uint64)
        vote = np.empty((self.B, self.natt), dtype=np.uint64)
        total = np.empty((self.B, self.natt), dtype=np.uint64)
        win = np.empty((self.B, self.nrec), dtype=np.uint32)
        lib.call("pz_epoch_state_results", self.st, local, ptr(bal), ptr(scal), ptr(vote), ptr(total), ptr(win))
        return bal, scal, vote, total, win

    def free(self):
        if self.st:
            lib.dll.pz_epoch_state_free(self.st)
            self.st = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # pragma: no cover - interpreter teardown
            pass


__all__ = ["Comm", "NativeEpoch", "_lib"]
