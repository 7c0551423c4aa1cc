"""Test double (tests/ only since round 6; the product's epoch driver is pz_epoch_state, which
prysm_amd.native.NativeEpoch wraps): a device-resident mirror of the epoch-transition state (SoA in
HBM) driven from Python over torch.distributed.

``DeviceEpoch`` holds B epoch instances' validator arrays, pending-attestation bitfields and
committees in HBM (torch tensors are used only as device allocations) and runs the
data-parallel part of stateRecalc (blockchain/core.go:433-464) through
``pz_dev_epoch_count`` / ``pz_dev_epoch_finish``.  With ``world > 1`` each rank owns a
contiguous validator range and the partial sums are combined by RCCL all-reduce over xGMI
(``torch.distributed`` with the "nccl" backend is RCCL on ROCm).
"""
import ctypes

import numpy as np

from prysm_amd import _lib
from prysm_amd._lib import EpochBatch, SCAL_COUNT, lib


def shard_words(nval_global, world):
    """64-validator words per shard: every shard but the last holds exactly 64 * this many
    validators, so the shards' active bitmasks concatenate (rank-major) into the global mask."""
    return max(1, -(-nval_global // (64 * world)))


def shard_range(nval_global, rank, world):
    """Contiguous, 64-aligned validator range [lo, hi) of ``rank``."""
    s = 64 * shard_words(nval_global, world)
    return min(nval_global, rank * s), min(nval_global, (rank + 1) * s)


def local_committees(committee, coffs, lo, hi, nval_global, keep_out_of_range):
    """The committee CSR restricted to members in [lo, hi) (plus, when
    ``keep_out_of_range``, members >= nval_global, whose panic that rank raises), with each
    kept member's position in its full committee -> (committee, coffs, cpos)."""
    committee = np.asarray(committee, dtype=np.uint32)
    coffs = np.asarray(coffs, dtype=np.uint64)
    rows = np.repeat(np.arange(len(coffs) - 1), np.diff(coffs).astype(np.int64))
    pos = np.arange(committee.size, dtype=np.int64) - coffs[rows].astype(np.int64)
    keep = (committee >= lo) & (committee < hi)
    if keep_out_of_range:
        keep |= committee >= nval_global
    counts = np.bincount(rows[keep], minlength=len(coffs) - 1)
    out_offs = np.zeros(len(coffs), dtype=np.uint64)
    out_offs[1:] = np.cumsum(counts)
    out = committee[keep]
    return (out if out.size else np.zeros(1, np.uint32)), out_offs, pos[keep].astype(np.uint32)


class HipEpochKernels:
    """The product kernels: the C-ABI entry points of libprysm_hip.so (include/prysm_hip.h)."""

    def count(self, batch, stream):
        lib.call("pz_dev_epoch_count", ctypes.byref(batch), stream)

    def gather_compact(self, batch, gmask_ptr, world, sw, gblk_ptr, stream):
        lib.call("pz_dev_epoch_gather_compact", ctypes.byref(batch), gmask_ptr, world, sw, gblk_ptr, stream)

    def finish(self, batch, stream):
        lib.call("pz_dev_epoch_finish", ctypes.byref(batch), stream)


class _Part:
    """A contiguous slice [i0, i0 + B) of the instances with its own batch struct and its own
    ping-pong reduction buffers {scal, vote, total} (one all-reduce combines a part's partial
    sums).  At N > 1 the batch is split in two parts so that one part's collectives overlap
    the other part's kernels."""

    def __init__(self, de, i0, B):
        torch, dev = de.torch, de.dev
        self.i0, self.B = i0, B
        natt, nrec, n, N, world = de.natt, de.nrec, de.n, de.N, de.world
        # two buffers ping-pong: the finish pass of step k zeroes the scal of step k+1, so no
        # memset launch is needed per step
        self.reds = [torch.zeros(B * SCAL_COUNT + 2 * B * natt, dtype=torch.int64, device=dev) for _ in range(2)]
        self.cur = 0
        if de.general:
            # this rank's mask padded to the common shard width, the gathered stack, and the
            # per-chunk counts of the global compaction
            self.mask_send = torch.zeros(B * de.sw, dtype=torch.int64, device=dev)
            self.gmask = torch.zeros(world * B * de.sw, dtype=torch.int64, device=dev)
            self.gblk = torch.zeros(B * ((N + 2047) // 2048), dtype=torch.int32, device=dev)
        wl, vbpi = (n + 63) // 64, (n + 2047) // 2048
        P = lambda t, off, esz=8: t.data_ptr() + off * esz  # noqa: E731
        b = EpochBatch()
        b.ninst, b.nval, b.val_offset, b.nval_global = B, n, de.lo, N
        b.kind = _lib.KIND_ACTIVE
        b.balance, b.start, b.end = P(de.balance, i0 * n), P(de.start, i0 * n), P(de.end, i0 * n)
        b.dynasty, b.total_deposit = P(de.dynasty, i0), P(de.total_deposit, i0)
        b.natt, b.bits, b.boffs = natt, de.bits.data_ptr(), P(de.boffs, i0 * natt)
        b.max_inst_bytes = de.max_inst_bytes
        b.pop_rank, b.pop_world = de.rank, world
        b.committee, b.coffs = de.committee.data_ptr(), de.coffs.data_ptr()
        b.cpos = de.cpos.data_ptr() if de.cpos is not None else None
        b.att_comm, b.att_shard = P(de.att_comm, i0 * natt, 4), P(de.att_shard, i0 * natt, 4)
        b.nrec, b.rec_dynasty, b.winner = nrec, P(de.rec_dynasty, i0 * nrec), P(de.winner, i0 * nrec, 4)
        b.act_mask, b.blk_cnt, b.act_list = P(de.act_mask, i0 * wl), P(de.blk_cnt, i0 * vbpi, 4), P(de.act_list, i0 * N, 4)
        self.batch = b
        self.bind()

    def bind(self):
        B, natt = self.B, self.batch.natt
        self.red = self.reds[self.cur]
        self.scal = self.red[:B * SCAL_COUNT]
        self.vote = self.red[B * SCAL_COUNT:B * SCAL_COUNT + B * natt]
        self.total = self.red[B * SCAL_COUNT + B * natt:]
        b = self.batch
        b.vote, b.total, b.scal = self.vote.data_ptr(), self.total.data_ptr(), self.scal.data_ptr()
        b.scal_next = self.reds[1 - self.cur].data_ptr()

    def flip(self):
        self.results_red = self.red
        self.cur = 1 - self.cur
        self.bind()


class DeviceEpoch:
    """B epoch instances resident on one GPU (one validator shard of each instance)."""

    def __init__(self, inst, device, rank=0, world=1, group=None, kernels=None, general=None, parts=None):
        """``kernels``: the pass implementations (default: the HIP library).  ``general``:
        run the multi-rank general rank path (all-gather of the active masks); by default
        it is enabled when some validator of some instance is not active at its dynasty.
        ``parts``: instance slices pipelined against each other's collectives (default 2
        at N > 1 when B >= 2, else 1)."""
        import torch
        self.torch = torch
        self.dev = torch.device(device)
        self.kernels = kernels or HipEpochKernels()
        self.rank, self.world, self.group = rank, world, group
        B, N = inst["ninst"], inst["nval"]
        if general is None:
            d = inst["dynasty"][:, None]
            general = not bool(np.all((inst["start"] <= d) & (d < inst["end"])))
        self.general = bool(general) and world > 1
        lo, hi = shard_range(N, rank, world)
        self.lo, self.hi = lo, hi
        n = hi - lo
        T = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        self.balance = T(inst["balance"][:, lo:hi].copy().view(np.int64))
        self.start = T(inst["start"][:, lo:hi].copy().view(np.int64))
        self.end = T(inst["end"][:, lo:hi].copy().view(np.int64))
        self.dynasty = T(inst["dynasty"].view(np.int64))
        self.total_deposit = T(inst["total_deposit"].view(np.int64))
        self.bits = T(np.concatenate([inst["bits"], np.zeros(16, np.uint8)]))
        self.boffs = T(inst["boffs"].view(np.int64))
        committee, coffs, cpos = inst["committee"], inst["coffs"], None
        if world > 1:  # this rank's members only (the crosslink gathers then shrink with N)
            committee, coffs, cpos = local_committees(committee, coffs, lo, hi, N, rank == 0)
        self.committee = T(committee.view(np.int32))
        self.coffs = T(coffs.view(np.int64))
        self.cpos = T(cpos.view(np.int32)) if cpos is not None else None
        self.att_comm = T(inst["att_comm"].view(np.int32))
        self.att_shard = T(inst["att_shard"].view(np.int32))
        self.rec_dynasty = T(inst["rec_dynasty"].view(np.int64))
        self.max_inst_bytes = inst["max_inst_bytes"]
        natt = inst["natt"]
        nrec = inst["rec_dynasty"].shape[1]
        self.B, self.N, self.n, self.natt, self.nrec = B, N, n, natt, nrec
        self.winner = torch.full((B * nrec,), -1, dtype=torch.int32, device=device)
        self.act_mask = torch.zeros(B * ((n + 63) // 64), dtype=torch.int64, device=device)
        self.blk_cnt = torch.zeros(B * ((n + 2047) // 2048 + 1), dtype=torch.int32, device=device)
        self.act_list = torch.zeros(max(B * N, 1), dtype=torch.int32, device=device)
        self.sw = shard_words(N, world)
        if parts is None:
            parts = 2 if (world > 1 and B >= 2) else 1
        cuts = [B * k // parts for k in range(parts + 1)]
        self.parts = [_Part(self, cuts[k], cuts[k + 1] - cuts[k]) for k in range(parts) if cuts[k + 1] > cuts[k]]
        self.batch = self.parts[0].batch  # (single-part tools)

    @property
    def red(self):
        return self.parts[0].red

    @property
    def scal(self):
        return self.parts[0].scal

    def _host_collectives(self):
        import torch.distributed as dist
        return self.dev.type == "cuda" and dist.get_backend(self.group) == "gloo"

    def _all_reduce(self, t, async_op=False):
        """Sum over ranks in place.  RCCL ("nccl") reduces device tensors over xGMI (with
        ``async_op`` the returned work makes the current stream wait on ``.wait()``); the
        gloo path (tests: several ranks sharing one GPU) reduces a host copy, synchronously."""
        import torch.distributed as dist
        if self._host_collectives():
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            t.copy_(h)
            return None
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)

    def _all_gather_masks(self, p):
        """act_mask [B][local words] of every rank -> gmask [world][B][sw] (rank-major), for
        the instances of part ``p``."""
        import torch.distributed as dist
        torch = self.torch
        sw = self.sw
        wl = self.act_mask.numel() // self.B
        send = p.mask_send.view(p.B, sw)
        send[:, :wl].copy_(self.act_mask.view(self.B, wl)[p.i0:p.i0 + p.B])
        if self._host_collectives():  # small: B * nval_global / 8 bytes
            bufs = [torch.empty(p.B * sw, dtype=torch.int64) for _ in range(self.world)]
            dist.all_gather(bufs, p.mask_send.cpu(), group=self.group)
            p.gmask.copy_(torch.cat(bufs))
        else:
            dist.all_gather_into_tensor(p.gmask, p.mask_send, group=self.group)

    def _stream_handle(self, stream):
        if self.dev.type != "cuda":
            return ctypes.c_void_p(0)
        s = stream if stream is not None else self.torch.cuda.current_stream(self.dev)
        return ctypes.c_void_p(s.cuda_stream)

    def step(self, stream=None):
        """One epoch transition of all B instances (enqueued on ``stream``; no host sync
        on a single GPU).  Results (``results()``) are in the buffers this step used.

        Multi-rank sequence, per part: count (local partial sums) -> all-reduce {scal, vote,
        total} -> [general path: all-gather active masks -> global compaction] -> finish
        (winners, rewards on the local shard, partial next-cycle balance) -> all-reduce of
        that column.  The parts are interleaved: part 1's count runs while part 0's sums are
        reduced, part 0's finish while part 1's are.  Integer sums mod 2^64 commute, so the
        result is bit-exact for any reduction order."""
        sh = self._stream_handle(stream)
        if self.world == 1:
            for p in self.parts:
                self.kernels.count(p.batch, sh)
                self.kernels.finish(p.batch, sh)
                p.flip()
            return
        works = []
        for p in self.parts:
            self.kernels.count(p.batch, sh)
            works.append(self._all_reduce(p.red, async_op=True))
        pending = []
        for p, w in zip(self.parts, works):
            if w is not None:
                w.wait()
            if self.general:
                self._all_gather_masks(p)
                self.kernels.gather_compact(p.batch, p.gmask.data_ptr(), self.world, self.sw,
                                            p.gblk.data_ptr(), sh)
            self.kernels.finish(p.batch, sh)
            col = p.scal.view(p.B, SCAL_COUNT)[:, _lib.SCAL_NEXT_BAL]
            nb = col.contiguous()
            pending.append((col, nb, self._all_reduce(nb, async_op=True)))
        for col, nb, w in pending:
            if w is not None:
                w.wait()
            col.copy_(nb)
        for p in self.parts:
            p.flip()

    def results(self):
        """Host copies: (balance [B][n] uint64, scal [B][8] uint64, vote, total, winner)."""
        cpu = lambda t: t.cpu().numpy()  # noqa: E731
        B = self.B
        scal, vote, total = [], [], []
        for p in self.parts:
            red = cpu(p.results_red).view(np.uint64)
            k = p.B * SCAL_COUNT
            scal.append(red[:k].reshape(p.B, SCAL_COUNT))
            vote.append(red[k:k + p.B * self.natt].reshape(p.B, -1))
            total.append(red[k + p.B * self.natt:].reshape(p.B, -1))
        return (cpu(self.balance).view(np.uint64).reshape(B, -1), np.concatenate(scal), np.concatenate(vote),
                np.concatenate(total), cpu(self.winner).view(np.uint32).reshape(B, -1))
