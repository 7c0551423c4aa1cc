"""Device-resident mirror of the epoch-transition state (SoA in HBM) and its drivers.

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


class DeviceEpoch:
    """B epoch instances resident on one GPU (one validator shard of each instance)."""

    def __init__(self, inst, device, rank=0, world=1, group=None, kernels=None, general=None):
        """``kernels``: the pass implementations (default: the HIP library).  ``general``:
        run the multi-rank general rank path (all-gather of the active masks); by default
        it is enabled when some validator of some instance is not active at its dynasty."""
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
        natt = inst["natt"]
        nrec = inst["rec_dynasty"].shape[1]
        # {scal, vote, total} contiguous: one all-reduce combines every partial sum.  Two such
        # buffers ping-pong: the finish pass of step k zeroes the scal of step k+1, so no
        # memset launch is needed per step.
        self.reds = [torch.zeros(B * SCAL_COUNT + 2 * B * natt, dtype=torch.int64, device=device)
                     for _ in range(2)]
        self.cur = 0
        self._bind_red(B, natt)
        self.winner = torch.full((B * nrec,), -1, dtype=torch.int32, device=device)
        self.act_mask = torch.zeros(B * ((n + 63) // 64), dtype=torch.int64, device=device)
        self.blk_cnt = torch.zeros(B * ((n + 2047) // 2048 + 1), dtype=torch.int32, device=device)
        self.act_list = torch.zeros(max(B * N, 1), dtype=torch.int32, device=device)
        self.sw = shard_words(N, world)
        if self.general:
            # this rank's mask padded to the common shard width, the gathered stack, and the
            # per-chunk counts of the global compaction
            self.mask_send = torch.zeros(B * self.sw, dtype=torch.int64, device=device)
            self.gmask = torch.zeros(world * B * self.sw, dtype=torch.int64, device=device)
            self.gblk = torch.zeros(B * ((N + 2047) // 2048), dtype=torch.int32, device=device)
        b = EpochBatch()
        b.ninst, b.nval, b.val_offset, b.nval_global = B, n, lo, N
        b.kind = _lib.KIND_ACTIVE
        b.balance, b.start, b.end = self.balance.data_ptr(), self.start.data_ptr(), self.end.data_ptr()
        b.dynasty, b.total_deposit = self.dynasty.data_ptr(), self.total_deposit.data_ptr()
        b.natt, b.bits, b.boffs = natt, self.bits.data_ptr(), self.boffs.data_ptr()
        b.max_inst_bytes = inst["max_inst_bytes"]
        b.pop_rank, b.pop_world = rank, world
        b.committee, b.coffs = self.committee.data_ptr(), self.coffs.data_ptr()
        b.cpos = self.cpos.data_ptr() if self.cpos is not None else None
        b.att_comm, b.att_shard = self.att_comm.data_ptr(), self.att_shard.data_ptr()
        b.nrec, b.rec_dynasty, b.winner = nrec, self.rec_dynasty.data_ptr(), self.winner.data_ptr()
        b.act_mask, b.blk_cnt, b.act_list = (self.act_mask.data_ptr(), self.blk_cnt.data_ptr(),
                                             self.act_list.data_ptr())
        self.batch = b
        self.B, self.N, self.natt, self.nrec = B, N, natt, nrec
        self._point_batch()

    def _bind_red(self, B, natt):
        self.red = self.reds[self.cur]
        self.scal = self.red[:B * SCAL_COUNT]
        self.vote = self.red[B * SCAL_COUNT:B * SCAL_COUNT + B * natt]
        self.total = self.red[B * SCAL_COUNT + B * natt:]

    def _point_batch(self):
        b = self.batch
        b.vote, b.total, b.scal = self.vote.data_ptr(), self.total.data_ptr(), self.scal.data_ptr()
        b.scal_next = self.reds[1 - self.cur].data_ptr()

    def _host_collectives(self):
        import torch.distributed as dist
        return self.dev.type == "cuda" and dist.get_backend(self.group) == "gloo"

    def _all_reduce(self, t):
        """Sum over ranks in place.  RCCL ("nccl") reduces device tensors over xGMI; the gloo
        path (tests: several ranks sharing one GPU) reduces a host copy."""
        import torch.distributed as dist
        if self._host_collectives():
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def _all_gather_masks(self):
        """act_mask [B][local words] of every rank -> gmask [world][B][sw] (rank-major)."""
        import torch.distributed as dist
        torch = self.torch
        B, sw = self.B, self.sw
        wl = self.act_mask.numel() // B
        send = self.mask_send.view(B, sw)
        send[:, :wl].copy_(self.act_mask.view(B, wl))
        if self._host_collectives():  # small: B * nval_global / 8 bytes
            parts = [torch.empty(B * sw, dtype=torch.int64) for _ in range(self.world)]
            dist.all_gather(parts, self.mask_send.cpu(), group=self.group)
            self.gmask.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(self.gmask, self.mask_send, group=self.group)

    def _stream_handle(self, stream):
        if self.dev.type != "cuda":
            return ctypes.c_void_p(0)
        s = stream if stream is not None else self.torch.cuda.current_stream(self.dev)
        return ctypes.c_void_p(s.cuda_stream)

    def step(self, stream=None):
        """One epoch transition of all B instances (enqueued on ``stream``; no host sync
        on a single GPU).  Results (``results()``) are in the buffer this step used.

        Multi-rank sequence: count (local partial sums) -> all-reduce {scal, vote, total}
        -> [general path: all-gather active masks -> global compaction] -> finish (winners,
        rewards on the local shard, partial next-cycle balance) -> all-reduce of that column.
        Integer sums mod 2^64 commute, so the result is bit-exact for any reduction order."""
        sh = self._stream_handle(stream)
        self.kernels.count(self.batch, sh)
        if self.world > 1:
            self._all_reduce(self.red)
            if self.general:
                self._all_gather_masks()
                self.kernels.gather_compact(self.batch, self.gmask.data_ptr(), self.world, self.sw,
                                            self.gblk.data_ptr(), sh)
        self.kernels.finish(self.batch, sh)
        if self.world > 1:
            col = self.scal.view(self.B, SCAL_COUNT)[:, _lib.SCAL_NEXT_BAL]
            nb = col.contiguous()
            self._all_reduce(nb)
            col.copy_(nb)
        self.last = self.cur
        self.cur = 1 - self.cur
        self.results_red = self.red
        self._bind_red(self.B, self.natt)
        self._point_batch()

    def results(self):
        """Host copies: (balance [B][n] uint64, scal [B][8] uint64, vote, total, winner)."""
        cpu = lambda t: t.cpu().numpy()  # noqa: E731
        B, natt = self.B, self.natt
        red = cpu(self.results_red).view(np.uint64)
        return (cpu(self.balance).view(np.uint64).reshape(B, -1),
                red[:B * SCAL_COUNT].reshape(B, SCAL_COUNT),
                red[B * SCAL_COUNT:B * SCAL_COUNT + B * natt].reshape(B, -1),
                red[B * SCAL_COUNT + B * natt:].reshape(B, -1),
                cpu(self.winner).view(np.uint32).reshape(B, -1))
