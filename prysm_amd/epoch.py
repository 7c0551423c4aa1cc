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


def shard_range(nval_global, rank, world):
    """Contiguous validator range [lo, hi) of ``rank`` (balanced to within one validator)."""
    lo = nval_global * rank // world
    hi = nval_global * (rank + 1) // world
    return lo, hi


class DeviceEpoch:
    """B epoch instances resident on one GPU (one validator shard of each instance)."""

    def __init__(self, inst, device, rank=0, world=1, group=None):
        import torch
        self.torch = torch
        self.dev = device
        self.rank, self.world, self.group = rank, world, group
        B, N = inst["ninst"], inst["nval"]
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
        self.committee = T(inst["committee"].view(np.int32))
        self.coffs = T(inst["coffs"].view(np.int64))
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
        b = EpochBatch()
        b.ninst, b.nval, b.val_offset, b.nval_global = B, n, lo, N
        b.kind = _lib.KIND_ACTIVE
        b.balance, b.start, b.end = self.balance.data_ptr(), self.start.data_ptr(), self.end.data_ptr()
        b.dynasty, b.total_deposit = self.dynasty.data_ptr(), self.total_deposit.data_ptr()
        b.natt, b.bits, b.boffs = natt, self.bits.data_ptr(), self.boffs.data_ptr()
        b.max_inst_bytes = inst["max_inst_bytes"]
        b.pop_rank, b.pop_world = rank, world
        b.committee, b.coffs = self.committee.data_ptr(), self.coffs.data_ptr()
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

    def step(self, stream=None):
        """One epoch transition of all B instances (enqueued on ``stream``; no host sync).
        Results (``results()``) are in the buffer this step used."""
        torch = self.torch
        s = stream if stream is not None else torch.cuda.current_stream(self.dev)
        sh = ctypes.c_void_p(s.cuda_stream)
        lib.call("pz_dev_epoch_count", ctypes.byref(self.batch), sh)
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(self.red, op=dist.ReduceOp.SUM, group=self.group)
        lib.call("pz_dev_epoch_finish", ctypes.byref(self.batch), sh)
        if self.world > 1:
            import torch.distributed as dist
            col = self.scal.view(self.B, SCAL_COUNT)[:, _lib.SCAL_NEXT_BAL]
            nb = col.contiguous()
            dist.all_reduce(nb, op=dist.ReduceOp.SUM, group=self.group)
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
