"""TEST DOUBLE (test infrastructure only): a numpy model of the three device passes behind
``pz_dev_epoch_count`` / ``pz_dev_epoch_gather_compact`` / ``pz_dev_epoch_finish``
(prysm_amd/csrc/epoch.hip), operating on ONE rank's shard exactly as the kernels do: partial
sums over the shard, popcount chunks split by (pop_rank, pop_world), crosslink partial
tallies over the members the shard owns, rewards by global rank position.

It lets the multi-rank orchestration in ``tests/torch_epoch.py DeviceEpoch`` (shard ranges,
buffer layout, the collective sequence) run on CPU tensors under ``gloo`` with no GPU, so
that the N>1 path is covered here; the GPU test of the same orchestration uses the real
kernels (tests/test_multirank.py).  It is never used by the product.
"""
import ctypes

import numpy as np

from prysm_amd import _lib

U64 = np.uint64
POP_CHUNK = 16 * 256 * 4  # kPopBytesPerBlock


def _arr(ptr, dtype, n):
    dt = np.dtype(dtype)
    if not ptr or n == 0:
        return np.zeros(0, dt)
    return np.ctypeslib.as_array((ctypes.c_uint8 * (n * dt.itemsize)).from_address(ptr)).view(dt)


class _View:
    def __init__(self, b):
        self.b = b
        self.B, self.n, self.off, self.N = b.ninst, b.nval, b.val_offset, b.nval_global
        self.natt = b.natt
        B, n = self.B, self.n
        self.bal = _arr(b.balance, U64, B * n).reshape(B, n)
        self.start = _arr(b.start, U64, B * n).reshape(B, n)
        self.end = _arr(b.end, U64, B * n).reshape(B, n)
        self.dyn = _arr(b.dynasty, U64, B)
        self.tdep = _arr(b.total_deposit, U64, B)
        self.boffs = _arr(b.boffs, U64, B * self.natt + 1)
        self.bits = _arr(b.bits, np.uint8, int(self.boffs[-1]) if self.natt else 0)
        self.scal = _arr(b.scal, U64, B * 8).reshape(B, 8)
        self.scal_next = _arr(b.scal_next, U64, B * 8).reshape(B, 8) if b.scal_next else None
        self.vote = _arr(b.vote, U64, B * self.natt).reshape(B, self.natt)
        self.total = _arr(b.total, U64, B * self.natt).reshape(B, self.natt)
        self.wl = (n + 63) // 64
        self.mask = _arr(b.act_mask, U64, B * self.wl).reshape(B, self.wl)
        self.act_list = _arr(b.act_list, np.uint32, B * self.N).reshape(B, self.N)
        self.att_comm = _arr(b.att_comm, np.uint32, B * self.natt).reshape(B, self.natt)
        self.att_shard = _arr(b.att_shard, np.uint32, B * self.natt).reshape(B, self.natt)
        self.nrec = b.nrec
        self.rec_dyn = _arr(b.rec_dynasty, U64, B * self.nrec).reshape(B, self.nrec)
        self.winner = _arr(b.winner, np.uint32, B * self.nrec).reshape(B, self.nrec)
        self.coffs = _arr(b.coffs, U64, int(self._ncomm()) + 1)
        self.committee = _arr(b.committee, np.uint32, int(self.coffs[-1]) if self.coffs.size else 0)
        self.cpos = _arr(b.cpos, np.uint32, self.committee.size) if b.cpos else None

    def _ncomm(self):
        if not self.natt:
            return 0
        return int(_arr(self.b.att_comm, np.uint32, self.B * self.natt).max()) + 1

    def active(self, i):
        d = self.dyn[i]
        return (self.start[i] <= d) & (d < self.end[i])

    def bf(self, i, a):
        g = i * self.natt + a
        return self.bits[int(self.boffs[g]):int(self.boffs[g + 1])]


def _bit(bf, idx):
    return (bf[idx >> 3] >> (7 - (idx & 7))) & 1


def _pack_mask(act, words):
    out = np.zeros(words, dtype=U64)
    bits = np.zeros(words * 64, dtype=np.uint8)
    bits[:act.size] = act
    for j in range(64):
        out |= bits[j::64].astype(U64) << U64(j)
    return out


class NumpyEpochKernels:
    def count(self, b, stream):
        v = _View(b)
        with np.errstate(over="ignore"):
            for i in range(v.B):
                act = v.active(i)
                v.scal[i, _lib.SCAL_NACT] += U64(act.sum())
                if v.wl:
                    v.mask[i] = _pack_mask(act, v.wl)
                if act.any():
                    m = v.off + int(np.nonzero(act)[0].max()) + 1
                    v.scal[i, _lib.SCAL_MAXIDX1] = max(int(v.scal[i, _lib.SCAL_MAXIDX1]), m)
                    L = v.bf(i, v.natt - 1).size if v.natt else 0
                    if v.natt == 0 or m - 1 >= 8 * L:
                        v.scal[i, _lib.SCAL_ERR_RWD] += U64(1)
                if v.natt:
                    beg, end = int(v.boffs[i * v.natt]), int(v.boffs[(i + 1) * v.natt])
                    for c, cb in enumerate(range(beg, end, POP_CHUNK)):
                        if c % b.pop_world == b.pop_rank:
                            seg = v.bits[cb:min(end, cb + POP_CHUNK)]
                            v.scal[i, _lib.SCAL_POP] += U64(np.unpackbits(seg).sum())
                if v.nrec:
                    v.winner[i] = 0xFFFFFFFF
                for a in range(v.natt if b.committee else 0):
                    c = int(v.att_comm[i, a])
                    lo_, hi_ = int(v.coffs[c]), int(v.coffs[c + 1])
                    mem = v.committee[lo_:hi_].astype(np.int64)
                    # bit position: index in the full committee (rank-local rows carry cpos)
                    pos = v.cpos[lo_:hi_].astype(np.int64) if v.cpos is not None else np.arange(mem.size)
                    bf = v.bf(i, a)
                    err = 0
                    if mem.size and mem.max() >= v.N:
                        err |= 1
                    if pos.size and pos.max() >= 8 * bf.size:
                        err |= 2
                    own = (mem >= v.off) & (mem < v.off + v.n) & (mem < v.N)
                    bal = np.zeros(mem.size, dtype=U64)
                    bal[own] = v.bal[i, mem[own] - v.off]
                    voted = np.zeros(mem.size, dtype=bool)
                    ok = pos < 8 * bf.size
                    voted[ok] = _bit(bf, pos[ok]).astype(bool)
                    v.total[i, a] = bal.sum(dtype=U64)
                    v.vote[i, a] = bal[voted].sum(dtype=U64)
                    if err:
                        v.scal[i, _lib.SCAL_ERR_XL] += U64(err)

    def gather_compact(self, b, gmask_ptr, world, sw, gblk_ptr, stream):
        v = _View(b)
        g = _arr(gmask_ptr, U64, world * v.B * sw).reshape(world, v.B, sw)
        for i in range(v.B):
            if int(v.scal[i, _lib.SCAL_NACT]) == v.N:
                continue
            words = g[:, i, :].reshape(-1)
            bits = ((words[:, None] >> np.arange(64, dtype=U64)[None, :]) & U64(1)).astype(bool).reshape(-1)
            idx = np.nonzero(bits[:v.N])[0].astype(np.uint32)
            v.act_list[i, :idx.size] = idx

    def finish(self, b, stream):
        v = _View(b)
        with np.errstate(over="ignore"):
            for i in range(v.B):
                if v.nrec and b.committee:
                    for a in range(v.natt):
                        if U64(3) * v.vote[i, a] >= U64(2) * v.total[i, a]:
                            s = int(v.att_shard[i, a])
                            if s >= v.nrec:
                                v.scal[i, _lib.SCAL_ERR_XL] += U64(4)
                            elif v.dyn[i] > v.rec_dyn[i, s]:
                                v.winner[i, s] = min(int(v.winner[i, s]), a)
                act = v.active(i)
                if v.n == v.N:  # single rank: local compaction
                    idx = np.nonzero(act)[0].astype(np.uint32)
                    v.act_list[i, :idx.size] = idx
                sc = v.scal[i]
                pop, nact = sc[_lib.SCAL_POP], int(sc[_lib.SCAL_NACT])
                thr = pop * U64(32) * U64(3) >= v.tdep[i] * U64(2)
                skip = sc[_lib.SCAL_ERR_XL] != 0 or (thr and nact > 0 and sc[_lib.SCAL_ERR_RWD] != 0)
                applied = bool(thr and not skip)
                all_active = nact == v.N
                lastbf = v.bf(i, v.natt - 1) if v.natt else None
                gp = v.off + np.arange(v.n)
                if applied:
                    sel = gp < nact
                    idx = gp[sel] if all_active else v.act_list[i, gp[sel]].astype(np.int64)
                    up = _bit(lastbf, idx).astype(bool)
                    v.bal[i, sel] = np.where(up, v.bal[i, sel] + U64(1), v.bal[i, sel] - U64(1))
                s = v.bal[i].sum(dtype=U64) if all_active else v.bal[i, act].sum(dtype=U64)
                if not skip:
                    sc[_lib.SCAL_NEXT_BAL] += s
                sc[_lib.SCAL_APPLIED] = 1 if applied else 0
                if v.scal_next is not None:
                    v.scal_next[i] = 0
