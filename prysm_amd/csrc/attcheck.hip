// processAttestation's checks for a batch of attestations, one lane each.
//
// Restates, in Go's order, blockchain/core.go:240-297 processAttestation with its helpers
// getSignedParentHashes (core.go:348-360: the RecentBlockHashes slice bounds),
// getAttesterIndices (core.go:363-374: the committee of (Slot - LastStateRecalc, ShardId))
// and validateAttesterBitfields (core.go:377-394: BitLength and zero trailing bits).  The
// comparisons keep Go's types: the slot window compares int(slot) with int(block slot), the
// slice bounds and the committee index are uint64 differences that wrap.
//
// Each attestation needs ~60 bytes of scalars and the last byte of its bitfield; the
// committee table (ShardAndCommitteesForSlots: 256 arrays of a few (shard, committee)
// pairs) is shared by all lanes and stays in L1/L2.  HBM-bound, no MFMA, no LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "runtime.h"

namespace pz {
namespace {

constexpr int kThreads = 256;

// One attestation's checks from its loaded scalars (Go's order; see the file comment).
// lastb: the bitfield's last byte when the caller supplies the column (b.last_byte), else -1
// (read from bits).
__device__ __forceinline__ void check_one(const pz_att_check_batch& b, uint64_t s, uint64_t bs, uint64_t js,
                                          uint64_t nob, uint64_t shard, uint64_t b0, uint64_t b1, int32_t* st_out,
                                          uint32_t* comm_out, uint64_t* pstart_out, int lastb = -1) {
  int32_t st = PZ_ATT_PROCESSED;
  uint32_t comm = UINT32_MAX;
  uint64_t pstart = 0;
  if ((int64_t)s > (int64_t)bs) {
    st = PZ_ATT_SLOT_HIGH;
  } else if ((int64_t)s < (int64_t)bs - PZ_CYCLE_LENGTH) {
    st = PZ_ATT_SLOT_LOW;
  } else if (js != b.last_justified_slot) {
    st = PZ_ATT_JUSTIFIED;
  } else {
    const uint64_t start = bs - s, end = bs - s - nob + PZ_CYCLE_LENGTH;
    const uint64_t idx = s - b.last_state_recalc;
    if (start > end || end > b.n_recent) {
      st = PZ_ERANGE;  // Go panics: slice bounds out of range (core.go:353)
    } else if (idx >= b.narr) {
      st = PZ_EINDEX;  // Go panics: index out of range (core.go:367)
    } else {
      pstart = start;
      for (uint64_t e = b.arr_offs[idx]; e < b.arr_offs[idx + 1]; ++e)
        if (b.arr_shard[e] == shard) {
          comm = b.arr_comm[e];
          break;
        }
      if (comm == UINT32_MAX) {
        st = PZ_ATT_NO_COMMITTEE;
      } else {
        const uint64_t k = b.coffs[comm + 1] - b.coffs[comm];
        const uint64_t blen = b1 - b0;
        if ((k + 7) / 8 != blen)
          st = PZ_ATT_BITFIELD_LEN;
        else if ((k & 7) && ((lastb >= 0 ? (uint32_t)lastb : (uint32_t)b.bits[b0 + blen - 1]) & (0xFFu >> (k & 7))))
          st = PZ_ATT_TRAILING_BITS;  // only when bits pad the byte
      }
    }
  }
  *st_out = st;
  *comm_out = comm;
  *pstart_out = pstart;
}

// One lane per attestation, 8-B column loads (any alignment).
extern "C" __global__ void __launch_bounds__(kThreads) pz_att_check_kernel(pz_att_check_batch b) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= b.natt) return;
  // every per-attestation column is loaded up front (independent loads in flight together);
  // only the committee table walk and the bitfield byte depend on them
  int32_t st;
  uint32_t comm;
  uint64_t pstart;
  check_one(b, b.slot[i], b.block_slot[i], b.justified_slot[i], b.n_oblique[i], b.shard_id[i], b.boffs[i],
            b.boffs[i + 1], &st, &comm, &pstart, b.last_byte ? (int)b.last_byte[i] : -1);
  b.status[i] = st;
  if (b.committee) b.committee[i] = comm;
  if (b.parents_start) b.parents_start[i] = pstart;
}

// Two attestations per lane with 16-B column loads and 8/16-B stores (every column and output
// 16-B aligned): half the memory instructions of the one-per-lane form and full-width
// streaming requests.
// NT: nontemporal column loads (every column is read once): 80 -> 67 us per 4 M attestations
// (tools/attcheck_probe.py, profiles/r02/attcheck_probe_r2o.txt).
// (The bitfield byte stays a cached load: a 64-B line holds ~2.5 bitfields, so a nontemporal
// byte load re-fetches it: 87 us against 67, profiles/r02/attcheck_probe_ntb_r2o.txt.)
__device__ __forceinline__ void att_check_x2_body(const pz_att_check_batch& b) {
  const uint64_t i = 2 * ((uint64_t)blockIdx.x * kThreads + threadIdx.x);
  if (i >= b.natt) return;
  if (i + 1 >= b.natt) {  // odd tail
    int32_t st;
    uint32_t comm;
    uint64_t pstart;
    check_one(b, b.slot[i], b.block_slot[i], b.justified_slot[i], b.n_oblique[i], b.shard_id[i], b.boffs[i],
              b.boffs[i + 1], &st, &comm, &pstart, b.last_byte ? (int)b.last_byte[i] : -1);
    b.status[i] = st;
    if (b.committee) b.committee[i] = comm;
    if (b.parents_start) b.parents_start[i] = pstart;
    return;
  }
  auto ld2 = [](const uint64_t* p) {
    typedef unsigned long long v2u __attribute__((ext_vector_type(2)));
    const v2u x = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
    return make_ulonglong2(x.x, x.y);
  };
  const ulonglong2 s = ld2(b.slot + i), bs = ld2(b.block_slot + i), js = ld2(b.justified_slot + i);
  const ulonglong2 nob = ld2(b.n_oblique + i), sh = ld2(b.shard_id + i), bo = ld2(b.boffs + i);
  const uint64_t bo2 = b.boffs[i + 2];
  // the caller's last-byte column: both bytes in one 2-B load (i is even), beside the columns
  int lb0 = -1, lb1 = -1;
  if (b.last_byte) {
    const uint32_t w = *reinterpret_cast<const uint16_t*>(b.last_byte + i);
    lb0 = (int)(w & 0xFF);
    lb1 = (int)(w >> 8);
  }
  int32_t st0, st1;
  uint32_t c0, c1;
  uint64_t p0, p1;
  check_one(b, s.x, bs.x, js.x, nob.x, sh.x, bo.x, bo.y, &st0, &c0, &p0, lb0);
  check_one(b, s.y, bs.y, js.y, nob.y, sh.y, bo.y, bo2, &st1, &c1, &p1, lb1);
  *reinterpret_cast<int2*>(b.status + i) = make_int2(st0, st1);
  if (b.committee) *reinterpret_cast<uint2*>(b.committee + i) = make_uint2(c0, c1);
  if (b.parents_start) *reinterpret_cast<ulonglong2*>(b.parents_start + i) = make_ulonglong2(p0, p1);
}

// (Measured and dropped: default-policy column loads, 80 against 67 us; nontemporal output stores,
// level -- profiles/r02/attcheck_probe_r2o.txt.)
extern "C" __global__ void __launch_bounds__(kThreads) pz_att_check_x2_kernel(pz_att_check_batch b) {
  att_check_x2_body(b);
}

// ---- round 6: persistent blocks with the committee table in LDS --------------------------------
// The x2 kernel is latency-bound (VALU-busy 0.15, counted traffic 1.00x): after its column loads
// every attestation walks the committee table in global memory -- arr_offs[idx], then
// arr_shard[e] entry by entry (a load per step, the exit data-dependent), arr_comm[e],
// coffs[comm], coffs[comm + 1] -- four to eight dependent L2 round trips per lane.  Here each
// block stages the table once into LDS as 32-bit words ({offsets | shards | committees |
// committee sizes}: the sizes resolved through coffs while staging), then its lanes loop over
// attestation pairs with the next pair's columns in flight while the current one is checked, so
// the walk is LDS lookups (~100 cycles each) under the next pair's HBM round trip.  A table too
// large for the LDS budget, or with a shard id or committee size past 32 bits, or malformed
// offsets, keeps the global walk (the same check_one) in every block.
constexpr int kPThreads = 512, kPBlocksPerCU = 3;  // (2: 47.7 us, 3: 46.7, 1: 52.3; profiles/r06/attcheck_probe_r6g.txt)
constexpr uint32_t kPTabWords = 12288;  // 48 KiB

struct PairLd {
  ulonglong2 s, bs, js, nob, sh, bo;
  uint64_t bo2;
  uint32_t lb;  // the two last bytes (last_byte column), else 0
};

__device__ __forceinline__ void load_pair(const pz_att_check_batch& b, uint64_t i, PairLd& x) {
  auto ld2 = [](const uint64_t* p) {
    typedef unsigned long long v2u __attribute__((ext_vector_type(2)));
    const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
    return make_ulonglong2(v.x, v.y);
  };
  x.s = ld2(b.slot + i), x.bs = ld2(b.block_slot + i), x.js = ld2(b.justified_slot + i);
  x.nob = ld2(b.n_oblique + i), x.sh = ld2(b.shard_id + i), x.bo = ld2(b.boffs + i);
  x.bo2 = b.boffs[i + 2];
  x.lb = b.last_byte ? (uint32_t)*reinterpret_cast<const uint16_t*>(b.last_byte + i) : 0u;
}

// check_one with the committee walk in the block's LDS table (same order and types)
__device__ __forceinline__ void check_one_lds(const pz_att_check_batch& b, const uint32_t* offs, const uint32_t* tsh,
                                              const uint32_t* tcm, const uint32_t* tkk, uint64_t s, uint64_t bs,
                                              uint64_t js, uint64_t nob, uint64_t shard, uint64_t b0, uint64_t b1,
                                              int32_t* st_out, uint32_t* comm_out, uint64_t* pstart_out, int lastb) {
  int32_t st = PZ_ATT_PROCESSED;
  uint32_t comm = UINT32_MAX;
  uint64_t pstart = 0;
  if ((int64_t)s > (int64_t)bs) {
    st = PZ_ATT_SLOT_HIGH;
  } else if ((int64_t)s < (int64_t)bs - PZ_CYCLE_LENGTH) {
    st = PZ_ATT_SLOT_LOW;
  } else if (js != b.last_justified_slot) {
    st = PZ_ATT_JUSTIFIED;
  } else {
    const uint64_t start = bs - s, end = bs - s - nob + PZ_CYCLE_LENGTH;
    const uint64_t idx = s - b.last_state_recalc;
    if (start > end || end > b.n_recent) {
      st = PZ_ERANGE;  // Go panics: slice bounds out of range (core.go:353)
    } else if (idx >= b.narr) {
      st = PZ_EINDEX;  // Go panics: index out of range (core.go:367)
    } else {
      pstart = start;
      uint64_t k = 0;
      const bool small = (shard >> 32) == 0;  // (every staged shard id is below 2^32)
      for (uint32_t e = offs[idx]; e < offs[idx + 1]; ++e)
        if (small && tsh[e] == (uint32_t)shard) {
          comm = tcm[e];
          k = tkk[e];
          break;
        }
      if (comm == UINT32_MAX) {
        st = PZ_ATT_NO_COMMITTEE;
      } else {
        const uint64_t blen = b1 - b0;
        if ((k + 7) / 8 != blen)
          st = PZ_ATT_BITFIELD_LEN;
        else if ((k & 7) && ((lastb >= 0 ? (uint32_t)lastb : (uint32_t)b.bits[b0 + blen - 1]) & (0xFFu >> (k & 7))))
          st = PZ_ATT_TRAILING_BITS;  // only when bits pad the byte
      }
    }
  }
  *st_out = st;
  *comm_out = comm;
  *pstart_out = pstart;
}

__device__ __forceinline__ void check_pair(const pz_att_check_batch& b, bool lds, const uint32_t* offs,
                                           const uint32_t* tsh, const uint32_t* tcm, const uint32_t* tkk, uint64_t i,
                                           const PairLd& x) {
  const int lb0 = b.last_byte ? (int)(x.lb & 0xFF) : -1, lb1 = b.last_byte ? (int)(x.lb >> 8) : -1;
  int32_t st0, st1;
  uint32_t c0, c1;
  uint64_t p0, p1;
  if (lds) {
    check_one_lds(b, offs, tsh, tcm, tkk, x.s.x, x.bs.x, x.js.x, x.nob.x, x.sh.x, x.bo.x, x.bo.y, &st0, &c0, &p0, lb0);
    check_one_lds(b, offs, tsh, tcm, tkk, x.s.y, x.bs.y, x.js.y, x.nob.y, x.sh.y, x.bo.y, x.bo2, &st1, &c1, &p1, lb1);
  } else {
    check_one(b, x.s.x, x.bs.x, x.js.x, x.nob.x, x.sh.x, x.bo.x, x.bo.y, &st0, &c0, &p0, lb0);
    check_one(b, x.s.y, x.bs.y, x.js.y, x.nob.y, x.sh.y, x.bo.y, x.bo2, &st1, &c1, &p1, lb1);
  }
  *reinterpret_cast<int2*>(b.status + i) = make_int2(st0, st1);
  if (b.committee) *reinterpret_cast<uint2*>(b.committee + i) = make_uint2(c0, c1);
  if (b.parents_start) *reinterpret_cast<ulonglong2*>(b.parents_start + i) = make_ulonglong2(p0, p1);
}

extern "C" __global__ void __launch_bounds__(kPThreads) pz_att_check_p_kernel(pz_att_check_batch b) {
  __shared__ uint32_t tab[kPTabWords];
  const int tid = threadIdx.x;
  const uint64_t npairs = b.natt / 2, stride = (uint64_t)gridDim.x * kPThreads;
  uint64_t p = (uint64_t)blockIdx.x * kPThreads + tid;
  // the first pair's columns go out before the table's loads
  PairLd cur;
  bool have = p < npairs;
  if (have) load_pair(b, 2 * p, cur);
  // stage the table: {arr_offs (narr + 1) | shard | committee | committee size (ne each)}
  const uint64_t narr = b.narr;
  const uint64_t ne = narr ? b.arr_offs[narr] : 0;
  bool ok = narr + 1 + 3 * ne <= kPTabWords;
  uint32_t* offs = tab;
  uint32_t* tsh = tab + (ok ? narr + 1 : 0);
  uint32_t* tcm = tsh + (ok ? ne : 0);
  uint32_t* tkk = tcm + (ok ? ne : 0);
  if (ok) {
    for (uint64_t a = tid; a <= narr; a += kPThreads) {
      const uint64_t o = b.arr_offs[a];
      ok = ok && o <= ne && (a == 0 || b.arr_offs[a - 1] <= o);
      offs[a] = (uint32_t)o;
    }
    for (uint64_t e = tid; e < ne; e += kPThreads) {
      const uint64_t sh = b.arr_shard[e];
      const uint32_t c = b.arr_comm[e];
      const uint64_t k = b.coffs[(uint64_t)c + 1] - b.coffs[c];
      ok = ok && (sh >> 32) == 0 && (k >> 32) == 0;
      tsh[e] = (uint32_t)sh, tcm[e] = c, tkk[e] = (uint32_t)k;
    }
  }
  const bool lds = __syncthreads_and(ok ? 1 : 0) != 0;
  while (have) {  // (lanes leave independently: no barrier below)
    const uint64_t q = p + stride;
    const bool hq = q < npairs;
    PairLd nx;
    if (hq) load_pair(b, 2 * q, nx);
    check_pair(b, lds, offs, tsh, tcm, tkk, 2 * p, cur);
    cur = nx;
    p = q;
    have = hq;
  }
  // the odd tail: the last attestation alone, by the grid's first lane
  if ((b.natt & 1) && blockIdx.x == 0 && tid == 0) {
    const uint64_t i = b.natt - 1;
    int32_t st;
    uint32_t comm;
    uint64_t pstart;
    check_one(b, b.slot[i], b.block_slot[i], b.justified_slot[i], b.n_oblique[i], b.shard_id[i], b.boffs[i],
              b.boffs[i + 1], &st, &comm, &pstart, b.last_byte ? (int)b.last_byte[i] : -1);
    b.status[i] = st;
    if (b.committee) b.committee[i] = comm;
    if (b.parents_start) b.parents_start[i] = pstart;
  }
}

#ifdef PZ_AB_BUILD
static int g_attcheck_variant = 0;  // 1: round 5's x2 kernel (one pair per lane, the walk in global memory)
#endif

int check_args(const pz_att_check_batch* b) {
  if (!b) return fail(PZ_EINVAL, "batch is null");
  if (b->natt && (!b->slot || !b->justified_slot || !b->shard_id || !b->n_oblique || !b->boffs || !b->block_slot ||
                  !b->status))
    return fail(PZ_EINVAL, "null attestation column");
  if (b->narr && (!b->arr_offs || !b->arr_shard || !b->arr_comm || !b->coffs))
    return fail(PZ_EINVAL, "null committee table");
  return PZ_OK;
}

hipError_t launch_att_check(const pz_att_check_batch& b, hipStream_t s) {
  if (!b.natt) return hipSuccess;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const bool x2 = al(b.slot) && al(b.block_slot) && al(b.justified_slot) && al(b.n_oblique) && al(b.shard_id) &&
                  al(b.boffs) && (reinterpret_cast<uintptr_t>(b.status) & 7) == 0 &&
                  (!b.committee || (reinterpret_cast<uintptr_t>(b.committee) & 7) == 0) &&
                  (!b.parents_start || al(b.parents_start)) &&
                  (!b.last_byte || (reinterpret_cast<uintptr_t>(b.last_byte) & 1) == 0);
  bool persistent = x2 && b.natt >= 2;
#ifdef PZ_AB_BUILD
  if (g_attcheck_variant == 1) persistent = false;
#endif
  if (persistent) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                  hipSuccess || cus <= 0)
        cus = 256;
    }
    const uint64_t npairs = b.natt / 2;
    uint64_t per_cu = kPBlocksPerCU;
#ifdef PZ_AB_BUILD
    if (g_attcheck_variant == 2) per_cu = 2;  // (A/B: blocks per CU)
    if (g_attcheck_variant == 3) per_cu = 1;
#endif
    const uint64_t nb = std::max<uint64_t>(1, std::min<uint64_t>((npairs + kPThreads - 1) / kPThreads,
                                                                 (uint64_t)cus * per_cu));
    hipLaunchKernelGGL(pz_att_check_p_kernel, dim3((uint32_t)nb), dim3(kPThreads), 0, s, b);
  } else if (x2) {
    const uint64_t lanes = (b.natt + 1) / 2;
    hipLaunchKernelGGL(pz_att_check_x2_kernel, dim3((uint32_t)((lanes + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       s, b);
  } else {
    hipLaunchKernelGGL(pz_att_check_kernel, dim3((uint32_t)((b.natt + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       s, b);
  }
  return hipGetLastError();
}

}  // namespace
}  // namespace pz

using namespace pz;

extern "C" {

int pz_dev_check_attestations(const pz_att_check_batch* b, void* stream) {
  int rc = check_args(b);
  if (rc) return rc;
  hipError_t e = launch_att_check(*b, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_att_check_kernel");
}

int pz_check_attestations(const pz_att_check_batch* hb) {
  int rc = check_args(hb);
  if (rc) return rc;
  const uint64_t n = hb->natt;
  if (!n) return PZ_OK;
  if ((rc = check_csr(hb->boffs, n, "bitfield"))) return rc;
  if (hb->narr && (rc = check_csr(hb->arr_offs, hb->narr, "committee table"))) return rc;
  uint64_t ncomm = 0;  // committee ids must index coffs
  for (uint64_t e = 0; hb->narr && e < hb->arr_offs[hb->narr]; ++e)
    ncomm = std::max<uint64_t>(ncomm, (uint64_t)hb->arr_comm[e] + 1);
  DeviceCtx* c;
  if ((rc = acquire(&c))) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = c->ensure_stream())) return rc;
  Stager st{c, c->stream};
  pz_att_check_batch d = *hb;
  d.slot = st.up(hb->slot, n);
  d.justified_slot = st.up(hb->justified_slot, n);
  d.shard_id = st.up(hb->shard_id, n);
  d.n_oblique = st.up(hb->n_oblique, n);
  d.block_slot = st.up(hb->block_slot, n);
  std::vector<uint64_t> bo = rebase(hb->boffs, n);
  d.bits = st.up(hb->bits ? hb->bits + hb->boffs[0] : nullptr, bo[n]);
  d.boffs = st.up(bo.data(), n + 1);
  if (hb->narr) {
    const uint64_t ne = hb->arr_offs[hb->narr];
    d.arr_offs = st.up(hb->arr_offs, hb->narr + 1);
    d.arr_shard = st.up(hb->arr_shard, ne);
    d.arr_comm = st.up(hb->arr_comm, ne);
    d.coffs = st.up(hb->coffs, ncomm + 1);
  }
  if (hb->last_byte) d.last_byte = st.up(hb->last_byte, n);
  d.status = st.up<int32_t>(nullptr, n);
  d.committee = hb->committee ? st.up<uint32_t>(nullptr, n) : nullptr;
  d.parents_start = hb->parents_start ? st.up<uint64_t>(nullptr, n) : nullptr;
  if (st.rc) return st.rc;
  st.check(launch_att_check(d, st.s), "pz_att_check_kernel");
  st.down(hb->status, d.status, n);
  if (hb->committee) st.down(hb->committee, d.committee, n);
  if (hb->parents_start) st.down(hb->parents_start, d.parents_start, n);
  return st.sync();
}

}  // extern "C"

#ifdef PZ_AB_BUILD
extern "C" int pz_debug_set_attcheck_variant(int v) {
  const int old = pz::g_attcheck_variant;
  pz::g_attcheck_variant = v;
  return old;
}
#endif
