// proto3 encoding of ValidatorRecord columns on the device.
//
// Replaces the validators span of gogo `proto.Marshal(CrystallizedState)` at
// types/state.go:141 (Marshal) and :240 (Hash); the record is messages.pb.go:803-809
// (public_key 1, withdrawal_shard 2, withdrawal_address 3, randao_commitment 4, balance 5,
// start_dynasty 6, end_dynasty 7).  proto3 rules: ascending field order, zero scalars and
// empty bytes omitted, every record framed as a length-delimited repeated field.
//
// One launch (after a one-dispatch reset of the tile-status words).  A workgroup takes a tile
// of records, derives their encoded sizes, scans them, and learns the tile's output offset by
// a decoupled look-back over its predecessors' published sizes.  Then it writes the tile's
// bytes.  This is HBM-bound byte work, with no MFMA, and the columns are read once.
//  * Scalar-only records (no bytes fields; the chain's CrystallizedState): 4,096 records per
//    512-thread tile, loaded with coalesced column loads and held in registers.  The tile's
//    encoding is built in a 64 KiB LDS stage while the look-back is in flight and stored with
//    16-B stores.  A tile larger than the stage (records averaging over 16 bytes) writes lane
//    by lane instead.
//  * Records with bytes fields: 4,096 records per tile, sizes first, then (after the
//    look-back) a second read of the records, written lane by lane straight to HBM.
#include "wire.h"

#include <hip/hip_runtime.h>

#include <algorithm>


#include "runtime.h"

namespace pz {
namespace {

constexpr int kThreads = 512;
// scalar kernel: sub-tiles of kThreads x kPer = 2,048 records, kSub of them (4,096 records, one
// ticket) per tile, and a 64 KiB stage for the tile's encoding (16 B per record); wire_val_body
// derives these from its PER parameter
constexpr int kPer = 4, kSub = 2;
constexpr int kBytesSub = 8, kBytesTileRecs = kBytesSub * kThreads;  // bytes-field kernel: 4,096

// varint length: (70 - clz) / 7 for 70 - clz in [6, 70] as a multiply by 37 and a shift (a
// 24-bit multiply instead of the quarter-rate high multiply of a division by 7)
__device__ __forceinline__ uint32_t vlen(uint64_t x) { return ((uint32_t)(70 - __clzll(x | 1)) * 37u) >> 8; }

__device__ __forceinline__ uint8_t* put_varint(uint8_t* p, uint64_t x) {
  while (x >= 0x80) {
    *p++ = (uint8_t)(x | 0x80);
    x >>= 7;
  }
  *p++ = (uint8_t)x;
  return p;
}

__device__ __forceinline__ uint32_t frame_size(const WireValArgs& a, uint64_t body) {
  return (uint32_t)(a.field ? a.tag_len + vlen(body) + body : body);
}

__device__ __forceinline__ uint8_t* put_frame(const WireValArgs& a, uint8_t* p, uint64_t body) {
  if (a.field) {
    p = put_varint(p, ((uint64_t)a.field << 3) | 2);
    p = put_varint(p, body);
  }
  return p;
}

// ---- scalar-only records -------------------------------------------------------------------
// NC = the number of non-NULL columns (WireValArgs.ccol/ctag, in field order): a record holds
// only those, so a tile's values fit in registers (3 columns for the chain's states).
template <int NC>
struct SRec {
  uint64_t v[NC > 0 ? NC : 1];
};

template <int NC>
__device__ __forceinline__ uint32_t srec_body(const SRec<NC>& r) {
  uint32_t body = 0;
#pragma unroll
  for (int k = 0; k < NC; ++k) body += r.v[k] ? 1 + vlen(r.v[k]) : 0;
  return body;
}

template <int NC>
__device__ __forceinline__ uint8_t* put_srec(const WireValArgs& a, const SRec<NC>& r, uint32_t body, uint8_t* p) {
  p = put_frame(a, p, body);
#pragma unroll
  for (int k = 0; k < NC; ++k)
    if (r.v[k]) {
      *p++ = (uint8_t)a.ctag[k];
      p = put_varint(p, r.v[k]);
    }
  return p;
}

// ---- records with bytes fields ---------------------------------------------------------------
struct Rec {
  uint64_t v[5];    // fields 1, 2, 5, 6, 7
  uint64_t b0, b1;  // byte offsets of fields 3, 4
  uint64_t l0, l1;  // their lengths
  uint64_t body, size;
};

__device__ __forceinline__ void load_rec(const WireValArgs& a, uint64_t i, Rec& r) {
  uint64_t body = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    r.v[k] = a.col[k] ? a.col[k][i] : 0;
    body += r.v[k] ? 1 + vlen(r.v[k]) : 0;
  }
  r.b0 = r.l0 = r.b1 = r.l1 = 0;
  if (a.wa_offs) {
    r.b0 = a.wa_offs[i];
    r.l0 = a.wa_offs[i + 1] - r.b0;
    body += r.l0 ? 1 + vlen(r.l0) + r.l0 : 0;
  }
  if (a.rc_offs) {
    r.b1 = a.rc_offs[i];
    r.l1 = a.rc_offs[i + 1] - r.b1;
    body += r.l1 ? 1 + vlen(r.l1) + r.l1 : 0;
  }
  r.body = body;
  r.size = a.field ? a.tag_len + vlen(body) + body : body;
}

__device__ __forceinline__ uint8_t* put_bytes(uint8_t* p, uint32_t tag, const uint8_t* src, uint64_t len) {
  if (!len) return p;
  *p++ = (uint8_t)tag;
  p = put_varint(p, len);
  for (uint64_t j = 0; j < len; ++j) p[j] = src[j];
  return p + len;
}

__device__ __forceinline__ void put_rec(const WireValArgs& a, const Rec& r, uint8_t* p) {
  p = put_frame(a, p, r.body);
  if (r.v[0]) { *p++ = 1 << 3; p = put_varint(p, r.v[0]); }
  if (r.v[1]) { *p++ = 2 << 3; p = put_varint(p, r.v[1]); }
  p = put_bytes(p, (3 << 3) | 2, a.wa + r.b0, r.l0);
  p = put_bytes(p, (4 << 3) | 2, a.rc + r.b1, r.l1);
  if (r.v[2]) { *p++ = 5 << 3; p = put_varint(p, r.v[2]); }
  if (r.v[3]) { *p++ = 6 << 3; p = put_varint(p, r.v[3]); }
  if (r.v[4]) { *p++ = 7 << 3; p = put_varint(p, r.v[4]); }
}

// ---- tile offsets ----------------------------------------------------------------------------
// Exclusive scan of one value per thread over the 512-thread block (shfl_up steps); returns the
// block total.  The scalar kernel scans its packed sizes with block_scan_packed (DPP) instead.
__device__ __forceinline__ uint64_t block_scan(uint64_t x, uint64_t* excl, uint64_t* lds4) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t inc = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(inc, d, 64);
    if (lane >= d) inc += y;
  }
  if (lane == 63) lds4[wid] = inc;
  __syncthreads();
  uint64_t before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) {
    before += w < wid ? lds4[w] : 0;
    total += lds4[w];
  }
  *excl = before + inc - x;
  return total;
}

// Inclusive scan of a u32 over the wave by DPP: row shifts 1, 2, 4, 8 (Hillis-Steele inside
// each 16-lane row; bound_ctrl feeds 0 where a shift leaves the row), then row broadcasts 15
// and 31 carry the row totals.  No LDS traffic (a __shfl_up is a ds_bpermute round trip).
__device__ __forceinline__ uint32_t wave_iscan_u32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast31
  return x;
}

// block_scan for values made of independent 16-bit lanes whose block sums stay below 2^16 (the
// scalar kernel's packed sub-tile sizes): each 32-bit half scans on its own, carry-free.
__device__ __forceinline__ uint64_t block_scan_packed(uint64_t x, uint64_t* excl, uint64_t* lds4) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t inc = ((uint64_t)wave_iscan_u32((uint32_t)(x >> 32)) << 32) | wave_iscan_u32((uint32_t)x);
  if (lane == 63) lds4[wid] = inc;
  __syncthreads();
  uint64_t before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) {
    before += w < wid ? lds4[w] : 0;
    total += lds4[w];
  }
  *excl = before + inc - x;
  return total;
}

// Tile status words: flag in the top two bits, value below.  A tile publishes its aggregate
// (A) as soon as it knows its size and its inclusive prefix (P) after the look-back.  Flag and
// value travel in one 64-bit word, so relaxed agent-scope atomics suffice (no fence, which on
// gfx950 would write back L2).
constexpr uint64_t kFlagA = 1ull << 62, kFlagP = 2ull << 62, kVal = kFlagA - 1;

__device__ __forceinline__ uint64_t ld_status(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A coherent re-read for the spin: an `sc1` load is served by this XCD's L2, which can hold a
// stale copy of another XCD's status line until it is evicted; an atomic is performed at the
// coherence point.  (Stale reads are safe -- flags only move 0 -> A -> P and every published
// value is final -- they only make the spin longer.)
__device__ __forceinline__ uint64_t ld_status_fresh(uint64_t* p) {
  return __hip_atomic_fetch_add(p, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Decoupled look-back by the whole workgroup: 512 threads x LB loads watch the 512*LB nearest
// predecessors at once, so one round trip usually reaches a published inclusive prefix even
// when every resident tile started together.  Entry q*512 + t of a window (distance from the
// tile) is thread t's q-th: each load instruction reads 64 consecutive status words (4 lines).
// Returns the exclusive prefix of `tile` to every thread.
constexpr int kLbPer = 4;

// First window's loads, issued early so their round trip overlaps other work.
template <int LB>
__device__ __forceinline__ void lookback_issue(uint64_t* status, uint64_t tile, uint64_t (&w)[LB]) {
#pragma unroll
  for (int q = 0; q < LB; ++q) {
    const int64_t idx = (int64_t)tile - 1 - (q * kThreads + threadIdx.x);
    w[q] = idx >= 0 ? ld_status(status + idx) : kFlagP;  // before tile 0: prefix 0
  }
}

// Sum of a u32 over the wave by DPP (no LDS traffic), returned to every lane: quad swaps,
// half-row and row mirrors, then the row broadcasts 15 and 31 into lane 63.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);   // quad_perm 1,0,3,2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false);   // quad_perm 2,3,0,1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xf, 0xf, false);  // row_half_mirror
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xf, 0xf, false);  // row_mirror
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast31
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// One look-back window reduced with ONE workgroup barrier (the scalar-only kernel).  Entry
// (q, thread t) sits at distance q*512 + t.  Every wave finds, by ballot, its nearest published
// prefix P and sums its entries per level by DPP; lane 0 publishes [nearest distance | sum of
// its entries before that P], the per-level sums and the P value.  After the barrier every
// thread combines the 8 waves' records: all entries nearer than the block's nearest P are
// aggregates, whose sums fit 32 bits (a scalar-only tile encodes to at most 4,096 x 61 B and
// a window holds at most 2,048 entries), plus the P itself.  `slots` is 8 waves x 4 u64.
// Returns the window's contribution; *found says whether it held a P.
template <int LB>
__device__ __forceinline__ uint64_t lookback_window_waves(const uint64_t (&w)[LB], uint64_t* slots, bool* found,
                                                          uint32_t* trace_first) {
  static_assert(LB <= 4, "per-level sums are packed two per slot");
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t dw = 0xffffffffu, pa = 0, T[4] = {0, 0, 0, 0};
  uint64_t pval = 0;
#pragma unroll
  for (int q = 0; q < LB; ++q) {
    const uint32_t v = (uint32_t)(w[q] & kVal);  // meaningful for aggregates only
    T[q] = wave_sum_u32(v);
    const uint64_t m = __ballot((w[q] >> 62) == 2);
    if (dw == 0xffffffffu && m) {  // wave-uniform
      const uint32_t lf = (uint32_t)__builtin_ctzll(m);
      dw = (uint32_t)q * kThreads + 64 * wv + lf;
      pa = wave_sum_u32(lane < lf ? v : 0);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w[q], (int)lf);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(w[q] >> 32), (int)lf);
      pval = (((uint64_t)hi << 32) | lo) & kVal;
    }
  }
  if (lane == 0) {
    slots[4 * wv + 0] = ((uint64_t)pa << 32) | dw;
    slots[4 * wv + 1] = ((uint64_t)T[1] << 32) | T[0];
    slots[4 * wv + 2] = ((uint64_t)T[3] << 32) | T[2];
    slots[4 * wv + 3] = pval;
  }
  __syncthreads();
  // Lane x < 8 of every wave reads wave x's record; the nearest P by 8 readlanes (scalar).
  constexpr int kW = kThreads / 64;
  static_assert(kW <= 64, "one lane per wave record");
  const uint32_t x = lane < kW ? lane : 0;
  const uint64_t s0 = slots[4 * x], s1 = slots[4 * x + 1], s2 = slots[4 * x + 2], s3 = slots[4 * x + 3];
  uint32_t first = 0xffffffffu, wf = 0;
#pragma unroll
  for (int y = 0; y < kW; ++y) {
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s0, y);
    if (d < first) first = d, wf = (uint32_t)y;
  }
  *found = first != 0xffffffffu;
  if (threadIdx.x == 0) *trace_first = first;  // tools/wire_trace.py: the nearest prefix's distance
  const uint32_t qf = *found ? first / kThreads : LB;
  const uint32_t tq[4] = {(uint32_t)s1, (uint32_t)(s1 >> 32), (uint32_t)s2, (uint32_t)(s2 >> 32)};
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < LB; ++q)
    if ((uint32_t)q < qf || ((uint32_t)q == qf && x < wf)) c += tq[q];
  if (lane == wf) c += (uint32_t)(s0 >> 32);  // the nearest P's wave: its aggregates before the P
  uint64_t sum = wave_sum_u32(lane < kW ? c : 0);
  if (*found) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s3, (int)wf);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(s3 >> 32), (int)wf);
    sum += ((uint64_t)hi << 32) | lo;
  }
  return sum;
}

template <int LB, bool kWaves = false>
__device__ uint64_t lookback_finish(uint64_t* status, uint64_t tile, uint64_t (&w)[LB], uint64_t* lds,
                                    uint32_t* lds_first, uint32_t* polls = nullptr, uint64_t* slots = nullptr,
                                    uint64_t* lbst = nullptr) {
  constexpr uint32_t kWin = kThreads * LB;
  uint64_t prefix = 0;
  int64_t j = (int64_t)tile - 1;
  for (uint32_t win = 0;; ++win) {
    // Poll with relaxed agent-scope (sc1) loads -- the R2 granule form of the HIP guide's
    // Guideline 16: every status word is written by an agent-scope atomic store -- and fall
    // back to the atomic re-read after 256 polls.  Polling by atomics alone made every
    // spinning tile queue at the memory-side atomic unit of the same few status lines
    // (~12 ns each): 295 us per 16.7 M records against 178 without the look-back.  A lane's
    // unpublished entries are re-read together: one round trip per poll, not one per entry.
    for (uint32_t spins = 0;; ++spins) {
      bool wait = false;
#pragma unroll
      for (int q = 0; q < LB; ++q) wait |= !(w[q] >> 62);
      if (!wait) break;
      if (polls) ++*polls;  // tools/ trace only
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int q = 0; q < LB; ++q) {
        const int64_t idx = j - (q * kThreads + threadIdx.x);
        if (!(w[q] >> 62)) w[q] = spins < 256 ? ld_status(status + idx) : ld_status_fresh(status + idx);
      }
    }
    if (lbst && win == 0 && threadIdx.x == 0) lbst[0] = wall_clock64();  // (trace: the flags all seen)
    if (kWaves) {  // slots alternate by window: a wave is at most one barrier ahead
      bool found;
      prefix += lookback_window_waves<LB>(w, slots + (win & 1) * 4 * (kThreads / 64), &found, lds_first);
      if (lbst && win == 0 && threadIdx.x == 0) lbst[1] = wall_clock64();  // (trace: the window reduced)
      if (found) return prefix;
      j -= kWin;
#pragma unroll
      for (int q = 0; q < LB; ++q) {
        const int64_t idx = j - (q * kThreads + threadIdx.x);
        w[q] = idx >= 0 ? ld_status(status + idx) : kFlagP;
      }
      continue;
    }
    // nearest published inclusive prefix (distance d = q * kThreads + threadIdx.x)
    if (threadIdx.x == 0) *lds_first = kWin;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < LB; ++q)
      if ((w[q] >> 62) == 2) {
        atomicMin(lds_first, q * kThreads + threadIdx.x);
        break;
      }
    __syncthreads();
    const uint32_t first = *lds_first;
    uint64_t part = 0;
#pragma unroll
    for (int q = 0; q < LB; ++q)
      if (q * kThreads + threadIdx.x <= first) part += w[q] & kVal;
    uint64_t e;
    prefix += block_scan(part, &e, lds);
    __syncthreads();
    if (first < kWin) return prefix;
    j -= kWin;
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int64_t idx = j - (q * kThreads + threadIdx.x);
      w[q] = idx >= 0 ? ld_status(status + idx) : kFlagP;
    }
  }
}

__device__ uint64_t lookback_block(uint64_t* status, uint64_t tile, uint64_t* lds, uint32_t* lds_first) {
  uint64_t w[kLbPer];
  lookback_issue<kLbPer>(status, tile, w);
  return lookback_finish<kLbPer>(status, tile, w, lds, lds_first);
}

// Store stage[0..span) at out+base with 16-B stores: bytes up to the first 16-aligned
// address, then 16-B chunks (each funnel-shifted out of five LDS words), then the tail.
template <bool kNt = false>
__device__ __forceinline__ void store_stage(uint8_t* out, uint64_t base, const uint32_t* stage, uint32_t span) {
  const uint8_t* st = reinterpret_cast<const uint8_t*>(stage);
  const uint32_t lead = (uint32_t)((16 - (base & 15)) & 15);
  const uint32_t head = lead < span ? lead : span;
  if (threadIdx.x < head) out[base + threadIdx.x] = st[threadIdx.x];
  const uint32_t nq = (span - head) >> 4, sh = head & 3;
  uint4* dst = reinterpret_cast<uint4*>(out + base + head);
  for (uint32_t j = threadIdx.x; j < nq; j += kThreads) {
    const uint32_t w0 = (head + 16 * j) >> 2;  // first LDS word of the chunk
    uint32_t x[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) x[k] = stage[w0 + k];
    const uint4 v = sh ? make_uint4(__builtin_amdgcn_alignbyte(x[1], x[0], sh), __builtin_amdgcn_alignbyte(x[2], x[1], sh),
                                    __builtin_amdgcn_alignbyte(x[3], x[2], sh), __builtin_amdgcn_alignbyte(x[4], x[3], sh))
                       : make_uint4(x[0], x[1], x[2], x[3]);
    if (kNt) {
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      v4u t;
      t.x = v.x, t.y = v.y, t.z = v.z, t.w = v.w;
      __builtin_nontemporal_store(t, reinterpret_cast<v4u*>(dst + j));
    } else {
      dst[j] = v;
    }
  }
  const uint32_t t0 = head + 16 * nq;
  if (t0 + threadIdx.x < span) out[base + t0 + threadIdx.x] = st[t0 + threadIdx.x];
}

// Record (j, p, t) of a tile = tile*kTileRecs + j*kSubRecs + p*kThreads + t: every column load
// of a wave reads 512 contiguous bytes.  kNt: nontemporal loads (the columns are read once;
// tools/wire_probe.py r2m: 164 -> 154 us per 16.7 M records).
template <int NC, bool kNt = false, int PER = kPer>
__device__ __forceinline__ void load_sub(const WireValArgs& a, uint64_t first, SRec<NC> (&r)[PER]) {
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const uint64_t i = first + p * kThreads + threadIdx.x;
#pragma unroll
    for (int k = 0; k < NC; ++k) r[p].v[k] = i < a.n ? (kNt ? __builtin_nontemporal_load(a.ccol[k] + i) : a.ccol[k][i]) : 0;
  }
}

// Sizes of one sub-tile's records and their offsets inside the sub-tile (record order), from
// ONE block scan: a record is at most 61 bytes and a sub-tile row p of 512 records at most
// 31,232, so the four rows' sizes travel as four 16-bit lanes of one u64.
template <int NC, bool kShflScan = false, int PER = kPer>
__device__ __forceinline__ uint32_t sub_offsets(const WireValArgs& a, uint64_t first, const SRec<NC> (&r)[PER],
                                                uint32_t (&off)[PER], uint64_t* lds) {
  static_assert(PER <= 4, "four 16-bit rows per scan");
  uint64_t packed = 0;
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const uint64_t i = first + p * kThreads + threadIdx.x;
    packed |= (uint64_t)(i < a.n ? frame_size(a, srec_body(r[p])) : 0) << (16 * p);
  }
  uint64_t e;
  const uint64_t t = kShflScan ? block_scan(packed, &e, lds) : block_scan_packed(packed, &e, lds);
  __syncthreads();  // lds is reused by the next scan
  uint32_t row = 0;
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    off[p] = row + (uint32_t)((e >> (16 * p)) & 0xffff);
    row += (uint32_t)((t >> (16 * p)) & 0xffff);
  }
  return row;
}

// One tile of kSub sub-tiles (4,096 records) per 512-thread workgroup, one ticket per tile.
// Phase 1 loads every column of the tile into registers at once (NC per record: only the
// non-NULL columns), sizes the records and scans each sub-tile (one block scan each); the tile
// publishes its size and issues the look-back's first window, builds its encoding in the
// 64 KiB LDS stage while that round trip is in flight, and after the look-back stores the
// stage with 16-B stores.  A tile whose encoding outgrows the stage (records averaging over
// 16 bytes), or a call that wants record offsets, writes lane by lane from registers instead.
// Tiles are large because a single contended ticket counter serialises its atomics (~11 ns).
// Measured (tools/wire_probe.py, 16.7 M records, us): r2b's 256-thread tiles of 2,048 with all
// five column slots in registers (152 VGPRs) 255; dropping the values after phase 1 and
// reloading them for the build (512-thread tiles) 241, but the reloads miss L2 (96 KiB per
// tile x 64 tiles per XCD > 4 MiB): 1,025 MB of traffic per launch against 654 algorithmic.
// Dropped: building the stage by dword ORs from a register accumulator instead of byte
// writes 305 (the 64-bit shifts cost more VALU than the LDS byte writes); persistent
// workgroups pipelining the next tile's phase 1 under the look-back 278 (128 VGPRs + spills).
// Round 2 (r2f-r2n): a coalesced look-back window without spills 175; its entries re-read
// halfway through the build, the window reduced by waves (one barrier), DPP sub-tile scans
// 163.5; nontemporal column loads 154.
// V: an ablation knob for tools/wire_probe.py (0 in the product; output wrong otherwise):
// bit 0 tile = blockIdx (no ticket), bit 1 no stage build, bit 2 no look-back, bit 3 no store,
// bit 4 reload the values for the build instead of holding them, bit 5 (the product plus)
// per-tile phase timestamps into a.trace (tools/wire_trace.py); bits 6/7 a look-back window of
// 1,024 / 512 predecessors instead of 2,048, bit 8 (trace) wait for the look-back's first
// window right after issuing it, to time its round trip, bit 9 no mid-build re-read of the
// window's unpublished entries, bit 10 the look-back window reduced by an LDS atomic and a
// block scan (four barriers) instead of by waves (one), bit 11 the sub-tile sizes scanned by
// __shfl_up (ds_bpermute) instead of DPP, bit 12 column loads with the default cache policy
// instead of nontemporal, bit 13 nontemporal output stores, bit 14 (tests) no inclusive
// prefixes published (every look-back walks back to tile 0; exact output).
// PER: records per thread per sub-tile (kPer in the product: 4,096-record tiles and a 64 KiB
// stage, two tiles per CU).  Smaller PER shrinks the tile, its stage and its held values
// (round 4 A/B: three tiles per CU at PER 3).
template <int V, int NC, int PER = kPer>
__device__ __forceinline__ void wire_val_body(WireValArgs a, uint32_t nt_arg) {
  // (the tile count held in an SGPR from the start: left to the compiler, its kernel-argument
  // load was re-issued after the look-back, and a scalar-cache miss there under the streaming
  // load cost ~2 us per tile -- tools/wire_trace.py's look-back tail)
  uint32_t nt = nt_arg;
  asm volatile("" : "+s"(nt));
  constexpr int kSubRecs = kThreads * PER, kTileRecs = kSub * kSubRecs, kStageBytes = 16 * kTileRecs;
  __shared__ uint64_t lds[kThreads / 64 + 1];
  __shared__ uint32_t s_tile, s_first, s_polls;
  __shared__ uint64_t s_build_end, s_lbslots[2 * 4 * (kThreads / 64)], s_lbst[4];
  __shared__ __attribute__((aligned(16))) uint32_t stage[kStageBytes / 4 + 8];
  uint64_t ts[6];
  if (V & 32) {
    ts[0] = wall_clock64();
    if (threadIdx.x == 0) s_build_end = 0, s_polls = 0;
  }
  if (V & 1) {
    if (threadIdx.x == 0) s_tile = blockIdx.x;
  } else if (threadIdx.x == 0) {
    s_tile = atomicAdd(a.ticket, 1u);
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  if (V & 32) ts[1] = wall_clock64();
  const uint64_t tfirst = (uint64_t)tile * kTileRecs;
  constexpr bool kHold = !(V & 16) && NC <= 3;  // 4-5 columns held would spill: reload them
  // phase 1: sizes -> offsets inside the tile
  SRec<NC> r[kSub][PER];
  // A record's body size is recomputed for its build rather than held: 8 more live VGPRs
  // spilled, and a spill reload's vmcnt(0) waited for the look-back loads in flight.
  uint32_t off[kSub][PER], agg = 0;
  if (kHold) {  // every sub-tile's loads in flight at once: one round trip, not kSub
#pragma unroll
    for (int j = 0; j < kSub; ++j) load_sub<NC, !(V & 4096), PER>(a, tfirst + (uint64_t)j * kSubRecs, r[j]);
  }
#pragma unroll
  for (int j = 0; j < kSub; ++j) {
    if (!kHold) load_sub<NC, false, PER>(a, tfirst + (uint64_t)j * kSubRecs, r[0]);
    const uint32_t sub =
        sub_offsets<NC, (V & 2048) != 0, PER>(a, tfirst + (uint64_t)j * kSubRecs, r[kHold ? j : 0], off[j], lds);
#pragma unroll
    for (int p = 0; p < PER; ++p) off[j][p] += agg;
    agg += sub;
  }
  // Every column load has landed (the scans used them).  Say so to the compiler's wait-count
  // pass: the loads sit under divergent branches, and without this it re-waits for them in
  // the stage build, where a vmcnt wait also drains the look-back loads issued below
  // (tools/wire_trace.py: the build took 6.8 us with them in flight, 4.7 without).
  __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt(0), expcnt/lgkmcnt untouched
  if (threadIdx.x == 0) st_status(a.status + tile, (tile == 0 ? kFlagP : kFlagA) | agg);
  if (V & 32) ts[2] = wall_clock64();
  // the look-back's first round trip overlaps the stage build
  constexpr int LB = (V & 128) ? 1 : (V & 64) ? 2 : kLbPer;  // window ablation (tools/)
  uint64_t w[LB];
  if (!(V & 4) && tile > 0) lookback_issue<LB>(a.status, tile, w);
  uint64_t ts_arrive = 0;
  uint32_t polls = 0;
  if (V & 256) {  // trace: the first window's round trip alone (no overlap with the build)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    ts_arrive = wall_clock64();
  }
  const bool staged = agg <= kStageBytes && !a.offs;
  if (staged && !(V & 2)) {
    uint8_t* st = reinterpret_cast<uint8_t*>(stage);
#pragma unroll
    for (int j = 0; j < kSub; ++j) {
      if (!kHold) load_sub<NC, false, PER>(a, tfirst + (uint64_t)j * kSubRecs, r[0]);
#pragma unroll
      for (int p = 0; p < PER; ++p)
        if (tfirst + j * kSubRecs + p * kThreads + threadIdx.x < a.n) {
          const SRec<NC>& rec = r[kHold ? j : 0][p];
          put_srec(a, rec, srec_body(rec), st + off[j][p]);
        }
      // Halfway through the build, re-read the window entries that were not yet published:
      // a predecessor that started just before this tile usually publishes while the first
      // window is in flight, and the re-read's round trip now overlaps the second half of the
      // build instead of following it (tools/wire_trace.py: one re-poll per tile, ~1.2 us).
      if (j == kSub / 2 - 1 && !(V & (512 | 4)) && tile > 0) {
#pragma unroll
        for (int q = 0; q < LB; ++q) {
          const int64_t idx = (int64_t)tile - 1 - (q * kThreads + threadIdx.x);
          if (!(w[q] >> 62)) w[q] = ld_status(a.status + idx);
        }
      }
    }
  }
  if (V & 32) {
    ts[3] = wall_clock64();
    if ((threadIdx.x & 63) == 0) atomicMax(&s_build_end, ts[3]);
  }
  uint64_t base = 0;
  if (V & 4) {
    base = (uint64_t)tile * 15 * kTileRecs;  // (ablation: output wrong)
  } else if (tile > 0) {
    base = lookback_finish<LB, !(V & 1024)>(a.status, tile, w, lds, &s_first, (V & 32) ? &polls : nullptr, s_lbslots,
                                            (V & 32) ? s_lbst : nullptr);
    if ((V & 32) && threadIdx.x == 0) s_lbst[2] = wall_clock64();  // (trace: returned)
    // (variant 16384, tests only: no inclusive prefix is published, so every look-back walks
    // window after window back to tile 0 -- the multi-window path, with exact output)
    if (threadIdx.x == 0 && !(V & 16384)) st_status(a.status + tile, kFlagP | (base + agg));
    if ((V & 32) && threadIdx.x == 0) s_lbst[3] = wall_clock64();  // (trace: prefix published)
    if (V & 32) {  // (a wave max first: an LDS atomic of a divergent value compiles to a 64-step lane loop)
      uint32_t m = polls;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
      if ((threadIdx.x & 63) == 0) atomicMax(&s_polls, m);
    }
  }
  if (tile == nt - 1 && threadIdx.x == 0) {
    *a.total = base + agg;
    if (a.offs) a.offs[a.n] = base + agg;
  }
  if (staged) {
    // the stage is complete: the wave-reduced look-back's barrier follows every wave's build
    if ((V & (4 | 1024)) || tile == 0) __syncthreads();
    if (V & 32) ts[4] = wall_clock64();
    if (!(V & 8)) store_stage<(V & 8192) != 0>(a.out, base, stage, agg);
    if (V & 32) {
      __syncthreads();
      ts[5] = wall_clock64();
      if (threadIdx.x == 0) {
        uint64_t* t = a.trace + 16 * (uint64_t)tile;
        for (int k = 0; k < 6; ++k) t[k] = ts[k];
        t[6] = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // XCC_ID
        t[7] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
        t[8] = (V & 256) ? ts_arrive : s_lbst[3];  // the first poll's arrival (256) or thread 0's prefix published
        t[9] = polls;                        // re-polls by thread 0 (the nearest entries)
        t[10] = tile > 0 ? s_first : 0;      // distance of the nearest published prefix (last window)
        t[11] = s_build_end;                 // the last wave's end of the stage build
        t[12] = s_polls;                     // re-polls, most of any thread
        t[13] = s_lbst[0];                   // thread 0: every window flag seen
        t[14] = s_lbst[1];                   // thread 0: the window reduced (after its barrier)
        t[15] = s_lbst[2];                   // thread 0: back from the look-back
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < kSub; ++j) {
    if (!kHold) load_sub<NC, false, PER>(a, tfirst + (uint64_t)j * kSubRecs, r[0]);
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const uint64_t i = tfirst + j * kSubRecs + p * kThreads + threadIdx.x;
      if (i < a.n) {
        const uint64_t o = base + off[j][p];
        if (a.offs) a.offs[i] = o;
        put_srec(a, r[kHold ? j : 0][p], srec_body(r[kHold ? j : 0][p]), a.out + o);
      }
    }
  }
}

#define PZ_WIRE_VAL_KERNEL(NAME, V, NC)                                        \
  extern "C" __global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) \
  NAME(WireValArgs a, uint32_t nt) {                                             \
    wire_val_body<V, NC>(a, nt);                                                 \
  }
PZ_WIRE_VAL_KERNEL(pz_wire_val_c0_kernel, 0, 0)
PZ_WIRE_VAL_KERNEL(pz_wire_val_c1_kernel, 0, 1)
PZ_WIRE_VAL_KERNEL(pz_wire_val_c2_kernel, 0, 2)
PZ_WIRE_VAL_KERNEL(pz_wire_val_kernel, 0, 3)  // the chain's states: balance, start, end
PZ_WIRE_VAL_KERNEL(pz_wire_val_c4_kernel, 0, 4)
PZ_WIRE_VAL_KERNEL(pz_wire_val_c5_kernel, 0, 5)
#ifdef PZ_AB_BUILD
// the A/B library only (make -C prysm_amd/csrc ab): per-tile phase stamps for tools/wire_trace.py,
// and the multi-window look-back path for tests (no inclusive prefix published: every tile walks
// back window after window to tile 0; exact output)
PZ_WIRE_VAL_KERNEL(pz_wire_val_v32_kernel, 32, 3)
PZ_WIRE_VAL_KERNEL(pz_wire_val_v16384_kernel, 16384, 3)
// trace forms (tools/wire_trace.py): 288 the first window's round trip timed alone, 36 no
// look-back (output wrong), 544 no mid-build re-read of the window
PZ_WIRE_VAL_KERNEL(pz_wire_val_v288_kernel, 288, 3)
PZ_WIRE_VAL_KERNEL(pz_wire_val_v36_kernel, 36, 3)
PZ_WIRE_VAL_KERNEL(pz_wire_val_v544_kernel, 544, 3)
#endif
#undef PZ_WIRE_VAL_KERNEL
// (Round 4 tile-geometry A/B, measured and dropped: 3,072-record tiles at 6 waves per SIMD and
// 2,048-record tiles at 6 or 8 spill their held values, profiles/r04/wire_geometry_dropped_r4g.txt.)

// Records with bytes fields: tiles of kBytesSub x 256 records, one per thread per sub-tile.
// Phase 1 scans the sizes; after the look-back, phase 2 reads the records again and writes
// each lane's record straight to HBM (a record has no size bound, so there is no stage).
extern "C" __global__ void __launch_bounds__(kThreads) pz_wire_val_bytes_kernel(WireValArgs a, uint32_t nt) {
  __shared__ uint64_t lds[kThreads / 64 + 1];
  __shared__ uint32_t s_tile, s_first;
  if (threadIdx.x == 0) s_tile = atomicAdd(a.ticket, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t tfirst = (uint64_t)tile * kBytesTileRecs + threadIdx.x;
  uint64_t excl[kBytesSub], sub_base[kBytesSub], agg = 0;
#pragma unroll
  for (int j = 0; j < kBytesSub; ++j) {
    const uint64_t i = tfirst + (uint64_t)j * kThreads;
    Rec r;
    uint64_t mine = 0;
    if (i < a.n) {
      load_rec(a, i, r);
      mine = r.size;
    }
    const uint64_t t = block_scan(mine, &excl[j], lds);
    __syncthreads();
    sub_base[j] = agg;
    agg += t;
  }
  if (threadIdx.x == 0) st_status(a.status + tile, (tile == 0 ? kFlagP : kFlagA) | agg);
  uint64_t base = 0;
  if (tile > 0) {
    base = lookback_block(a.status, tile, lds, &s_first);
    if (threadIdx.x == 0) st_status(a.status + tile, kFlagP | (base + agg));
  }
  if (tile == nt - 1 && threadIdx.x == 0) {
    *a.total = base + agg;
    if (a.offs) a.offs[a.n] = base + agg;
  }
#pragma unroll
  for (int j = 0; j < kBytesSub; ++j) {
    const uint64_t i = tfirst + (uint64_t)j * kThreads;
    if (i < a.n) {
      Rec r;
      load_rec(a, i, r);
      const uint64_t o = base + sub_base[j] + excl[j];
      if (a.offs) a.offs[i] = o;
      put_rec(a, r, a.out + o);
    }
  }
}

// Zeroes the look-back scratch: one dispatch (hipMemsetAsync of an odd number of 8-B words
// issued two ROCclr fill kernels, ~10 us per call).
extern "C" __global__ void __launch_bounds__(kThreads) pz_wire_zero_kernel(uint64_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kThreads) p[i] = 0;
}

}  // namespace

#ifdef PZ_AB_BUILD
static int g_wire_variant = 0;            // 32: trace (g_wire_trace), 16384: no inclusive prefixes
static uint64_t* g_wire_trace = nullptr;
#endif

static uint64_t tile_recs(bool bytes, int per) { return bytes ? kBytesTileRecs : (uint64_t)kSub * kThreads * per; }

uint64_t wire_tiles(uint64_t n) {  // scratch bound: the smallest tile of the kernels (PER 2)
  constexpr uint64_t t = kBytesTileRecs < kSub * kThreads * 2 ? kBytesTileRecs : kSub * kThreads * 2;
  return (n + t - 1) / t;
}

// Scratch: status[nt] then the ticket; zeroed before every launch.
hipError_t launch_wire_validators(WireValArgs a, uint64_t* scratch, hipStream_t s) {
  const bool bytes = a.wa_offs || a.rc_offs;
  a.nc = 0;  // the non-NULL columns, in field order (the scalar-only kernel holds only these)
  const uint32_t tags[5] = {1 << 3, 2 << 3, 5 << 3, 6 << 3, 7 << 3};
  for (int k = 0; k < 5; ++k)
    if (a.col[k]) {
      a.ccol[a.nc] = a.col[k];
      a.ctag[a.nc++] = tags[k];
    }
  const uint64_t tr = tile_recs(bytes, kPer);
  const uint64_t nt = (a.n + tr - 1) / tr;
  if (nt == 0) {
    hipError_t e = hipMemsetAsync(a.total, 0, 8, s);
    if (e == hipSuccess && a.offs) e = hipMemsetAsync(a.offs, 0, 8, s);
    return e;
  }
  a.status = scratch;
  a.ticket = reinterpret_cast<uint32_t*>(scratch + nt);
  {
    const uint64_t words = nt + 1;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(64, (words + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(pz_wire_zero_kernel, dim3(blocks), dim3(kThreads), 0, s, scratch, words);
  }
  if (bytes)
    hipLaunchKernelGGL(pz_wire_val_bytes_kernel, dim3((uint32_t)nt), dim3(kThreads), 0, s, a, (uint32_t)nt);
  else
  {
    const dim3 g((uint32_t)nt), b(kThreads);
    const uint32_t n32 = (uint32_t)nt;
#ifdef PZ_AB_BUILD
    if (g_wire_variant && a.nc == 3) {
      if (g_wire_variant == 32 || g_wire_variant == 288 || g_wire_variant == 36 || g_wire_variant == 544) {
        if (!g_wire_trace) return hipErrorInvalidValue;
        a.trace = g_wire_trace;
        const void* k = g_wire_variant == 288 ? (const void*)pz_wire_val_v288_kernel
                        : g_wire_variant == 36 ? (const void*)pz_wire_val_v36_kernel
                        : g_wire_variant == 544 ? (const void*)pz_wire_val_v544_kernel
                                                : (const void*)pz_wire_val_v32_kernel;
        void* args[] = {&a, const_cast<uint32_t*>(&n32)};
        if (hipLaunchKernel(k, g, b, args, 0, s) != hipSuccess) return hipGetLastError();
      } else if (g_wire_variant == 16384) {
        hipLaunchKernelGGL(pz_wire_val_v16384_kernel, g, b, 0, s, a, n32);
      } else {
        return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
#endif
    {
      switch (a.nc) {
        case 0: hipLaunchKernelGGL(pz_wire_val_c0_kernel, g, b, 0, s, a, n32); break;
        case 1: hipLaunchKernelGGL(pz_wire_val_c1_kernel, g, b, 0, s, a, n32); break;
        case 2: hipLaunchKernelGGL(pz_wire_val_c2_kernel, g, b, 0, s, a, n32); break;
        case 3: hipLaunchKernelGGL(pz_wire_val_kernel, g, b, 0, s, a, n32); break;
        case 4: hipLaunchKernelGGL(pz_wire_val_c4_kernel, g, b, 0, s, a, n32); break;
        default: hipLaunchKernelGGL(pz_wire_val_c5_kernel, g, b, 0, s, a, n32);
      }
    }
  }
  return hipGetLastError();
}

#ifdef PZ_AB_BUILD
int set_wire_variant(int v) {
  const int old = g_wire_variant;
  g_wire_variant = v;
  return old;
}

void set_wire_trace(uint64_t* dev) { g_wire_trace = dev; }
#endif

int wire_val_args(const pz_validator_cols* v, uint64_t n, uint32_t field_num, WireValArgs* a) {
  if (!v) return fail(PZ_EINVAL, "columns are null");
  if (field_num >= (1u << 29)) return fail(PZ_EINVAL, "field number %u out of range", field_num);
  if ((v->withdrawal_address_offs && !v->withdrawal_address) ||
      (v->randao_commitment_offs && !v->randao_commitment))
    return fail(PZ_EINVAL, "bytes column without data");
  *a = WireValArgs{};
  a->col[0] = v->public_key;
  a->col[1] = v->withdrawal_shard;
  a->col[2] = v->balance;
  a->col[3] = v->start_dynasty;
  a->col[4] = v->end_dynasty;
  a->wa = v->withdrawal_address;
  a->wa_offs = v->withdrawal_address_offs;
  a->rc = v->randao_commitment;
  a->rc_offs = v->randao_commitment_offs;
  a->n = n;
  a->field = field_num;
  uint64_t tag = ((uint64_t)field_num << 3) | 2;
  a->tag_len = 1;
  while (tag >= 0x80) {
    tag >>= 7;
    ++a->tag_len;
  }
  return PZ_OK;
}

}  // namespace pz

using namespace pz;

extern "C" {

uint64_t pz_wire_validators_bound(uint64_t n, uint64_t bytes_total) { return n * 92 + bytes_total; }

uint64_t pz_wire_scratch_bytes(uint64_t n) { return (wire_tiles(n) + 1) * 8; }

#ifdef PZ_AB_BUILD
int pz_debug_set_wire_variant(int v) { return set_wire_variant(v); }

void pz_debug_set_wire_trace(void* dev) { set_wire_trace(static_cast<uint64_t*>(dev)); }
#endif

int pz_dev_wire_validators(const pz_validator_cols* v, uint64_t n, uint32_t field_num, uint8_t* d_out,
                           uint64_t* d_offsets, void* d_scratch, uint64_t* d_total, void* stream) {
  WireValArgs a;
  int rc = wire_val_args(v, n, field_num, &a);
  if (rc) return rc;
  if (!d_scratch || !d_total || (n && !d_out)) return fail(PZ_EINVAL, "null device pointer");
  a.out = d_out;
  a.offs = d_offsets;
  a.total = d_total;
  hipError_t e = launch_wire_validators(a, static_cast<uint64_t*>(d_scratch), static_cast<hipStream_t>(stream));
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_wire_val_kernel");
}

int pz_wire_validators(const pz_validator_cols* v, uint64_t n, uint32_t field_num, uint8_t* out, uint64_t cap,
                       uint64_t* offsets, uint64_t* len) {
  if (!len) return fail(PZ_EINVAL, "len is null");
  *len = 0;
  WireValArgs a;
  int rc = wire_val_args(v, n, field_num, &a);
  if (rc) return rc;
  if (n == 0) {
    if (offsets) offsets[0] = 0;
    return PZ_OK;
  }
  for (const uint64_t* o : {v->withdrawal_address_offs, v->randao_commitment_offs})
    if (o && (rc = check_csr(o, n, "bytes column"))) return rc;
  DeviceCtx* c;
  if ((rc = acquire(&c))) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = c->ensure_stream())) return rc;
  Stager st{c, c->stream};
  for (int k = 0; k < 5; ++k)
    if (a.col[k]) a.col[k] = st.up(a.col[k], n);
  std::vector<uint64_t> wo, ro;
  if (a.wa_offs) {
    wo = rebase(a.wa_offs, n);
    a.wa = st.up(v->withdrawal_address + v->withdrawal_address_offs[0], wo[n]);
    a.wa_offs = st.up(wo.data(), n + 1);
  }
  if (a.rc_offs) {
    ro = rebase(a.rc_offs, n);
    a.rc = st.up(v->randao_commitment + v->randao_commitment_offs[0], ro[n]);
    a.rc_offs = st.up(ro.data(), n + 1);
  }
  uint64_t nbytes = 0;
  if (a.wa_offs) nbytes += wo[n];
  if (a.rc_offs) nbytes += ro[n];
  uint64_t* scratch = st.zeros<uint64_t>(wire_tiles(n) + 1);
  a.total = st.zeros<uint64_t>(1);
  a.offs = offsets ? st.zeros<uint64_t>(n + 1) : nullptr;
  a.out = st.up<uint8_t>(nullptr, pz_wire_validators_bound(n, nbytes));
  if (st.rc) return st.rc;
  st.check(launch_wire_validators(a, scratch, st.s), "pz_wire_val_kernel");
  uint64_t total = 0;
  st.down(&total, a.total, 1);
  if (st.sync()) return st.rc;
  *len = total;
  if (total > cap) return fail(PZ_ERANGE, "output needs %llu bytes, capacity %llu", (unsigned long long)total,
                               (unsigned long long)cap);
  if (!out) return fail(PZ_EINVAL, "out is null");
  st.down(out, a.out, total);
  if (offsets) st.down(offsets, a.offs, n + 1);
  return st.sync();
}

}  // extern "C"
