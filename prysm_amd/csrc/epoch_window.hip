// The window pass: the one-pass epoch step on the committee-order layout in ONE launch
// (round 5; epoch.h "one-pass epoch" states why one pass is exact).  It replaces round 4's
// pre + fused launches, whose waves each took one committee piece through three dependent
// round trips (piece descriptor -> stream -> reward-bit lookups through L2) and ran the
// 1M x 16 cold step at 0.36 of 8 TB/s.
//
// Block (instance i, range r): the committees [cr0, cr1) of this rank, whose positions are
// contiguous (committee order).  The ranges partition the committees, so every committee's
// tallies are complete inside ONE block: they are summed in LDS and leave with plain stores,
// and the block applies the winner rule (core.go:549-555) itself -- no tally atomics to HBM,
// no winner pass.
//
//   prologue  the first pieces' loads go out first; then GetAttestersTotalDeposit
//             (validator.go:93-102) as a bit count over every bitfield of the instance (each
//             block counts them: nothing precedes the launch) with the last bitfield
//             (CalculateRewards reads it by validator index, incentives.go:22-27) copied into
//             LDS by DMA, and the bitfield-length panics (core.go:538-541)
//   loop      committee pieces (<= 256 positions of ONE committee, from its first position
//             rounded down to 4), each with its per-instance descriptor (committee, attestation
//             kind, the single attestation's bitfield position): lane l takes 4 contiguous
//             positions, every column load 16 B per lane plus 8 B of the committee's bitfield
//             holding the 4 vote bits, kWinDepth pieces ahead; the reward bit of position p is
//             bit co_index[p] of the LDS copy; the crosslink tallies (core.go:533-545) are four
//             32-bit DPP wave sums of the pre-reward u32 balance offsets (low 15 bits with the
//             count above them, high 17 bits), added into LDS
//   epilogue  every attestation of the range: vote / total stored, the winner rule as an
//             atomicMin on its shard; the block's next-cycle partial sum (core.go:459-464)
//             as one atomic
//
// Committees with several attestations (kind 2) take a slower in-loop path per attestation
// (its bitfield bytes from global memory); committees without one add nothing.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "epoch.h"
#include "votes_dev.h"

namespace pz {

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldnt16(const void* p) {
  const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ uint64_t pk64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// Sum of a u32 over the wave by DPP, wave-uniform (every lane active): quad swaps, half-row
// and row mirrors, row broadcasts 15 / 31 into lane 63.
__device__ __forceinline__ uint32_t wsum32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);   // quad_perm 1,0,3,2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false);   // quad_perm 2,3,0,1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xf, 0xf, false);  // row_half_mirror
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xf, 0xf, false);  // row_mirror
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast31
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// One piece's column words per lane: the balances of its 4 positions (u32 offsets: one 16-B
// load; u64: two), their {start, end} bounds (16-bit pairs: one load; 32-bit pairs: two; the
// 64-bit columns: four), their co_index entries, and 8 bytes of the committee's bitfield
// holding their 4 vote bits.
template <bool B32, int SEW>
struct WinCols {
  uint4 b[B32 ? 1 : 2];
  uint4 s[SEW == 16 ? 1 : SEW == 32 ? 2 : 4];
  uint4 ci;
  uint2 vb;
};

// A piece of one instance (WinArgs.pinfo), wave-uniform
struct Piece {
  uint32_t s0, cnt, cl, kind, kb, vbit, vlim;
};

// The instance's columns (wave-uniform bases: the loads take a 32-bit per-lane offset)
struct WinCol {
  const uint32_t* bal32;
  const uint64_t* bal;
  const uint32_t* se16;
  const uint2* se;
  const uint64_t* start;
  const uint64_t* end;
  const uint32_t* ci;
  const uint8_t* vbits;  // the instance's bitfields from its 16-B aligned start (vbit counts from here)
};

// the bit of the lane's first position in the piece's bitfield (kind 1; may precede the
// bitfield by up to 3 bits when the piece starts mid-quad: the buffer has 16 B before it)
__device__ __forceinline__ int64_t vbit_of(const Piece& d, uint32_t p) { return (int64_t)d.vbit + (int64_t)p - d.s0; }

// (NTB: the balances stream nontemporally too -- read once and written once per step, they
// leave the caches to the tables every block re-reads: co_index, the piece descriptors, the
// bitfields; round 6: 59 -> 53 us per cold 65,536 x 256 step, profiles/r06/epoch_cold_nt_r6c.txt)
template <bool B32, int SEW, bool NTB = true>
__device__ __forceinline__ void win_load(const WinCol& c, const Piece& d, uint32_t lane, WinCols<B32, SEW>& x) {
  const uint32_t pa = d.s0 & ~3u, p = pa + 4 * lane;
  const bool any = p + 3 >= d.s0 && p < d.s0 + d.cnt;
  const uint32_t pp = any ? p : pa;  // (a lane wholly outside the piece re-reads the first quad)
  if (B32) {
    x.b[0] = NTB ? ldnt16(c.bal32 + pp) : *reinterpret_cast<const uint4*>(c.bal32 + pp);
  } else {
    x.b[0] = NTB ? ldnt16(c.bal + pp) : *reinterpret_cast<const uint4*>(c.bal + pp);
    x.b[B32 ? 0 : 1] = NTB ? ldnt16(c.bal + pp + 2) : *reinterpret_cast<const uint4*>(c.bal + pp + 2);
  }
  // the bounds are read once per step: nontemporal
  if (SEW == 16) {
    x.s[0] = ldnt16(c.se16 + pp);
  } else if (SEW == 32) {
    x.s[0] = ldnt16(c.se + pp);
    x.s[SEW == 32 ? 1 : 0] = ldnt16(c.se + pp + 2);
  } else {
    x.s[0] = ldnt16(c.start + pp);
    x.s[SEW == 64 ? 1 : 0] = ldnt16(c.start + pp + 2);
    x.s[SEW == 64 ? 2 : 0] = ldnt16(c.end + pp);
    x.s[SEW == 64 ? 3 : 0] = ldnt16(c.end + pp + 2);
  }
  x.ci = *reinterpret_cast<const uint4*>(c.ci + pp);
  // the 4 vote bits sit in bytes j / 8 and j / 8 + 1 (j = the first position's bit): 8 bytes
  // from the dword below them (unused for kind != 1, and then from the region's start)
  const int64_t j = d.kind == 1 ? vbit_of(d, pp) : 0;
  const int64_t byte = j >> 3;  // (arithmetic: down to -1)
  __builtin_memcpy(&x.vb, __builtin_assume_aligned(c.vbits + (byte & ~3ll), 4), 8);
}

// the lane's 4 vote bits, position i -> bit i (CheckBit, utils/checkbit.go:4-12: bit j of a
// bitfield is bit 7 - j % 8 of byte j / 8)
__device__ __forceinline__ uint32_t vote4(const Piece& d, uint32_t p, uint2 raw) {
  const int64_t j = vbit_of(d, p);
  const uint32_t sh = (uint32_t)((j >> 3) & 3) * 8, jb = (uint32_t)(j & 7);
  const uint64_t w8 = pk64(raw.x, raw.y) >> sh;
  const uint32_t u16 = ((uint32_t)(w8 & 0xFF) << 8) | (uint32_t)((w8 >> 8) & 0xFF);  // bytes j/8, j/8+1, MSB first
  return __builtin_bitreverse32((u16 >> (12 - jb)) & 0xFu) >> 28;
}

// validator.go:45-53 on position i of the lane's quad (the saturated bounds classify exactly:
// the host takes the 16- / 32-bit columns only when every CurrentDynasty is below them)
template <bool B32, int SEW>
__device__ __forceinline__ bool win_active(const WinCols<B32, SEW>& x, int i, uint32_t d32, uint64_t d) {
  if (SEW == 16) {  // (then every CurrentDynasty < 0xFFFF: 32-bit compares are exact)
    const uint32_t s4[4] = {x.s[0].x, x.s[0].y, x.s[0].z, x.s[0].w};
    return (s4[i] & 0xFFFFu) <= d32 && d32 < (s4[i] >> 16);
  } else if (SEW == 32) {  // (every CurrentDynasty < 2^32 - 1)
    const uint4 q = x.s[i >> 1];
    const uint32_t lo = (i & 1) ? q.z : q.x, hi = (i & 1) ? q.w : q.y;
    return lo <= d32 && d32 < hi;
  } else {
    const uint4 qs = x.s[i >> 1], qe = x.s[SEW == 64 ? 2 + (i >> 1) : 0];
    const uint64_t s = (i & 1) ? pk64(qs.z, qs.w) : pk64(qs.x, qs.y);
    const uint64_t e = (i & 1) ? pk64(qe.z, qe.w) : pk64(qe.x, qe.y);
    return s <= d && d < e;
  }
}

}  // namespace

// LDS carve-up of one block (bytes; WinArgs.lds_* from the host's plan)
struct WinLds {
  uint64_t* tot;    // [maxc] committee totals
  uint64_t* vot;    // [maxk] vote per attestation (catt index - the range's first)
  uint8_t* lbf;     // [lds_lbf] the instance's last bitfield from (lb & ~15)
};

__device__ __forceinline__ WinLds win_lds(uint8_t* base, const WinArgs& w) {
  WinLds L;
  L.tot = reinterpret_cast<uint64_t*>(base);
  L.vot = L.tot + w.lds_maxc;
  L.lbf = reinterpret_cast<uint8_t*>(L.vot + w.lds_maxk);  // (16-B aligned: lds_maxc + lds_maxk is even)
  return L;
}

size_t window_lds_bytes(const WinArgs& w) { return 8ull * ((size_t)w.lds_maxc + w.lds_maxk) + w.lds_lbf + 16; }

// AB: measurement ablations, instantiated only in the A/B library (results wrong for AB != 0
// except 16, 48, 64): 1 no crosslink tallies, 2 no bit count / length checks in the prologue
// (applied taken as true), 4 no reward-bit lookups, 16 the R blocks of an instance each count
// 1/R of its bitfields and meet in WinArgs.pacc (exact; measured 2 us slower at 1M x 16 than
// every block counting everything, profiles/r05/epoch_abl_window_v4_r5h.txt), 48 = 16 with the
// meeting's wait bound at zero (the fallback count in every block that arrives before its
// partners; exact), 64 the first pieces' loads issued after the prologue (exact), 128 an
// instance's blocks grouped on one XCD (exact), 144 = 128 + 16, 4096 the four-sum tallies on
// narrow offsets (exact), 8192 no speculation: the whole count before the loop (exact), 32
// (alone) the speculating blocks' post-loop meeting skipped, the fallback count every time (exact);
// 16384 the product's L2 form (the reward bits looked up in the last bitfield in global memory,
// no LDS copy; exact), 1 << 23 the next round's loads issued at the waves' base priority (round
// 6's first form; exact).
template <bool B32, int SEW, bool LLB, int AB = 0, int D = kWinDepth, bool TR = false, bool NA = false, bool NP = true,
          int KD = 0>
__device__ __forceinline__ void window_body(const EpochArgs& a, const WinArgs& w) {
  extern __shared__ __align__(16) uint8_t lds_dyn[];
  constexpr int NT = kWinThreads, NW = NT / 64;
  constexpr bool NTB = !(AB & (1 << 20));  // the balances nontemporal (A/B bit 1 << 20: round 5's cached form)
  __shared__ uint64_t red[NW][2], red2[NW][2];  // (the prologue's and the loop's: no barrier between their uses)
  __shared__ uint64_t tstamp[4];  // (TR only)
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = rfl(tid >> 6);
  if (TR && tid == 0) tstamp[0] = __builtin_amdgcn_s_memrealtime();
  // block -> (instance, range); AB & 128: an instance's blocks on one XCD (block b runs on XCD
  // b % 8), so its bitfields are fetched into one L2 once
  uint32_t lb_id = blockIdx.x;
  if ((AB & 128) && (gridDim.x & 7) == 0) lb_id = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const uint64_t inst = lb_id / w.R;
  const uint32_t r = lb_id - (uint32_t)inst * w.R;
  // (NP: the range's descriptor from the kernel arguments when they hold it -- a scalar load of
  // the kernarg segment; the table in global memory only past kWinKargR ranges)
  typedef const __attribute__((address_space(4))) uint32_t kuint32;
  const kuint32* rdp = (kuint32*)(NP && w.R <= kWinKargR ? w.rdk : w.rdesc) + 4 * r;
  const uint4 rd = make_uint4(rdp[0], rdp[1], rdp[2], rdp[3]);
  const uint32_t cr0 = rd.x, cr1 = rd.y, pb = rd.z, np = rd.w;
  const uint2 rkk = w.rk[inst * w.R + r];
  const uint32_t k0 = rkk.x, nk = rkk.y;  // the range's attestations: catt[k0, k0 + nk)
  const uint64_t gb = inst * a.natt;
  // The wave's pieces go round by round, slot j of round t being piece t * D * NW + j * NW +
  // wave; past the range's end a slot takes a dummy (the last piece with no positions), so
  // every load below is issued unconditionally and the loop's waits count exactly the loads in
  // flight.  Lanes 2j, 2j + 1 load slot j's two descriptor words: one load a round.
  const uint32_t npm = np ? np - 1 : 0, nround = (np + D * NW - 1) / (D * NW);
  const uint32_t dslot = wave + (uint32_t)((lane >> 1) % D) * NW;
  const uint4* pinfo = w.pinfo + 2 * (inst * w.ptot + pb);
  auto desc = [&](uint32_t rnd) {  // this lane's word of its slot's descriptor for round rnd
    const uint32_t k = rnd * D * NW + dslot;
    return pinfo[2 * min(k, npm) + (lane & 1)];
  };
  auto piece = [&](const uint4& x, int j, uint32_t rnd) {  // slot j's piece of round rnd
    Piece d;
    const bool dummy = rnd * D * NW + (uint32_t)j * NW + wave >= np;  // (a dummy: no positions)
    d.s0 = __builtin_amdgcn_readlane(x.x, 2 * j);
    d.cnt = dummy ? 0u : (uint32_t)__builtin_amdgcn_readlane(x.y, 2 * j);
    d.cl = __builtin_amdgcn_readlane(x.z, 2 * j), d.kind = __builtin_amdgcn_readlane(x.w, 2 * j);
    d.kb = __builtin_amdgcn_readlane(x.x, 2 * j + 1), d.vbit = __builtin_amdgcn_readlane(x.y, 2 * j + 1);
    d.vlim = __builtin_amdgcn_readlane(x.z, 2 * j + 1);
    return d;
  };
  uint4 dv = desc(0);
  // NP: round 1's descriptors go out with round 0's (both depend on the kernel arguments alone)
  const uint4 dv1 = NP ? desc(1) : make_uint4(0, 0, 0, 0);
  // (NP: nothing is scheduled above this point from below it, so the bitfield offsets' scalar
  // loads -- and their wait -- come after the descriptors' loads have gone out)
  if (NP) __builtin_amdgcn_sched_barrier(0);
  const uint64_t pbeg = a.boffs[gb], pend = a.boffs[gb + a.natt], lb = a.boffs[gb + a.natt - 1];
  const uint64_t pbase = pbeg & ~15ull, lbase = lb & ~15ull;
  const uint64_t vrow = inst * w.vstride;
  const WinCol col{w.bal32 + vrow, a.balance + vrow, w.se16 + vrow, w.se + vrow, a.start + vrow, a.end + vrow,
                   a.co_index, a.bits + pbase};
  const WinLds L = win_lds(lds_dyn, w);
  const uint32_t ncr = cr1 - cr0;
  // GetAttestersTotalDeposit (every bitfield's bits) and the bitfield-length panics.  The
  // region's 16-B chunks [0, nch) from pbase; the last bitfield's, [clb, nch), go into LDS by
  // DMA (no registers, 1 KiB per wave instruction) for the reward bits.  With R > 1 the block
  // counts only its share of the chunks and attestations and the R blocks meet in pacc.
  uint64_t pop = 0, err = 0;
  const uint64_t nch = (pend - pbase + 15) / 16, clb = LLB ? (lbase - pbase) / 16 : nch;
  // Speculation (the product, R > 1): each of the instance's R blocks counts its 1/R share and
  // publishes it without waiting, runs the loop as if the reward applies (the common case), and
  // meets its partners after the loop, when they have long published; if the reward does not
  // apply after all, the block puts its own positions back (the rare path).  A/B bit 8192: the
  // whole count before the loop in every block (round 5's first form).
  const bool spec = !(AB & (8192 | 16 | 2)) && w.pacc != nullptr && w.R > 1;
  const bool coop = spec || ((AB & 16) && w.pacc != nullptr && w.R > 1);
  static_assert(!NP || !(AB & 16), "the A/B meeting before the loop keeps the round-5 prologue");
  // floor(n r / R) in 32-bit divisions (n < 2^28 bitfield chunks or attestations, R <= 511):
  // n = q R + m gives q r + floor(m r / R), m r < 2^18
  auto share = [&](uint64_t n, uint32_t rr) -> uint64_t {
    const uint32_t q = (uint32_t)n / w.R, m = (uint32_t)n - q * w.R;
    return (uint64_t)q * rr + (m * rr) / w.R;
  };
  const uint64_t s0 = coop ? share(nch, r) : 0, s1 = coop ? share(nch, r + 1) : nch;
  const uint64_t g0s = coop ? share(a.natt, r) : 0, g1s = coop ? share(a.natt, r + 1) : a.natt;
  // bits of chunk c (its bytes inside [pbeg, pend) only)
  auto chunk_pop = [&](uint64_t c, uint4 x) -> uint32_t {
    const uint64_t ad = pbase + 16 * c;
    const uint32_t wd[4] = {x.x, x.y, x.z, x.w};
    if (ad >= pbeg && ad + 16 <= pend) return __popc(wd[0]) + __popc(wd[1]) + __popc(wd[2]) + __popc(wd[3]);
    uint32_t n = 0;
#pragma unroll
    for (int dd = 0; dd < 4; ++dd) {
      uint32_t m = 0;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const uint64_t at = ad + 4 * dd + bb;
        if (at >= pbeg && at < pend) m |= 0xFFu << (8 * bb);
      }
      n += __popc(wd[dd] & m);
    }
    return n;
  };
  // NP: the count's loads as {issue, take} halves, so they go out before the first descriptors
  // are waited for and are taken after the first pieces' loads are in flight.  Iteration `it`
  // covers chunks [c_lo + it CU NT, +CU NT) and attestations [g_lo + it CG NT, +CG NT) (every
  // load issued, past the end clamped, as count_range)
  constexpr int CU = 2, CG = 1;
  struct CountLd {
    uint4 x[CU];
    uint32_t csz[CG];
    uint64_t bo0[CG], bo1[CG];
  };
  auto cnt_issue = [&](uint64_t c_lo, uint64_t nc, uint64_t g_lo, uint64_t ng, uint64_t it, CountLd& cl) {
    const uint64_t c0 = it * CU * NT + tid, gi0 = it * CG * NT + tid;
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      const uint64_t c = c_lo + std::min<uint64_t>(c0 + (uint64_t)u * NT, nc ? nc - 1 : 0);
      cl.x[u] = *reinterpret_cast<const uint4*>(a.bits + pbase + 16 * c);
    }
#pragma unroll
    for (int u = 0; u < CG; ++u) {
      const uint64_t g = g_lo + std::min<uint64_t>(gi0 + (uint64_t)u * NT, ng ? ng - 1 : 0);
      cl.csz[u] = w.att_csize[gb + g];
      cl.bo0[u] = a.boffs[gb + g];
      cl.bo1[u] = a.boffs[gb + g + 1];
    }
  };
  auto cnt_take = [&](uint64_t c_lo, uint64_t nc, uint64_t ng, uint64_t it, const CountLd& cl) {
    const uint64_t c0 = it * CU * NT + tid, gi0 = it * CG * NT + tid;
#pragma unroll
    for (int u = 0; u < CU; ++u)
      if (c0 + (uint64_t)u * NT < nc) pop += chunk_pop(c_lo + c0 + (uint64_t)u * NT, cl.x[u]);
    // the crosslink bitfield-length panic (core.go:538-541): a committee longer than its bitfield
#pragma unroll
    for (int u = 0; u < CG; ++u)
      if (gi0 + (uint64_t)u * NT < ng && (uint64_t)cl.csz[u] > 8 * (cl.bo1[u] - cl.bo0[u])) err = 1;
  };
  auto cnt_iters = [&](uint64_t nc, uint64_t ng) {
    return std::max<uint64_t>((nc + CU * NT - 1) / (CU * NT), (ng + CG * NT - 1) / (CG * NT));
  };
  auto count_np = [&](uint64_t c_lo, uint64_t c_hi, uint64_t g_lo, uint64_t g_hi) {  // issue + take
    const uint64_t nc = c_hi > c_lo ? c_hi - c_lo : 0, ng = g_hi - g_lo;
    for (uint64_t it = 0, nit = cnt_iters(nc, ng); it < nit; ++it) {
      CountLd cl;
      cnt_issue(c_lo, nc, g_lo, ng, it, cl);
      cnt_take(c_lo, nc, ng, it, cl);
    }
  };
  // chunks [c_lo, c_hi) below the last bitfield and attestations [g_lo, g_hi) from global memory
  auto count_range = [&](uint64_t c_lo, uint64_t c_hi, uint64_t g_lo, uint64_t g_hi) {
    constexpr int U = 4, UC = 4;  // (U = 8 spills at 1024 threads)
    const uint64_t nc = c_hi > c_lo ? c_hi - c_lo : 0, ng = g_hi - g_lo;
    const uint64_t nit = std::max<uint64_t>((nc + U * NT - 1) / (U * NT), (ng + UC * NT - 1) / (UC * NT));
    for (uint64_t it = 0; it < nit; ++it) {  // (uniform: every load issued, past the end clamped)
      const uint64_t c0 = it * U * NT + tid, gi0 = it * UC * NT + tid;
      uint4 x[U];
      uint32_t csz[UC];
      uint64_t bo0[UC], bo1[UC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t c = c_lo + std::min<uint64_t>(c0 + (uint64_t)u * NT, nc ? nc - 1 : 0);
        x[u] = *reinterpret_cast<const uint4*>(a.bits + pbase + 16 * c);
      }
#pragma unroll
      for (int u = 0; u < UC; ++u) {
        const uint64_t g = g_lo + std::min<uint64_t>(gi0 + (uint64_t)u * NT, ng ? ng - 1 : 0);
        csz[u] = w.att_csize[gb + g];
        bo0[u] = a.boffs[gb + g];
        bo1[u] = a.boffs[gb + g + 1];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (c0 + (uint64_t)u * NT < nc) pop += chunk_pop(c_lo + c0 + (uint64_t)u * NT, x[u]);
      // the crosslink bitfield-length panic (core.go:538-541): a committee longer than its bitfield
#pragma unroll
      for (int u = 0; u < UC; ++u)
        if (gi0 + (uint64_t)u * NT < ng && (uint64_t)csz[u] > 8 * (bo1[u] - bo0[u])) err = 1;
    }
  };
  auto count_lds = [&](uint64_t c_lo, uint64_t c_hi) {  // chunks of the last bitfield, from its LDS copy
    for (uint64_t c = c_lo + tid; c < c_hi; c += NT)
      pop += chunk_pop(c, *reinterpret_cast<const uint4*>(L.lbf + 16 * (c - clb)));
  };
  auto last_bitfield_dma = [&]() {
    typedef __attribute__((address_space(3))) void lds_void_t;
    typedef const __attribute__((address_space(1))) void gbl_void_t;
    const uint64_t nl = nch - clb;
    // (NP: a fixed unrolled count -- the copy fits the CU's LDS -- so the loads issued after it
    // keep exact waits; a loop of unknown trip count would make every later wait a full drain)
    constexpr int kDmaMax = (160 * 1024 + 16 * NT - 1) / (16 * NT);
    if (NP) {
#pragma unroll
      for (int u = 0; u < kDmaMax; ++u) {
        const uint64_t c0 = (uint64_t)wave * 64 + (uint64_t)u * NT;  // (wave-uniform)
        if (c0 < nl && c0 + lane < nl)
          __builtin_amdgcn_global_load_lds((gbl_void_t*)(a.bits + lbase + 16 * (c0 + lane)), (lds_void_t*)(L.lbf + 16 * c0),
                                           16, 0, 0);
      }
      return;
    }
    for (uint64_t c0 = (uint64_t)wave * 64; c0 < nl; c0 += NT) {  // (wave-uniform c0)
      const uint64_t c = std::min<uint64_t>(c0 + lane, nl - 1);
      if (c0 + lane < nl)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(a.bits + lbase + 16 * c), (lds_void_t*)(L.lbf + 16 * c0), 16, 0,
                                         0);
    }
  };
  // KD > 0 (the plan's WinArgs.dma_k): exactly KD wave instructions, no branch, no predicate --
  // past the copy's end a lane re-reads its last chunk into the padding (lds_lbf holds KD x NT
  // chunks) -- so the loads issued after it keep exact waits and it can go out first
  auto last_bitfield_dma_k = [&]() {
    typedef __attribute__((address_space(3))) void lds_void_t;
    typedef const __attribute__((address_space(1))) void gbl_void_t;
    const uint32_t nlm = (uint32_t)(nch - clb) - 1;  // (>= 0: the plan takes KD only for non-empty copies)
#pragma unroll
    for (int u = 0; u < (KD > 0 ? KD : 1); ++u) {
      const uint32_t c0 = wave * 64 + (uint32_t)u * NT;
      const uint32_t c = min(c0 + (uint32_t)lane, nlm);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(a.bits + lbase + 16ull * c), (lds_void_t*)(L.lbf + 16 * c0), 16, 0, 0);
    }
  };
  // NP, step 1: the count's first loads, before any wait (the DMA follows the count's take:
  // issued earlier, its branches would turn every later wait into a full drain)
  CountLd cl0;
  const uint64_t ncn = s1 - s0, ngn = g1s - g0s;
  if (NP && KD > 0 && LLB && !(AB & 2)) last_bitfield_dma_k();  // (straight-line: the waits stay exact)
  if (NP && !(AB & 2)) cnt_issue(s0, ncn, g0s, ngn, 0, cl0);
  if (NP && (AB & (1 << 21)) && !(AB & 2) && LLB && KD == 0) last_bitfield_dma();  // (A/B: the DMA loop before the first wait)
  Piece dq[D];
#pragma unroll
  for (int j = 0; j < D; ++j) dq[j] = piece(dv, j, 0);
  WinCols<B32, SEW> q[D];
  if (!(AB & 64)) {
#pragma unroll
    for (int j = 0; j < D; ++j) win_load<B32, SEW, NTB>(col, dq[j], lane, q[j]);
  }
  dv = NP ? dv1 : desc(1);
  if (NP) {
    // step 2: the count taken (its loads went out with the descriptors, a round trip before the
    // pieces'), then the last bitfield's DMA, the tallies zeroed, and one barrier for the wave
    // sums, the DMA and the zeroed tallies; every thread then has the block's count (R = 1: the
    // instance's -- no meeting, no speculation; R > 1: its share, published by one atomic)
    if (!(AB & 2)) {
      cnt_take(s0, ncn, ngn, 0, cl0);
      for (uint64_t it = 1, nit = cnt_iters(ncn, ngn); it < nit; ++it) {
        CountLd cl;
        cnt_issue(s0, ncn, g0s, ngn, it, cl);
        cnt_take(s0, ncn, ngn, it, cl);
      }
      if (LLB && KD == 0 && !(AB & (1 << 21))) last_bitfield_dma();
    } else {
      pop = tid == 0 ? a.total_deposit[inst] : 0;  // (ablation: the threshold holds)
    }
    for (uint32_t i = tid; i < ncr; i += NT) L.tot[i] = 0;
    for (uint32_t i = tid; i < nk; i += NT) L.vot[i] = 0;
    pop = wsum64_dpp(pop);
    err = __builtin_amdgcn_ballot_w64(err != 0) ? 1 : 0;
    if (lane == 0) red[wave][0] = pop, red[wave][1] = err;
    __syncthreads();
    pop = 0, err = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) pop += red[k][0], err += red[k][1];
    if (spec && tid == 0) {
      const uint64_t add = (1ull << 48) | (err ? 1ull << 39 : 0) | pop;
      atomicAdd((unsigned long long*)&w.pacc[inst], (unsigned long long)add);
    }
  } else {
    for (uint32_t i = tid; i < ncr; i += NT) L.tot[i] = 0;
    for (uint32_t i = tid; i < nk; i += NT) L.vot[i] = 0;
    if (!(AB & 2)) {
      if (LLB) last_bitfield_dma();
      count_range(s0, std::min(s1, clb), g0s, g1s);
    } else {
      pop = tid == 0 ? a.total_deposit[inst] : 0;  // (ablation: the threshold holds)
    }
    __syncthreads();  // the last bitfield is in LDS, the tallies zeroed
    if (!(AB & 2)) count_lds(std::max(s0, clb), s1);
    pop = wsum64_dpp(pop);
    err = wsum64_dpp(err);
    if (lane == 0) red[wave][0] = pop, red[wave][1] = err;
    __syncthreads();
    pop = 0, err = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) pop += red[k][0], err += red[k][1];
    if (spec) {  // publish this block's share; the meeting is after the loop
      if (tid == 0) {
        const uint64_t add = (1ull << 48) | (err ? 1ull << 39 : 0) | pop;
        atomicAdd((unsigned long long*)&w.pacc[inst], (unsigned long long)add);
      }
    } else if (coop && !(AB & 2)) {
      // the instance's R blocks meet: one atomic adds this block's share, then thread 0 polls the
      // word (at the coherence point) until all R have arrived, or the bound passes and the block
      // counts everything itself (so no block ever depends on another being resident)
      __shared__ uint64_t s_meet;
      if (tid == 0) {
        const uint64_t add = (1ull << 48) | (err ? 1ull << 39 : 0) | pop;
        uint64_t v = atomicAdd((unsigned long long*)&w.pacc[inst], (unsigned long long)add) + add;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while ((v >> 48) < w.R && __builtin_amdgcn_s_memrealtime() - t0 < ((AB & 32) ? 0 : kCoopSpinTicks)) {
          __builtin_amdgcn_s_sleep(2);
          v = __hip_atomic_fetch_add(&w.pacc[inst], (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_meet = v;
      }
      __syncthreads();
      const uint64_t v = s_meet;
      if ((v >> 48) >= w.R) {
        pop = v & ((1ull << 39) - 1);
        err = (v >> 39) & 511;
      } else {  // (a partner not resident in time: the whole count here)
        pop = 0, err = 0;
        count_range(0, clb, 0, a.natt);
        count_lds(clb, nch);
        pop = wsum64_dpp(pop);
        err = wsum64_dpp(err);
        __syncthreads();
        if (lane == 0) red[wave][0] = pop, red[wave][1] = err;
        __syncthreads();
        pop = 0, err = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) pop += red[k][0], err += red[k][1];
      }
    }
  }
  if (AB & 64) {  // (A/B: the first pieces' loads only now, behind the prologue's)
#pragma unroll
    for (int j = 0; j < D; ++j) win_load<B32, SEW, NTB>(col, dq[j], lane, q[j]);
  }
  if (TR && tid == 0) tstamp[1] = __builtin_amdgcn_s_memrealtime();
  // the next step's accumulators start from zero, its winners empty (its own buffers: issued
  // here, the stores drain under the loop instead of at the kernel's end)
  if (r == 0) {
    if (a.scal_next && tid < kScal) a.scal_next[inst * kScal + tid] = 0;
    if (w.pacc_next && tid == 0) w.pacc_next[inst] = 0;
    for (uint32_t s = tid; s < a.nrec; s += NT) w.winner_next[inst * a.nrec + s] = 0xFFFFFFFFu;
    if (w.vote_next)
      for (uint32_t g = tid; g < a.natt; g += NT) w.vote_next[gb + g] = 0, w.total_next[gb + g] = 0;
  }
  const uint64_t lastL = pend - lb;
  const bool rwd_err = (a.nval_global - 1) >= 8 * lastL;  // CheckBit(last, N-1) panics (incentives.go:23)
  bool thr = (pop * PZ_DEFAULT_BALANCE * 3ull) >= (a.total_deposit[inst] * 2ull);  // incentives.go:18-20
  uint64_t ferr = err ? (uint64_t)kErrBitfield : 0;
  bool skip = ferr != 0 || (thr && rwd_err);  // Go panics: balances stay untouched
  // (speculating: pop and err are this block's share; rwd_err rules the reward out whatever
  // the count says, so then there is nothing to speculate on)
  const bool spec_on = spec && !rwd_err;
  bool applied = spec_on || (!spec && thr && !skip);
  const uint64_t d = a.dynasty[inst];
  const uint32_t d32 = (uint32_t)std::min<uint64_t>(d, 0xFFFFFFFFull);
  const uint64_t bbase = B32 ? w.bal32_base[inst] : 0;
  const uint8_t* lbf8 = LLB ? L.lbf + (lb - lbase) : a.bits + lb;
  uint64_t* Bal = a.balance + vrow;
  uint32_t* Bal32 = w.bal32 + vrow;
  // per lane: the next-cycle sum (B32: of the new offsets, with the active count; base added
  // at the end), the positions whose bounds do not classify them active
  uint64_t sum = 0;
  uint32_t nact = 0, nm = 0;
  int32_t dsum = 0;  // the rewards' part of sum (taken back if the speculated reward does not apply)
  const uint32_t rwd = applied ? 1u : 0u;  // (not applied: the balances stay, offsets +- 0)
  for (uint32_t t = 0; t < nround; ++t) {
    const uint4 dnx = dv;     // round t + 1's descriptors (loaded a round ago)
    dv = desc(t + 2);         // round t + 2's
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const WinCols<B32, SEW>& x = q[j];
      const Piece& pc = dq[j];
      const uint32_t s0p = pc.s0, cnt = pc.cnt, cl = pc.cl, kind = pc.kind, kb = pc.kb;
      const uint32_t pa = s0p & ~3u, p = pa + 4 * (uint32_t)lane;
      bool v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = p + i - s0p < cnt;  // (u32: p + i < s0 wraps high)
      uint32_t o4[4] = {0, 0, 0, 0};
      uint64_t b[4] = {0, 0, 0, 0};
      if (B32) {
        o4[0] = x.b[0].x, o4[1] = x.b[0].y, o4[2] = x.b[0].z, o4[3] = x.b[0].w;
      } else {
        b[0] = pk64(x.b[0].x, x.b[0].y), b[1] = pk64(x.b[0].z, x.b[0].w);
        b[2] = pk64(x.b[B32 ? 0 : 1].x, x.b[B32 ? 0 : 1].y), b[3] = pk64(x.b[B32 ? 0 : 1].z, x.b[B32 ? 0 : 1].w);
      }
      // the reward bits first: their LDS lookups overlap the tallies
      uint32_t rb[4] = {0, 0, 0, 0};
      if (applied && !(AB & 4)) {
        const uint32_t c4[4] = {x.ci.x, x.ci.y, x.ci.z, x.ci.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t ix = v[i] ? c4[i] : 0u;  // (a position outside the piece looks bit 0 up)
          rb[i] = lbf8[ix >> 3] >> (7 - (ix & 7));
        }
      }
      // crosslink tallies of the piece's committee on the pre-reward balances (core.go:533-545)
      if (kind && !(AB & 1)) {
        uint32_t vw = 0;  // vote bits present only below vlim (from the piece's first position)
        if (kind == 1) {
          vw = vote4(pc, p, x.vb);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (p + i - s0p >= pc.vlim) vw &= ~(1u << i);
        }
        uint64_t T, V;
        if (B32 && NA && !(AB & 4096)) {
          // every offset within [floor, floor + 2^23): (offset - floor) sums to < 2^31 over the
          // <= 256 positions; the voters' count from four ballots (the positions' count is cnt)
          uint32_t ts = 0, vs = 0, nv = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t x = o4[i] - kTallyFloor;
            const bool vt = v[i] && ((vw >> i) & 1);
            ts += v[i] ? x : 0;
            vs += vt ? x : 0;
            nv += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(vt));
          }
          ts = wsum32(ts), vs = wsum32(vs);
          const uint64_t fb = bbase + kTallyFloor;
          T = (uint64_t)cnt * fb + ts;
          V = (uint64_t)nv * fb + vs;
        } else if (B32) {
          // offsets split 17 | 15 bits: low parts with the count in bits 23+ (<= 256 x 2^15 < 2^23,
          // <= 256 positions), high parts (<= 256 x 2^17 < 2^25): four 32-bit sums, exact
          uint32_t at = 0, ht = 0, av = 0, hv = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t lo = (o4[i] & 0x7FFFu) | (1u << 23), hi = o4[i] >> 15;
            const bool vt = v[i] && ((vw >> i) & 1);
            at += v[i] ? lo : 0;
            ht += v[i] ? hi : 0;
            av += vt ? lo : 0;
            hv += vt ? hi : 0;
          }
          at = wsum32(at), ht = wsum32(ht), av = wsum32(av), hv = wsum32(hv);
          T = (uint64_t)(at >> 23) * bbase + (at & 0x7FFFFFu) + ((uint64_t)ht << 15);
          V = (uint64_t)(av >> 23) * bbase + (av & 0x7FFFFFu) + ((uint64_t)hv << 15);
        } else {
          uint64_t tt = 0, vv = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            tt += v[i] ? b[i] : 0;
            vv += (v[i] && ((vw >> i) & 1)) ? b[i] : 0;
          }
          T = wsum64_dpp(tt);
          V = wsum64_dpp(vv);
        }
        if (lane == 0) {
          if (T) atomicAdd((unsigned long long*)&L.tot[cl], (unsigned long long)T);
          if (kind == 1 && V) atomicAdd((unsigned long long*)&L.vot[kb - k0], (unsigned long long)V);
        }
        if (kind == 2 && !(AB & 65536)) {  // several attestations: each one's bits from its bitfield in global memory
          const uint32_t cs = pc.vbit;  // (kind 2: the committee's first position)
          const uint32_t ke = pc.vlim;  // (kind 2: the committee's attestations end at catt index ke)
          if (AB & 131072) {  // (A/B: one attestation at a time, three dependent round trips each)
            for (uint32_t kq = kb; kq < ke; ++kq) {
              const uint64_t ga = w.catt[gb + kq];
              const uint64_t bo = a.boffs[gb + ga], nb = 8 * (a.boffs[gb + ga + 1] - bo);
              uint64_t sv = 0;
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const uint64_t xb = (uint64_t)(p + i) - cs;  // the position's bit in the bitfield
                const bool in = v[i] && xb < nb;
                const uint32_t by = in ? a.bits[bo + (xb >> 3)] : 0u;
                sv += (in && ((by >> (7 - (uint32_t)(xb & 7))) & 1)) ? (B32 ? bbase + o4[i] : b[i]) : 0;
              }
              sv = wsum64_dpp(sv);
              if (lane == 0 && sv) atomicAdd((unsigned long long*)&L.vot[kq - k0], (unsigned long long)sv);
            }
          } else {
            // two attestations per trip: both bitfields' {first byte, bits} from the plan's catt-ordered
            // table (one round of loads, no catt -> boffs chain), both bitfields' bytes in the next;
            // every lane loads (a position outside a bitfield reads its first byte, a bitfield of no
            // bytes the other one's) and the bytes are pinned, so no load sits in a branch
            const uint2* ckb = w.ckb + gb;
            for (uint32_t kq = kb; kq < ke; kq += 2) {
              const bool two = kq + 1 < ke;
              uint2 e0 = ckb[kq], e1 = ckb[two ? kq + 1 : kq];
              asm volatile("" : "+v"(e0.x), "+v"(e0.y), "+v"(e1.x), "+v"(e1.y));  // (both words before the branch)
              const uint32_t nb0 = e0.y, nb1 = two ? e1.y : 0u;
              if (!(nb0 | nb1)) continue;
              const uint8_t* bq0 = col.vbits + (nb0 ? e0.x : e1.x);
              const uint8_t* bq1 = col.vbits + (nb1 ? e1.x : e0.x);
              uint32_t by0[4], by1[4];
              bool in0[4], in1[4];
              uint32_t xb[4];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                xb[i] = p + i - cs;  // the position's bit in the bitfields (u32: below cs wraps high)
                in0[i] = v[i] && xb[i] < nb0;
                in1[i] = v[i] && xb[i] < nb1;
                by0[i] = bq0[(in0[i] ? xb[i] : 0u) >> 3];
                by1[i] = bq1[(in1[i] ? xb[i] : 0u) >> 3];
              }
#pragma unroll
              for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(by0[i]), "+v"(by1[i]));
              uint64_t sv0 = 0, sv1 = 0;
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const uint32_t sh = 7 - (xb[i] & 7);
                const uint64_t bv = B32 ? bbase + o4[i] : b[i];
                sv0 += (in0[i] && ((by0[i] >> sh) & 1)) ? bv : 0;
                sv1 += (in1[i] && ((by1[i] >> sh) & 1)) ? bv : 0;
              }
              sv0 = wsum64_dpp(sv0);
              sv1 = wsum64_dpp(sv1);
              if (lane == 0) {
                if (sv0) atomicAdd((unsigned long long*)&L.vot[kq - k0], (unsigned long long)sv0);
                if (sv1) atomicAdd((unsigned long long*)&L.vot[kq + 1 - k0], (unsigned long long)sv1);
              }
            }
          }
        }
      }
      // classify, reward (incentives.go:22-27), store, next-cycle sum (core.go:459-464)
      bool act[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        act[i] = win_active<B32, SEW>(x, i, d32, d);
        nm += (v[i] && !act[i]) ? 1 : 0;
      }
      const bool all = v[0] && v[1] && v[2] && v[3];
      if (B32) {
        // the offsets: (base + o +- 1) - base = o +- 1, inside u32 (the state's re-base bound)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t dl = (rb[i] & 1) ? rwd : 0u - rwd;
          o4[i] += dl;
          const bool ai = v[i] && act[i];
          sum += ai ? o4[i] : 0u;
          nact += ai ? 1u : 0u;
          dsum += ai ? (int32_t)dl : 0;
        }
        if (applied) {
          if (all) {
            if (NTB) {
              v4u o;
              o.x = o4[0], o.y = o4[1], o.z = o4[2], o.w = o4[3];
              __builtin_nontemporal_store(o, reinterpret_cast<v4u*>(Bal32 + p));
            } else {
              *reinterpret_cast<uint4*>(Bal32 + p) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
            }
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (v[i]) {
                if (NTB) __builtin_nontemporal_store(o4[i], Bal32 + p + i);
                else Bal32[p + i] = o4[i];
              }
          }
        }
      } else {
        if (applied) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            b[i] = (rb[i] & 1) ? b[i] + PZ_ATTESTER_REWARD : b[i] - PZ_ATTESTER_REWARD;
            dsum += (v[i] && act[i]) ? ((rb[i] & 1) ? (int32_t)PZ_ATTESTER_REWARD : -(int32_t)PZ_ATTESTER_REWARD) : 0;
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * h;
            if (v[i] && v[i + 1]) {
              v4u o;
              o.x = (uint32_t)b[i], o.y = (uint32_t)(b[i] >> 32), o.z = (uint32_t)b[i + 1], o.w = (uint32_t)(b[i + 1] >> 32);
              if (NTB) __builtin_nontemporal_store(o, reinterpret_cast<v4u*>(Bal + p + i));
              else *reinterpret_cast<v4u*>(Bal + p + i) = o;
            } else if (v[i]) {
              if (NTB) __builtin_nontemporal_store(b[i], Bal + p + i);
              else Bal[p + i] = b[i];
            } else if (v[i + 1]) {
              if (NTB) __builtin_nontemporal_store(b[i + 1], Bal + p + i + 1);
              else Bal[p + i + 1] = b[i + 1];
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) sum += (v[i] && act[i]) ? b[i] : 0;
      }
      // slot j's piece of the next round (past the last round: a dummy, loaded and unused)
      // (at raised priority: the SIMD's arbiter issues the wave's loads ahead of the other
      // waves' ALU work, so they go out sooner; 54.5 -> 54.0 / 58.2 -> 57.7 us cold,
      // profiles/r06/epoch_cold_prio_r6k.txt)
      // (measured and dropped: the raised priority from the descriptor's readlanes on, and
      // level 3, both level or slower, profiles/r06/prio_variants_dropped_r6m.txt)
      dq[j] = piece(dnx, j, t + 1);
      if (!(AB & (1 << 23))) __builtin_amdgcn_s_setprio(2);
      win_load<B32, SEW, NTB>(col, dq[j], lane, q[j]);
      if (!(AB & (1 << 23))) __builtin_amdgcn_s_setprio(0);
    }
  }
  // the epilogue's first kEpiPf attestations per thread: their words now, ahead of the meeting
  // (clamped indices: every load unconditional, none in a branch)
  constexpr int kEpiPf = 3;
  uint4 ep[kEpiPf];
  const uint4* cq = w.cq + gb + k0;
  const uint32_t nkm = nk ? nk - 1 : 0;
#pragma unroll
  for (int u = 0; u < kEpiPf; ++u) ep[u] = nk ? cq[min((uint32_t)tid + u * NT, nkm)] : make_uint4(0, 0, 0, 0);
  if (spec) {
    // the meeting: every partner published its share in its prologue; the bound and the
    // fallback (the whole count here) keep a block from ever depending on another's residency
    __shared__ uint64_t s_meet2;
    if (tid == 0) {
      uint64_t v = __hip_atomic_fetch_add(&w.pacc[inst], (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (AB & 32) v = 0;  // (A/B, tests: the fallback count every time)
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while ((v >> 48) < w.R && !(AB & 32) && __builtin_amdgcn_s_memrealtime() - t0 < kCoopSpinTicks) {
        __builtin_amdgcn_s_sleep(2);
        v = __hip_atomic_fetch_add(&w.pacc[inst], (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      s_meet2 = v;
    }
    __syncthreads();
    const uint64_t v = s_meet2;
    if ((v >> 48) >= w.R) {
      pop = v & ((1ull << 39) - 1);
      err = (v >> 39) & 511;
    } else {
      pop = 0, err = 0;
      if (NP) {
        count_np(0, nch, 0, a.natt);
      } else {
        count_range(0, clb, 0, a.natt);
        count_lds(clb, nch);
      }
      pop = wsum64_dpp(pop);
      err = wsum64_dpp(err);
      if (lane == 0) red[wave][0] = pop, red[wave][1] = err;
      __syncthreads();
      pop = 0, err = 0;
#pragma unroll
      for (int k = 0; k < NW; ++k) pop += red[k][0], err += red[k][1];
    }
    thr = (pop * PZ_DEFAULT_BALANCE * 3ull) >= (a.total_deposit[inst] * 2ull);
    ferr = err ? (uint64_t)kErrBitfield : 0;
    skip = ferr != 0 || (thr && rwd_err);
    const bool final_applied = thr && !skip;
    if (spec_on && !final_applied) {
      // the rare path: this block's positions back to their pre-reward values (each lane the
      // positions it wrote: piece k of the range went to wave k mod NW)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (uint32_t k = wave; k < np; k += NW) {
        const uint4 d0 = pinfo[2 * k];
        const uint32_t pa = d0.x & ~3u, pp = pa + 4 * (uint32_t)lane;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (pp + i - d0.x >= d0.y) continue;  // (u32: outside the piece)
          const uint32_t ix = a.co_index[pp + i];
          const bool up = (lbf8[ix >> 3] >> (7 - (ix & 7))) & 1;
          // (the block's own stores read back at L2: agent-scope loads, past any L1 copy)
          if (B32) {
            const uint32_t o = __hip_atomic_load(&Bal32[pp + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            Bal32[pp + i] = o - (up ? 1u : 0u - 1u);
          } else {
            const uint64_t o = __hip_atomic_load(&Bal[pp + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            Bal[pp + i] = up ? o - PZ_ATTESTER_REWARD : o + PZ_ATTESTER_REWARD;
          }
        }
      }
      sum -= (uint64_t)(int64_t)dsum;
    }
    applied = final_applied;
  }
  if (B32) sum += (uint64_t)nact * bbase;  // (the lane's sum of base + offset over its active positions)
  sum = wsum64_dpp(sum);
  const uint64_t nmw = wsum64_dpp(nm);
  if (lane == 0) red2[wave][0] = sum, red2[wave][1] = nmw;
  __syncthreads();  // (also: every wave's LDS tallies are in)
  if (TR && tid == 0) tstamp[2] = __builtin_amdgcn_s_memrealtime();
  uint64_t* sc = a.scal + inst * kScal;
  if (tid == 0) {
    uint64_t s = 0, n = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) s += red2[k][0], n += red2[k][1];
    if (s && !skip) atomicAdd((unsigned long long*)&sc[kNextBal], (unsigned long long)s);
    if (n) {  // the layout's rank == index premise is broken (the state never allows it)
      atomicAdd((unsigned long long*)&sc[kNoMatch], (unsigned long long)n);
      atomicOr((unsigned long long*)&sc[kErrXl], (unsigned long long)kErrLayout);
    }
    if (r == 0 && w.rank0) {  // the per-instance scalars (the all-reduce must not multiply them)
      sc[kPop] = pop;
      sc[kApplied] = applied ? 1 : 0;
      sc[kNact] = a.nval_global;
      sc[kMaxIdx1] = a.nval_global;
      sc[kErrRwd] = rwd_err ? 1 : 0;
      if (ferr) atomicAdd((unsigned long long*)&sc[kErrXl], (unsigned long long)ferr);
    }
  }
  // the range's attestations: tallies out, the winner rule (core.go:549-555: the first
  // attestation, in order, whose 3 * vote >= 2 * total and whose dynasty beats its shard's record)
  // (the dynasty compare on 32-bit saturated words: exact while the dynasty is below 2^32 - 1,
  // else the plan adds the record dynasties' high words)
  const uint32_t* cqh = w.cqh ? w.cqh + gb + k0 : nullptr;
  auto epi = [&](uint32_t kq, const uint4 e) {  // {attestation, cl, shard, record dynasty}
    const uint32_t ga = e.x;
    const uint64_t V = L.vot[kq], T = L.tot[e.y];
    a.vote[gb + ga] = V;
    a.total[gb + ga] = T;
    const bool beats = cqh ? d > pk64(e.w, cqh[kq]) : d32 > e.w;
    if (3ull * V >= 2ull * T && beats) atomicMin(&a.winner[inst * a.nrec + e.z], ga);
  };
#pragma unroll
  for (int u = 0; u < kEpiPf; ++u)
    if ((uint32_t)tid + u * NT < nk) epi(tid + u * NT, ep[u]);
  for (uint32_t kq = tid + kEpiPf * NT; kq < nk; kq += NT) epi(kq, cq[kq]);
  if (TR) {
    __syncthreads();
    if (tid == 0) {
      const uint64_t t3 = __builtin_amdgcn_s_memrealtime();
      w.trace[4ull * blockIdx.x] = tstamp[0], w.trace[4ull * blockIdx.x + 1] = tstamp[1];
      w.trace[4ull * blockIdx.x + 2] = tstamp[2], w.trace[4ull * blockIdx.x + 3] = t3;
    }
  }
}

#define PZ_WINDOW_KERNEL(NAME, B32, SEW, LLB, NA)                                                        \
  extern "C" __global__ void __launch_bounds__(kWinThreads) NAME(EpochArgs a, WinArgs w) {             \
    window_body<B32, SEW, LLB, 0, (B32 && SEW == 16) ? kWinDepth16 : kWinDepth, false, NA>(a, w);      \
  }
// balances as u32 offsets (the narrow tallies or not) / u64; {start, end} at 16 / 32 / 64 bits;
// the last bitfield in LDS or not
PZ_WINDOW_KERNEL(pz_epoch_window_b32n_s16_kernel, true, 16, true, true)
// (one piece in flight per wave: the product form when an instance has several ranges, R > 1)
extern "C" __global__ void __launch_bounds__(kWinThreads) pz_epoch_window_b32n_s16_d1_kernel(EpochArgs a, WinArgs w) {
  window_body<true, 16, true, 0, 1, false, true>(a, w);
}
// the product form with the straight-line last-bitfield copy (WinArgs.dma_k, kWinDmaK)
#define PZ_WINDOW_KERNEL_K(K)                                                                                 \
  extern "C" __global__ void __launch_bounds__(kWinThreads) pz_epoch_window_b32n_s16_k##K##_kernel(EpochArgs a, \
                                                                                                WinArgs w) {  \
    window_body<true, 16, true, 0, kWinDepth16, false, true, true, K>(a, w);                                 \
  }
PZ_WINDOW_KERNEL_K(1) PZ_WINDOW_KERNEL_K(2) PZ_WINDOW_KERNEL_K(3) PZ_WINDOW_KERNEL_K(5) PZ_WINDOW_KERNEL_K(9)
#undef PZ_WINDOW_KERNEL_K
PZ_WINDOW_KERNEL(pz_epoch_window_b32n_s32_kernel, true, 32, true, true)
PZ_WINDOW_KERNEL(pz_epoch_window_b32n_s64_kernel, true, 64, true, true)
PZ_WINDOW_KERNEL(pz_epoch_window_b32_s16_kernel, true, 16, true, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b32_s32_kernel, true, 32, true, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b32_s64_kernel, true, 64, true, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b64_s16_kernel, false, 16, true, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b64_s32_kernel, false, 32, true, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b64_s64_kernel, false, 64, true, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b32n_s16_g_kernel, true, 16, false, true)
PZ_WINDOW_KERNEL(pz_epoch_window_b32n_s32_g_kernel, true, 32, false, true)
PZ_WINDOW_KERNEL(pz_epoch_window_b32n_s64_g_kernel, true, 64, false, true)
PZ_WINDOW_KERNEL(pz_epoch_window_b32_s16_g_kernel, true, 16, false, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b32_s32_g_kernel, true, 32, false, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b32_s64_g_kernel, true, 64, false, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b64_s16_g_kernel, false, 16, false, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b64_s32_g_kernel, false, 32, false, false)
PZ_WINDOW_KERNEL(pz_epoch_window_b64_s64_g_kernel, false, 64, false, false)
#undef PZ_WINDOW_KERNEL

#ifdef PZ_AB_BUILD
// the A/B library's ablations of the product form (u32 offsets, 16-bit bounds, last bitfield in LDS)
#define PZ_WINDOW_ABL(X, D)                                                                              \
  extern "C" __global__ void __launch_bounds__(kWinThreads) pz_epoch_window_abl##X##_d##D##_kernel(EpochArgs a, \
                                                                                              WinArgs w) {  \
    window_body<true, 16, true, X, D, false, true, !((X) & 16)>(a, w);                                     \
  }
PZ_WINDOW_ABL(0, 1) PZ_WINDOW_ABL(0, 2) PZ_WINDOW_ABL(0, 3) PZ_WINDOW_ABL(0, 4)
PZ_WINDOW_ABL(1, 2) PZ_WINDOW_ABL(2, 2) PZ_WINDOW_ABL(4, 2) PZ_WINDOW_ABL(7, 2) PZ_WINDOW_ABL(16, 2)
PZ_WINDOW_ABL(48, 2) PZ_WINDOW_ABL(64, 2) PZ_WINDOW_ABL(128, 2) PZ_WINDOW_ABL(144, 2) PZ_WINDOW_ABL(4096, 2)
PZ_WINDOW_ABL(8192, 2) PZ_WINDOW_ABL(32, 2) PZ_WINDOW_ABL(65536, 2) PZ_WINDOW_ABL(131072, 2)
PZ_WINDOW_ABL(1048576, 2) PZ_WINDOW_ABL(2097152, 2) PZ_WINDOW_ABL(8388608, 2)
// the product form with phase stamps (tools/epoch_trace.py)
extern "C" __global__ void __launch_bounds__(kWinThreads) pz_epoch_window_trace_kernel(EpochArgs a, WinArgs w) {
  window_body<true, 16, true, 0, kWinDepth16, true, true>(a, w);
}
// (and the R > 1 product form's: one piece in flight)
extern "C" __global__ void __launch_bounds__(kWinThreads) pz_epoch_window_trace_d1_kernel(EpochArgs a, WinArgs w) {
  window_body<true, 16, true, 0, 1, true, true>(a, w);
}
// round 5's product (its prologue: the count after the first pieces' descriptors, two barriers,
// the range descriptor from global memory; the balances through the caches): A/B bit 1 << 18,
// with and without phase stamps
extern "C" __global__ void __launch_bounds__(kWinThreads) pz_epoch_window_np0_kernel(EpochArgs a, WinArgs w) {
  window_body<true, 16, true, 1 << 20, kWinDepth16, false, true, false>(a, w);
}
extern "C" __global__ void __launch_bounds__(kWinThreads) pz_epoch_window_trace_np0_kernel(EpochArgs a, WinArgs w) {
  window_body<true, 16, true, 1 << 20, kWinDepth16, true, true, false>(a, w);
}
#undef PZ_WINDOW_ABL
static int g_window_ablation = 0;
static uint64_t* g_window_trace = nullptr;
extern "C" int pz_debug_set_window_ablation(int x) {
  const int old = g_window_ablation;
  g_window_ablation = x;
  return old;
}
// the next launches stamp [blocks][4] {start, prologue done, loop done, end} into d_trace
extern "C" void pz_debug_set_window_trace(uint64_t* d_trace) { g_window_trace = d_trace; }
#endif

hipError_t launch_epoch_window(const EpochArgs& a, const WinArgs& w, hipStream_t s) {
  if (!a.ninst || !w.R) return hipSuccess;
  const bool b32 = w.bal32 != nullptr, llb = w.lds_lbf != 0;
  const int sew = w.se16 ? 16 : w.se ? 32 : 64;
  const void* k = nullptr;
#define PZ_PICK(B, S)                                                                            \
  k = llb ? (const void*)pz_epoch_window_##B##_s##S##_kernel : (const void*)pz_epoch_window_##B##_s##S##_g_kernel
  // One piece in flight per wave, and the last bitfield's copy after the count's take, when an
  // instance has several ranges (R > 1): 1M x 16 cold 58.0 -> 55.8 us; at R = 1 two pieces and
  // the straight-line copy first are faster, 54.3 against 57.8 (profiles/r06/
  // epoch_cold_depth1_r6s.txt; with the straight-line copy one piece gains only 58.0 -> 56.8,
  // epoch_cold_depth1_kd_r6t.txt)
  bool d1 = w.R > 1;
#ifdef PZ_AB_BUILD
  if (g_window_ablation == (1 << 22)) d1 = false;  // (A/B: the R = 1 form at R > 1 too)
#endif
  if (b32 && w.narrow) {
    if (sew == 16) PZ_PICK(b32n, 16);
    if (sew == 16 && llb && d1) {
      k = (const void*)pz_epoch_window_b32n_s16_d1_kernel;
    } else if (sew == 16 && llb && w.dma_k) {  // (the straight-line copy: WinArgs.dma_k)
      switch (w.dma_k) {
        case 1: k = (const void*)pz_epoch_window_b32n_s16_k1_kernel; break;
        case 2: k = (const void*)pz_epoch_window_b32n_s16_k2_kernel; break;
        case 3: k = (const void*)pz_epoch_window_b32n_s16_k3_kernel; break;
        case 5: k = (const void*)pz_epoch_window_b32n_s16_k5_kernel; break;
        case 9: k = (const void*)pz_epoch_window_b32n_s16_k9_kernel; break;
        default: return hipErrorInvalidValue;
      }
    }
    else if (sew == 32) PZ_PICK(b32n, 32);
    else PZ_PICK(b32n, 64);
  } else if (b32) {
    if (sew == 16) PZ_PICK(b32, 16);
    else if (sew == 32) PZ_PICK(b32, 32);
    else PZ_PICK(b32, 64);
  } else {
    if (sew == 16) PZ_PICK(b64, 16);
    else if (sew == 32) PZ_PICK(b64, 32);
    else PZ_PICK(b64, 64);
  }
#undef PZ_PICK
#ifdef PZ_AB_BUILD
  // (the A/B forms are the narrow product form's)
  if (g_window_trace && b32 && w.narrow && sew == 16 && llb)
    k = g_window_ablation == (1 << 18) ? (const void*)pz_epoch_window_trace_np0_kernel
        : d1                           ? (const void*)pz_epoch_window_trace_d1_kernel
                                       : (const void*)pz_epoch_window_trace_kernel;
  if (g_window_ablation && !g_window_trace && b32 && w.narrow && sew == 16 && llb) {
    switch (g_window_ablation) {  // ablation bits | prefetch depth << 8
      case 1 << 8: k = (const void*)pz_epoch_window_abl0_d1_kernel; break;
      case 2 << 8: k = (const void*)pz_epoch_window_abl0_d2_kernel; break;
      case 3 << 8: k = (const void*)pz_epoch_window_abl0_d3_kernel; break;
      case 4 << 8: k = (const void*)pz_epoch_window_abl0_d4_kernel; break;
      case 1: k = (const void*)pz_epoch_window_abl1_d2_kernel; break;
      case 2: k = (const void*)pz_epoch_window_abl2_d2_kernel; break;
      case 4: k = (const void*)pz_epoch_window_abl4_d2_kernel; break;
      case 7: k = (const void*)pz_epoch_window_abl7_d2_kernel; break;
      case 16: k = (const void*)pz_epoch_window_abl16_d2_kernel; break;
      case 48: k = (const void*)pz_epoch_window_abl48_d2_kernel; break;
      case 128: k = (const void*)pz_epoch_window_abl128_d2_kernel; break;
      case 4096: k = (const void*)pz_epoch_window_abl4096_d2_kernel; break;
      case 144: k = (const void*)pz_epoch_window_abl144_d2_kernel; break;
      case 64: k = (const void*)pz_epoch_window_abl64_d2_kernel; break;
      case 8192: k = (const void*)pz_epoch_window_abl8192_d2_kernel; break;
      case 32: k = (const void*)pz_epoch_window_abl32_d2_kernel; break;
      case 16384: k = (const void*)pz_epoch_window_b32n_s16_g_kernel; break;  // (the reward bits from L2, no LDS copy)
      case 65536: k = (const void*)pz_epoch_window_abl65536_d2_kernel; break;  // (timing: no multi-attestation votes)
      case 131072: k = (const void*)pz_epoch_window_abl131072_d2_kernel; break;  // (one attestation per trip)
      case 1 << 18: k = (const void*)pz_epoch_window_np0_kernel; break;  // (round 5's prologue)
      case 1 << 20: k = (const void*)pz_epoch_window_abl1048576_d2_kernel; break;  // (round 5's cached balances)
      case 1 << 21: k = (const void*)pz_epoch_window_abl2097152_d2_kernel; break;  // (the DMA before the first wait)
      case 1 << 23: k = (const void*)pz_epoch_window_abl8388608_d2_kernel; break;  // (loads at base priority)
      case 1 << 22: break;  // (the R = 1 product form at R > 1 too: two pieces, the straight-line copy)
      default: return hipErrorInvalidValue;
    }
  }
#endif
#ifdef PZ_AB_BUILD
  WinArgs wt = w;
  wt.trace = g_window_trace;
  const WinArgs& wl = wt;
#else
  const WinArgs& wl = w;
#endif
  const size_t lds = window_lds_bytes(w);
  if (lds > 48 * 1024) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  void* args[] = {const_cast<EpochArgs*>(&a), const_cast<WinArgs*>(&wl)};
  return hipLaunchKernel(k, dim3(a.ninst * w.R), dim3(kWinThreads), args, lds, s);
}

}  // namespace pz
