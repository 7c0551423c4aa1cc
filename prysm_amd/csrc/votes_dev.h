// Device code of the vote-cache tally shared by votes.hip and epoch.hip (the block engine's
// voter-major pass also runs inside pz_vote_words_count_kernel, beside a stateRecalc's epoch
// count blocks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "votes.h"

namespace pz {

__device__ __forceinline__ uint64_t wsum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One wave: attestation `att` (committee c, bitfield) adds its new voters to `slot`.
// A validator-range shard (lo, nval of nval_global) adds only its own members: balance and
// bm are indexed by v - lo.
__device__ __forceinline__ void tally_item(const uint32_t* __restrict__ committee, const uint64_t* __restrict__ coffs,
                                           uint32_t c, const uint8_t* bf, uint64_t blen,
                                           const uint64_t* __restrict__ balance, uint64_t nval, uint32_t* bm,
                                           uint64_t* total, uint64_t* errp, uint64_t lo = 0,
                                           uint64_t nval_global = 0) {
  if (!nval_global) nval_global = nval;
  const int lane = threadIdx.x & 63;
  const uint64_t cb = coffs[c], k = coffs[c + 1] - cb;
  uint64_t add = 0, err = 0;
  for (uint64_t i = lane; i < k; i += 64) {
    if (i >= 8 * blen) { err |= PZ_XLERR_BITFIELD; continue; }  // CheckBit would panic
    if (!((bf[i >> 3] >> (7 - (uint32_t)(i & 7))) & 1u)) continue;
    const uint32_t v = committee[cb + i];
    if (v >= nval_global) { err |= PZ_XLERR_MEMBER; continue; }
    const uint64_t lv = (uint64_t)v - lo;  // wraps huge below the range
    if (lv >= nval) continue;              // another rank's validator
    const uint32_t m = 1u << (lv & 31);
    // Voter bits only ever get set, so a plain read that already shows the bit is final;
    // a stale 0 (another XCD's L2) just falls through to the atomic, which decides.  After
    // the first attestation of a committee most voters are set: the atomics mostly vanish.
    if (bm[lv >> 5] & m) continue;
    const uint32_t old = atomicOr(&bm[lv >> 5], m);
    if (!(old & m)) add += balance[lv];
  }
  add = wsum64(add);
  const uint64_t e1 = __ballot(err != 0);
  if (lane == 0) {
    if (add) atomicAdd((unsigned long long*)total, (unsigned long long)add);
    if (e1) atomicOr((unsigned long long*)errp, 1ull);
  }
}

// 64-bit sum over the wave by DPP (no LDS round trips), wave-uniform.  Every lane of the wave
// must be active (lane 63 ends holding the total): call it in wave-uniform control flow.
__device__ __forceinline__ uint64_t wsum64_dpp(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#define PZ_DPP_STEP(CTRL, RM)                                                                   \
  {                                                                                             \
    const uint32_t l2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, RM, 0xf, false); \
    const uint32_t h2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, RM, 0xf, false); \
    const uint64_t t = (((uint64_t)hi << 32) | lo) + (((uint64_t)h2 << 32) | l2);               \
    lo = (uint32_t)t;                                                                           \
    hi = (uint32_t)(t >> 32);                                                                   \
  }
  PZ_DPP_STEP(0xB1, 0xf)   // quad_perm 1,0,3,2
  PZ_DPP_STEP(0x4E, 0xf)   // quad_perm 2,3,0,1
  PZ_DPP_STEP(0x141, 0xf)  // row_half_mirror
  PZ_DPP_STEP(0x140, 0xf)  // row_mirror
  PZ_DPP_STEP(0x142, 0xa)  // row_bcast15 into rows 1 and 3
  PZ_DPP_STEP(0x143, 0xc)  // row_bcast31 into rows 2 and 3
#undef PZ_DPP_STEP
  const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
  const uint32_t rh = (uint32_t)__builtin_amdgcn_readlane((int)hi, 63);
  return ((uint64_t)rh << 32) | rl;
}

// 64-bit OR over the wave by DPP, wave-uniform (every lane active; as wsum64_dpp).
__device__ __forceinline__ uint64_t wor64_dpp(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#define PZ_DPP_STEP(CTRL, RM)                                                          \
  lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, RM, 0xf, false);       \
  hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, RM, 0xf, false);
  PZ_DPP_STEP(0xB1, 0xf)
  PZ_DPP_STEP(0x4E, 0xf)
  PZ_DPP_STEP(0x141, 0xf)
  PZ_DPP_STEP(0x140, 0xf)
  PZ_DPP_STEP(0x142, 0xa)
  PZ_DPP_STEP(0x143, 0xc)
#undef PZ_DPP_STEP
  const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
  const uint32_t rh = (uint32_t)__builtin_amdgcn_readlane((int)hi, 63);
  return ((uint64_t)rh << 32) | rl;
}

// A block's justification-total partial sums (LDS): up to kVoteLdsWords id words, one running sum
// per parent.  Every wave of the flush adds to the same handful of totals (the transition's
// window), and device-scope atomics on one address serialise (~12 ns each): summed per block
// first, a flush issues one atomic per (block, parent) instead of one per (wave, parent).
constexpr int kVoteLdsWords = 4;
constexpr uint32_t kVoteLdsEmpty = 0xFFFFFFFFu;
struct VoteLds {
  uint32_t key[kVoteLdsWords];  // the id word of each slot, or kVoteLdsEmpty
  unsigned long long acc[kVoteLdsWords][64];
};

// The block's LDS slot for id word w (found, or claimed by lane 0), or -1 when all are taken
// (the caller then adds to the device totals directly).  Wave-uniform.
__device__ __forceinline__ int vote_lds_slot(VoteLds* L, uint32_t w) {
  int ls = -1;
  if ((threadIdx.x & 63) == 0) {
    for (int i = 0; i < kVoteLdsWords; ++i) {
      const uint32_t o = atomicCAS(&L->key[i], kVoteLdsEmpty, w);
      if (o == kVoteLdsEmpty || o == w) {
        ls = i;
        break;
      }
    }
  }
  return __builtin_amdgcn_readlane(ls, 0);
}

// The id word w's bits of the id range [lo, hi)
__device__ __forceinline__ uint64_t range_word_mask(uint32_t lo, uint32_t hi, uint32_t w) {
  const uint32_t b = 64 * w, l = lo > b ? lo - b : 0, h = hi < b + 64 ? (hi > b ? hi - b : 0) : 64;
  if (h <= l) return 0;
  return (h - l == 64 ? ~0ull : ((1ull << (h - l)) - 1)) << l;
}

// One wave of the voter-major tally: members [256 chunk, 256 chunk + 256) of attestation
// `att`'s committee (calculateBlockVoteCache, core.go:300-345, for all of its signed parent
// hashes at once).  Lane l holds members l + 64 q and parent l's id; the record (votes.h VoteRec:
// the bitfield, the parents' id run) loads in one request, then the member ids, then the
// balances.  The parents' ids are grouped by id word (a ballot per word, the word's mask by a
// DPP OR); per word one 64-bit atomicOr per voter, whose returned bits that were clear are the
// parents this voter is new for.  With M the parents any voter of the wave is new for: when
// every voter is new for all of M or for none of it (the usual cases: a new voter, or a voter
// seen one block before, whose window has moved by one parent), each of M's parents gains the
// new voters' balance sum (lane j adds it for parent bit j); otherwise, per distinct new-parent
// mask among the voters, their sum to each of its parents.  The sums go to the block's LDS
// totals (L).  Chunk 0 marks the
// parents' map entries present (core.go:322-326).
// (tools/tally_probe.hip: with `tr` non-null each wave stamps its phases, draining its memory
// operations first; the product passes none and the stamps compile away)
#define PZ_VSTAMP(i)                                       \
  if (tr) {                                                \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
    if ((threadIdx.x & 63) == 0) tr[i] = wall_clock64();   \
  }
__device__ __forceinline__ void vote_words_wave(const VoteWordArgs& a, uint64_t wid, VoteLds* L,
                                                uint64_t* tr = nullptr) {
  const int lane = threadIdx.x & 63;
  const uint64_t att = wid / a.chunks;
  const uint32_t chunk = (uint32_t)(wid % a.chunks);
  if (att >= a.natt) return;  // (wave-uniform)
  PZ_VSTAMP(0)
  // The record in one 64-B request (lane l reads its 16-B piece l & 3; the pieces go wave-wide by
  // readlane), beside it the bitfield bytes when they are not inline (a fixed stride: no record ->
  // bitfield hop); then the member ids.
  const uint4 pc = reinterpret_cast<const uint4*>(a.rec + att)[lane & 3];
  const uint32_t i0 = chunk * 256;
  uint32_t by[4];
  if (a.bits) {  // (wave-uniform)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t byte = (i0 + lane + 64 * q) >> 3;
      by[q] = a.bits[(uint64_t)att * a.bstride + (byte < a.bstride ? byte : a.bstride - 1)];
    }
  }
  auto rl = [](uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); };
  const uint32_t cb = rl(pc.x, 0), k = rl(pc.y, 0), s0 = rl(pc.z, 0), form = rl(pc.w, 0);
  PZ_VSTAMP(1)
  if (chunk > 0 && i0 >= k) return;
  if (!a.bits) {
    // member i = lane + 64 q (chunk 0): byte (lane >> 3) + 8 q = byte (lane >> 3) & 3 of word
    // 2 q + (lane >> 5); the words are lanes 2 and 3's pieces
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int src = q < 2 ? 2 : 3;  // (words 0-3 are lane 2's piece, 4-7 lane 3's)
      const uint32_t w0 = rl((q & 1) ? pc.z : pc.x, src), w1 = rl((q & 1) ? pc.w : pc.y, src);
      const uint32_t w = (lane & 32) ? w1 : w0;
      by[q] = w >> (8 * ((lane >> 3) & 3));
    }
  }
  uint32_t sl;
  if (form & kVoteIdsRow) {  // (wave-uniform) an explicit id row: one more round trip
    sl = a.slots[(uint64_t)s0 * 64 + lane];
  } else {
    const uint64_t step = ((uint64_t)rl(pc.y, 1) << 32) | rl(pc.x, 1);
    const uint64_t absent = ((uint64_t)rl(pc.w, 1) << 32) | rl(pc.z, 1);
    sl = ((absent >> lane) & 1) ? 0xFFFFFFFFu : s0 + (uint32_t)__builtin_popcountll(step & (~0ull >> (63 - lane)));
  }
  uint32_t v[4];
  bool on[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t i = i0 + lane + 64 * q;
    v[q] = i < k ? a.committee[cb + i] : 0u;
  }
  PZ_VSTAMP(2)
  uint64_t lv[4], bal[4], err = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t i = i0 + lane + 64 * q;
    on[q] = i < k && ((by[q] >> (7 - (i & 7))) & 1u);
    if (on[q] && v[q] >= a.nval_global) {  // validators[attesterIndex] would panic
      err = 1;
      on[q] = false;
    }
    lv[q] = (uint64_t)v[q] - a.val_offset;  // wraps huge below the range
    if (on[q] && lv[q] >= a.nval) on[q] = false;  // another rank's validator
    bal[q] = on[q] ? a.balance[lv[q]] : 0;
  }
  PZ_VSTAMP(3)
  const bool ok = sl != 0xFFFFFFFFu;
  if (chunk == 0 && ok) a.present[sl] = 1;
  // The parents' id words: the first two (the usual attestation spans two) have their atomics
  // issued together, one round trip for both; any further word follows one at a time.
  uint64_t pending = __ballot(ok);
  for (int round = 0; pending; ++round) {  // (wave-uniform)
    constexpr int kW = 2;
    uint32_t wv[kW];
    uint64_t mk[kW];
    int nwd = 0;
    for (; pending && nwd < (round == 0 ? kW : 1); ++nwd) {
      const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)sl, (int)__builtin_ctzll(pending)) >> 6;
      const bool in = ok && (sl >> 6) == w;
      pending &= ~__ballot(in);
      wv[nwd] = w;
      mk[nwd] = wor64_dpp(in ? 1ull << (sl & 63) : 0);
    }
    uint64_t nw[kW][4];
#pragma unroll
    for (int d = 0; d < kW; ++d) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        nw[d][q] = 0;
        if (d < nwd && on[q]) {
          uint64_t* row = a.bm + (uint64_t)wv[d] * a.nval;
          nw[d][q] = mk[d] & ~(uint64_t)atomicOr((unsigned long long*)&row[lv[q]], (unsigned long long)mk[d]);
        }
      }
    }
    if (round == 0) PZ_VSTAMP(4)
    for (int d = 0; d < nwd; ++d) {
      const uint32_t w = wv[d];
      // M: the word's parents some voter of the wave is new for (a block's attestation usually
      // brings one new parent for voters seen the block before, or all of them for new voters)
      const uint64_t M = wor64_dpp(nw[d][0] | nw[d][1] | nw[d][2] | nw[d][3]);
      if (!M) continue;  // (wave-uniform: nothing new)
      // the word's LDS slot (found or claimed by lane 0), or -1: the totals directly
      const int ls = vote_lds_slot(L, w);
      uint64_t xs = 0;
      bool uni = true;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // all or nothing: a voter new for every one of M's parents, or for none (the usual cases)
        uni = uni && (nw[d][q] == 0 || nw[d][q] == M);
        xs += nw[d][q] == M && on[q] ? bal[q] : 0;
      }
      if (__ballot(!uni) == 0) {
        const uint64_t S = wsum64_dpp(xs);  // the balances of the voters new for M's parents
        if (S && ((M >> lane) & 1)) {
          if (ls >= 0) atomicAdd(&L->acc[ls][lane], (unsigned long long)S);
          else atomicAdd((unsigned long long*)&a.totals[64ull * w + lane], (unsigned long long)S);
        }
      } else {
        // one pass per distinct new-parent mask among the wave's voters (ballot): its voters'
        // balance sum to each of its parents (a handful of masks, where a per-parent pass made
        // up to 64 and held the flush's last wave ~13 us, profiles/r04/vote_trace_r4z.txt)
        uint64_t rq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) rq[q] = __ballot(nw[d][q] != 0);
        for (;;) {  // (wave-uniform)
          const int qq = rq[0] ? 0 : rq[1] ? 1 : rq[2] ? 2 : rq[3] ? 3 : -1;
          if (qq < 0) break;
          const int leader = __builtin_ctzll(rq[qq]);
          const uint64_t src = qq == 0 ? nw[d][0] : qq == 1 ? nw[d][1] : qq == 2 ? nw[d][2] : nw[d][3];
          const uint64_t lm = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(src >> 32), leader) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)src, leader);
          uint64_t x = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const bool mine = nw[d][q] == lm && ((rq[q] >> lane) & 1);
            rq[q] &= ~__ballot(mine);
            x += mine ? bal[q] : 0;
          }
          const uint64_t Sm = wsum64_dpp(x);
          if (Sm && ((lm >> lane) & 1)) {
            if (ls >= 0) atomicAdd(&L->acc[ls][lane], (unsigned long long)Sm);
            else atomicAdd((unsigned long long*)&a.totals[64ull * w + lane], (unsigned long long)Sm);
          }
        }
      }
    }
  }
  if (__ballot(err != 0) && lane == 0) atomicOr((unsigned long long*)a.err, 1ull);
  PZ_VSTAMP(5)
}

// A grouped unit's LDS: the four waves' per-voter unions, merged.
struct VoteGroupLds {
  unsigned long long U[kVoteGroupWords][64];  // per word and voter lane: the parents it voted for
  unsigned long long UP[kVoteGroupWords];     // per word: every record's parents (map entries)
  uint32_t any[64];                            // per voter lane: its bit is set in some record
};

// One block (4 waves) of the grouped tally (votes.h VoteGroup): unit `unit` = members
// [64 m, 64 m + 64) of group g's committee, lane l holding member 64 m + l.  The group's records
// are split over the 4 waves (16 of every 64 each); a wave loads its records one per lane and
// computes each one's id range as masks over the group's words (the ids of a run are the range
// [s0, s0 + popcount(step)]), then a record-by-record loop ORs a record's masks into the union U
// of every voter whose bit it has.  The waves' unions merge in LDS; then wave w takes word w:
// one atomicOr per voter, the returned bits that were clear are the parents it is new for, and
// per distinct new-parent mask in the wave (ballot) its voters' balance sum goes to those
// parents' LDS totals.  Sums mod 2^64 commute: the totals are those of the reference's
// sequential loop (calculateBlockVoteCache, core.go:300-345, over the flush's attestations).
// Every thread of the block calls it (it holds a barrier).
__device__ __forceinline__ void vote_groups_block(const VoteWordArgs& a, uint32_t unit, VoteLds* L, VoteGroupLds* S,
                                                  uint64_t* tr = nullptr) {
  const int lane = threadIdx.x & 63, wq = threadIdx.x >> 6;
  const bool live = unit < a.nwaves;  // (block-uniform)
  int g = 0;
  while (g + 1 < (int)a.ngroups && a.groups[g + 1].wave0 <= unit) ++g;
  const VoteGroup G = a.groups[g];
  const uint32_t m = live ? unit - G.wave0 : 0;
  const uint32_t i = 64 * m + lane;
  const bool vin = live && i < G.k;
  PZ_VSTAMP(0)
  if (live) {
    uint64_t U[kVoteGroupWords], UP[kVoteGroupWords];
#pragma unroll
    for (int w = 0; w < kVoteGroupWords; ++w) U[w] = UP[w] = 0;
    bool any = false;
    for (uint32_t a0 = 16 * wq; a0 < G.n; a0 += 64) {  // (wave-uniform) this wave's 16 of every 64
      const uint32_t n = G.n - a0 < 16 ? G.n - a0 : 16;
      const uint32_t t0 = a0 + lane;
      const uint32_t att = lane < (int)n ? (G.stride ? G.first + G.stride * t0 : a.perm[G.first + t0]) : 0u;
      uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0, r2 = r0, r3 = r0;
      if (lane < (int)n) {
        const uint4* rp = reinterpret_cast<const uint4*>(a.rec + att);
        r0 = rp[0];
        r1 = rp[1];
        r2 = rp[2];
        r3 = rp[3];
      }
      // this unit's two bitfield words (members 64 m .. 64 m + 63): words 2 m and 2 m + 1 of the
      // record's eight (words 0-3 in r2, 4-7 in r3)
      const uint32_t bA = m == 0 ? r2.x : m == 1 ? r2.z : m == 2 ? r3.x : r3.z;
      const uint32_t bB = m == 0 ? r2.y : m == 1 ? r2.w : m == 2 ? r3.y : r3.w;
      uint64_t rm[kVoteGroupWords];
      {
        const uint64_t step = ((uint64_t)r1.y << 32) | r1.x, absent = ((uint64_t)r1.w << 32) | r1.z;
        const bool none = lane >= (int)n || absent == ~0ull;
        const uint32_t lo = r0.z, hi = r0.z + (uint32_t)__builtin_popcountll(step) + 1;
#pragma unroll
        for (int w = 0; w < kVoteGroupWords; ++w) {
          rm[w] = none ? 0 : range_word_mask(lo, hi, G.wlo + w);
          UP[w] |= wor64_dpp(rm[w]);
        }
      }
      if (a0 == 16u * wq) PZ_VSTAMP(1)
      const uint32_t sh = 8 * ((lane >> 3) & 3) + 7 - (lane & 7);
#pragma unroll
      for (int t = 0; t < 16; ++t) {  // record by record (unrolled: constant lanes)
        // (records past n have no bit and no parents: lanes >= n hold zero words)
        const uint32_t wA = (uint32_t)__builtin_amdgcn_readlane((int)bA, t);
        const uint32_t wB = (uint32_t)__builtin_amdgcn_readlane((int)bB, t);
        const bool bit = vin && ((((lane & 32) ? wB : wA) >> sh) & 1u);
        any = any || bit;
        const uint64_t sel = bit ? ~0ull : 0ull;
#pragma unroll
        for (int w = 0; w < kVoteGroupWords; ++w) {
          const uint64_t mk = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(rm[w] >> 32), t) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rm[w], t);
          U[w] |= mk & sel;
        }
      }
    }
#pragma unroll
    for (int w = 0; w < kVoteGroupWords; ++w) {
      if (U[w]) atomicOr(&S->U[w][lane], (unsigned long long)U[w]);
      if (lane == 0 && UP[w]) atomicOr(&S->UP[w], (unsigned long long)UP[w]);
    }
    if (any) atomicOr(&S->any[lane], 1u);
  }
  PZ_VSTAMP(2)
  __syncthreads();
  if (!live) return;
  const uint32_t v = vin ? a.committee[G.cb + i] : 0u;
  uint64_t lv = (uint64_t)v - a.val_offset;  // wraps huge below the range
  bool on = S->any[lane] != 0;
  uint64_t err = 0;
  if (on && v >= a.nval_global) {  // validators[attesterIndex] would panic
    err = 1;
    on = false;
  }
  if (on && lv >= a.nval) on = false;  // another rank's validator
  if (wq == 0 && __ballot(err != 0) && lane == 0) atomicOr((unsigned long long*)a.err, 1ull);
  if (wq >= (int)G.nw) return;  // (wave-uniform) wave wq: id word G.wlo + wq
  const uint32_t wd = G.wlo + wq;
  const uint64_t U = S->U[wq][lane];
  if (m == 0 && ((S->UP[wq] >> lane) & 1)) a.present[64ull * wd + lane] = 1;
  const uint64_t bal = on && U ? a.balance[lv] : 0;
  PZ_VSTAMP(3)
  uint64_t nw = 0;
  if (on && U) nw = U & ~(uint64_t)atomicOr((unsigned long long*)&a.bm[(uint64_t)wd * a.nval + lv], (unsigned long long)U);
  PZ_VSTAMP(4)
  uint64_t rem = __ballot(nw != 0);
  if (rem) {
    const int ls = vote_lds_slot(L, wd);
    while (rem) {  // (wave-uniform) one pass per distinct new-parent mask
      const int leader = __builtin_ctzll(rem);
      const uint64_t lm = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(nw >> 32), leader) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)nw, leader);
      const bool mine = nw == lm && ((rem >> lane) & 1);
      rem &= ~__ballot(mine);
      const uint64_t Sm = wsum64_dpp(mine ? bal : 0);
      if (Sm && ((lm >> lane) & 1)) {
        if (ls >= 0) atomicAdd(&L->acc[ls][lane], (unsigned long long)Sm);
        else atomicAdd((unsigned long long*)&a.totals[64ull * wd + lane], (unsigned long long)Sm);
      }
    }
  }
  PZ_VSTAMP(5)
}

// The tally part of a launch: nblk blocks of blockDim.x / 64 waves, this one `bid` (the block's
// totals summed in LDS, then one device atomic per parent it added to).  With a.gather_out the
// last block to finish gathers the justification totals (MI355X_MICROARCH.md's last-block
// hand-off: every wave drains its atomics before the block barrier, one lane per block takes a
// ticket, the block taking the last reads the totals with agent-scope loads -- they are only
// written by device-scope atomics -- into the pinned output, the sequence word last).
__device__ __forceinline__ void vote_words_body(const VoteWordArgs& a, uint32_t nblk, uint32_t bid,
                                                uint64_t* trace = nullptr) {
  __shared__ VoteLds L;
  __shared__ VoteGroupLds S;
  for (uint32_t t = threadIdx.x; t < kVoteLdsWords * 64; t += blockDim.x) L.acc[t >> 6][t & 63] = 0;
  if (threadIdx.x < kVoteLdsWords) L.key[threadIdx.x] = kVoteLdsEmpty;
  if (a.ngroups) {
    for (uint32_t t = threadIdx.x; t < kVoteGroupWords * 64; t += blockDim.x) S.U[t >> 6][t & 63] = 0;
    if (threadIdx.x < kVoteGroupWords) S.UP[threadIdx.x] = 0;
    if (threadIdx.x < 64) S.any[threadIdx.x] = 0;
  }
  __syncthreads();
  const uint64_t wid = (uint64_t)bid * (blockDim.x >> 6) + (threadIdx.x >> 6);
  uint64_t* tr = trace ? trace + wid * 8 : nullptr;
  if (a.ngroups)
    vote_groups_block(a, bid, &L, &S, tr);  // (blockDim.x == kVoteWordThreads: 4 waves)
  else
    vote_words_wave(a, wid, &L, tr);
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < kVoteLdsWords * 64; t += blockDim.x) {
    const uint32_t w = L.key[t >> 6];
    const unsigned long long x = L.acc[t >> 6][t & 63];
    if (w != kVoteLdsEmpty && x) atomicAdd((unsigned long long*)&a.totals[64ull * w + (t & 63)], x);
  }
  PZ_VSTAMP(6)
  if (!a.gather_out) return;
  __shared__ uint32_t last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == nblk - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last) return;
  const int j = threadIdx.x;
  if (j < kJustifySlots) {
    const uint32_t sl = a.gq.slot[j];
    a.gather_out[j] =
        sl == 0xFFFFFFFFu ? 0 : __hip_atomic_load(&a.totals[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (j == 0) {
    a.gather_out[kJustifySlots] = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the sequence word last: every lane's stores drained, then one system-scope release store
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (j == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&a.gather_out[kJustifySlots + 1], a.gather_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  PZ_VSTAMP(7)
}
#undef PZ_VSTAMP

}  // namespace pz
