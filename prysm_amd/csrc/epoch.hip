// Epoch-transition (T/R) kernels for gfx950: participation tallies, crosslink tallies,
// FFG rewards and the post-reward total balance, all uint64 with Go wrap-around.
//
// Restates (paths relative to /root/reference/beacon-chain):
//   casper/validator.go:45-77   Active/Exited/QueuedValidatorIndices  (classify + compaction)
//   casper/validator.go:93-102  GetAttestersTotalDeposit               (bitfield popcount)
//   casper/incentives.go:14-32  CalculateRewards                       (rank-targeted RMW)
//   blockchain/core.go:459-464  next-cycle total balance               (fused into the RMW)
//   blockchain/core.go:515-555  processCrosslinks tallies + winner     (committee gather-sums)
// HBM streaming is SoA and coalesced (each wave-instruction reads 512 contiguous bytes of a
// u64 array); participation uses wave ballots, sums use DPP/shuffle wave reductions and one
// integer atomic per block (u64 adds commute, so results are order-independent and exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "../../include/prysm_hip.h"
#include "epoch.h"
#include "votes_dev.h"

namespace pz {

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// The same sum by DPP (votes_dev.h wsum64_dpp: no LDS round trips, where the xor-shuffle form
// is a dependent chain of 12 ds_bpermute); wave-uniform, every lane active.
__device__ __forceinline__ uint64_t wave_sum_dpp(uint64_t v) { return wsum64_dpp(v); }
// Sum over the wave of a per-lane count of at most 4 (a ballot per unit; wave-uniform).
__device__ __forceinline__ uint64_t wave_count4(const bool (&x)[4]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) c += __popcll(__ballot(x[i]));
  return c;
}
__device__ __forceinline__ uint64_t wave_max(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

__device__ __forceinline__ bool kind_pred(int kind, uint64_t s, uint64_t e, uint64_t d) {
  return kind == PZ_KIND_ACTIVE ? (s <= d && d < e) : kind == PZ_KIND_EXITED ? (s < d && e <= d) : (s > d);
}

// utils/checkbit.go:4-15 — MSB-first bit `i` of `bf` (caller guarantees i < 8*len).
__device__ __forceinline__ uint32_t bit_at(const uint8_t* bf, uint64_t i) {
  return (bf[i >> 3] >> (7 - (uint32_t)(i & 7))) & 1u;
}

// Block-wide u64 sum/max of per-thread values; result valid in thread 0.
template <bool MAX>
__device__ __forceinline__ uint64_t block_reduce(uint64_t v, uint64_t* sh) {
  v = MAX ? wave_max(v) : wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  uint64_t r = 0;
  if (threadIdx.x == 0) {
    r = sh[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = MAX ? (sh[w] > r ? sh[w] : r) : r + sh[w];
  }
  return r;
}

// ------------------------------------------------------------------------------------------
// Pass 1: [validator blocks | popcount blocks | crosslink blocks (1 wave per attestation)]
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t pack64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

// Bit i of x -> bit 2i of the result (interleaves two 32-lane ballots into a 64-bit mask).
__device__ __forceinline__ uint64_t spread32(uint32_t x) {
  uint64_t v = x;
  v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
  v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
  v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
  v = (v | (v << 2)) & 0x3333333333333333ull;
  v = (v | (v << 1)) & 0x5555555555555555ull;
  return v;
}

constexpr uint32_t kGroup = 32;  // chunks of one instance per round (validator / reward blocks)

struct CountGrid {
  uint64_t vbpi, nvb, pbpi, npb, nxb;
  int vec;            // 1: validator arrays read 16 B per lane (nval even, 16-B aligned)
  uint64_t xl_j;      // crosslink blocks per instance (4 attestations per block)
  int xl_affine;      // 1: crosslink blocks of instance i land on XCD i % 8 (>= 8 instances)
  int do_pop;         // 0: the popcount blocks only reset the winners (no bitfield bytes, or
                      //    a crosslink-only launch)
};

// Crosslink tally for one attestation, one wave (core.go:533-545).  Members are processed
// 256 at a time with every committee load, then every balance gather, in flight together
// (two dependent round trips per 256 members instead of two per 64).
// Committee-order layout (a.co_index): committee c is the contiguous storage range
// [coffs[c], coffs[c+1]), so its balances stream coalesced and the bitfield bit of a member is
// its offset in the range -- no member-index loads, no random balance gathers.  A rank adds
// the part of the range it holds.
__device__ __forceinline__ void crosslink_wave_co(const EpochArgs& a, uint64_t ga, int lane) {
  const uint64_t inst = (uint32_t)ga / (uint32_t)a.natt;
  const uint32_t c = a.att_comm[ga];
  const uint64_t cb = a.coffs[c], ce = a.coffs[c + 1];
  const uint64_t lo = cb > a.val_offset ? cb : a.val_offset;
  const uint64_t hi = ce < a.val_offset + a.nval ? ce : a.val_offset + a.nval;
  const uint64_t bb = a.boffs[ga], blen = a.boffs[ga + 1] - bb;
  const uint8_t* bf = a.bits + bb;
  const uint64_t* B = a.balance + inst * a.nval - a.val_offset;  // indexed by storage position
  uint64_t tot = 0, vote = 0;
  bool e_bf = false;
  for (uint64_t p0 = lo; p0 < hi; p0 += 256) {
    uint64_t bal[4];
    uint32_t byte[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t p = p0 + j * 64 + lane;
      const uint64_t pos = p - cb;
      bal[j] = p < hi ? B[p] : 0;
      byte[j] = (p < hi && pos < 8 * blen) ? bf[pos >> 3] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t p = p0 + j * 64 + lane;
      if (p < hi) {
        const uint64_t pos = p - cb;
        e_bf |= pos >= 8 * blen;
        tot += bal[j];
        vote += ((byte[j] >> (7 - (uint32_t)(pos & 7))) & 1u) ? bal[j] : 0;
      }
    }
  }
  tot = wave_sum(tot);
  vote = wave_sum(vote);
  const uint64_t e2 = __ballot(e_bf);
  if (lane == 0) {
    a.vote[ga] = vote;
    a.total[ga] = tot;
    if (e2) atomicAdd((unsigned long long*)&a.scal[inst * kScal + kErrXl], (unsigned long long)kErrBitfield);
  }
}

template <int V>
__device__ __forceinline__ void crosslink_wave(const EpochArgs& a, uint64_t ga, int lane) {
  if (a.co_index) {
    crosslink_wave_co(a, ga, lane);
    return;
  }
  const uint64_t inst = (uint32_t)ga / (uint32_t)a.natt;  // 32-bit: B*natt < 2^32 (host-checked)
  const uint32_t c = a.att_comm[ga];
  const uint64_t cb = a.coffs[c], k = a.coffs[c + 1] - cb;
  const uint64_t bb = a.boffs[ga], blen = a.boffs[ga + 1] - bb;
  const uint8_t* bf = a.bits + bb;
  const uint64_t* B = a.balance + inst * a.nval;
  const uint32_t* C = a.committee + cb;
  uint64_t tot = 0, vote = 0;
  bool e_mem = false, e_bf = false;
  for (uint64_t r0 = 0; r0 < k; r0 += 256) {
    uint32_t mem[4];
    uint32_t byte[4];
    uint64_t bal[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t i = r0 + j * 64 + lane;
      mem[j] = C[i < k ? i : 0];
    }
    uint32_t pos[4];  // bitfield position of the member (its index in the full committee)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t i = r0 + j * 64 + lane;
      pos[j] = a.cpos ? a.cpos[cb + (i < k ? i : 0)] : (uint32_t)i;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t i = r0 + j * 64 + lane;
      byte[j] = (i < k && pos[j] < 8 * blen) ? bf[pos[j] >> 3] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t i = r0 + j * 64 + lane;
      const uint64_t local = (uint64_t)mem[j] - a.val_offset;  // wraps huge when mem < val_offset
      const bool own = i < k && mem[j] < a.nval_global && local < a.nval;
      if (V & 8)  // probe: nontemporal gather
        bal[j] = own ? __builtin_nontemporal_load(B + local) : 0;
      else if (V & 16)  // probe: sc1 (L1-bypassing) gather
        bal[j] = own ? __hip_atomic_load(B + local, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      else
        bal[j] = own ? B[local] : 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t i = r0 + j * 64 + lane;
      if (i < k) {
        e_mem |= mem[j] >= a.nval_global;
        e_bf |= pos[j] >= 8 * blen;
        tot += bal[j];
        vote += ((byte[j] >> (7 - (pos[j] & 7))) & 1u) ? bal[j] : 0;
      }
    }
  }
  tot = wave_sum(tot);
  vote = wave_sum(vote);
  const uint64_t e1 = __ballot(e_mem), e2 = __ballot(e_bf);
  if (lane == 0) {
    a.vote[ga] = vote;
    a.total[ga] = tot;
    const uint64_t ebits = (e1 ? kErrMember : 0) | (e2 ? kErrBitfield : 0);
    if (ebits) atomicAdd((unsigned long long*)&a.scal[inst * kScal + kErrXl], (unsigned long long)ebits);
  }
}

// V is an A/B knob for tools/ (0 in the product): bit 0 = validator blocks in rounds of
// kGroup chunks per instance; bit 1 = a max-index atomic from every block; bit 2 = no
// non-matching-count atomic (timing probe only: its results are wrong); 8 / 16 = the crosslink
// balance gathers as nontemporal / sc1 loads.
template <int V>
__device__ __forceinline__ void count_body(const EpochArgs& a, const CountGrid& g, uint64_t bid) {
  __shared__ uint64_t sh[kThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // Grid order: [crosslink blocks | validator blocks | popcount blocks]: the latency-bound
  // gathers start first.  (An even interleave measured slower: its per-block 64-bit index
  // division costs more than the overlap gains.)
  if (bid < g.nxb) {
    const uint64_t x = bid;
    uint64_t inst, j;
    if (g.xl_affine) {  // blocks x and x+8 share an XCD: keep one instance's balances in one L2
      const uint64_t qj = x >> 3;
      const uint32_t q32 = (uint32_t)qj / (uint32_t)g.xl_j;
      inst = (uint64_t)q32 * 8 + (x & 7);
      j = (uint32_t)qj - q32 * (uint32_t)g.xl_j;
    } else {
      inst = (uint32_t)x / (uint32_t)g.xl_j;
      j = (uint32_t)x - (uint32_t)inst * (uint32_t)g.xl_j;
    }
    const uint64_t att = j * (kThreads / 64) + wave;
    if (inst >= a.ninst || att >= a.natt) return;
    crosslink_wave<V>(a, inst * a.natt + att, lane);
    return;
  }
  const uint64_t b = bid - g.nxb;

  if (b < g.nvb) {  // ---- classify + count + active mask + max active index
    // Instance-major order, one chunk of 2,048 validators per block (DRAM locality).  The
    // epilogue's per-instance atomics are device-scope, performed at the memory side at ~12 ns
    // each on one address, so they serialise when the blocks of one instance finish together
    // (512 blocks per 1M-validator instance: 57.6 us for the pass against 47.5 without them).
    // Blocks therefore count the validators that do NOT match `kind` (slot kNoMatch, an atomic
    // only from a block that has some) and the finish pass turns that into kNact; with every
    // validator active the pass issues one atomic per instance (the max index).
    uint64_t chunk, inst;
    if (V & 1) {  // r02 probe: rounds of kGroup chunks per instance
      const uint32_t per_round = kGroup * a.ninst;
      const uint32_t r = (uint32_t)b / per_round, rem = (uint32_t)b - r * per_round;
      inst = rem / kGroup;
      chunk = (uint64_t)r * kGroup + (rem % kGroup);
      if (chunk >= g.vbpi) return;  // the last round's tail
    } else {
      inst = (uint32_t)b / (uint32_t)g.vbpi;
      chunk = (uint32_t)b - (uint32_t)inst * (uint32_t)g.vbpi;
    }
    const uint64_t base = chunk * kValPerBlock;
    const uint64_t d = a.dynasty[inst];
    const uint64_t* S = a.start + inst * a.nval;
    const uint64_t* E = a.end + inst * a.nval;
    uint64_t* mask = a.act_mask ? a.act_mask + inst * ((a.nval + 63) / 64) : nullptr;
    uint32_t cnt = 0;
    uint64_t maxi1 = 0;
    // the validator just past this block, loaded up front (it decides whether this block's
    // max-index atomic is needed; see the epilogue)
    const uint64_t bend = base + kValPerBlock < a.nval ? base + kValPerBlock : a.nval;
    bool next_act = false;
    if (!(V & 2) && tid == 0 && bend < a.nval) next_act = kind_pred(a.kind, S[bend], E[bend], d);
    if (g.vec) {  // 16 B per lane: validators i0, i0+1 (nval even, arrays 16-B aligned)
#pragma unroll
      for (int j = 0; j < kValPerThread / 2; ++j) {
        const uint64_t wb = base + (uint64_t)j * (2 * kThreads) + wave * 128;
        const uint64_t i0 = base + (uint64_t)j * (2 * kThreads) + 2 * tid;
        bool a0 = false, a1 = false;
        if (i0 < a.nval) {
          const uint4 s = *reinterpret_cast<const uint4*>(S + i0);
          const uint4 e = *reinterpret_cast<const uint4*>(E + i0);
          a0 = kind_pred(a.kind, pack64(s.x, s.y), pack64(e.x, e.y), d);
          a1 = kind_pred(a.kind, pack64(s.z, s.w), pack64(e.z, e.w), d);
        }
        const uint64_t b0 = __ballot(a0), b1 = __ballot(a1);
        if (a1) maxi1 = a.val_offset + i0 + 2;
        else if (a0) maxi1 = a.val_offset + i0 + 1;
        if (lane == 0) {
          cnt += (uint32_t)(__popcll(b0) + __popcll(b1));
          if (mask) {  // lane L holds validators 2L, 2L+1: interleave the two ballots
            const uint64_t w0 = wb >> 6;
            const uint64_t m0 = spread32((uint32_t)b0) | (spread32((uint32_t)b1) << 1);
            const uint64_t m1 = spread32((uint32_t)(b0 >> 32)) | (spread32((uint32_t)(b1 >> 32)) << 1);
            if ((w0 << 6) < a.nval) mask[w0] = m0;
            if (((w0 + 1) << 6) < a.nval) mask[w0 + 1] = m1;
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < kValPerThread; ++j) {
        const uint64_t i = base + (uint64_t)j * kThreads + tid;
        bool act = false;
        if (i < a.nval) act = kind_pred(a.kind, S[i], E[i], d);
        const uint64_t bal = __ballot(act);
        if (act) maxi1 = a.val_offset + i + 1;
        if (lane == 0) {
          cnt += (uint32_t)__popcll(bal);
          const uint64_t w = (base + (uint64_t)j * kThreads + wave * 64) >> 6;
          if (mask && (w << 6) < a.nval) mask[w] = bal;
        }
      }
    }
    const uint64_t c = block_reduce<false>(lane == 0 ? cnt : 0, sh);
    const uint64_t m = block_reduce<true>(maxi1, sh);
    if (tid == 0) {
      if (a.blk_cnt) a.blk_cnt[inst * g.vbpi + chunk] = (uint32_t)c;
      const uint64_t nomatch = (bend - base) - c;
      if (nomatch && !(V & 4)) atomicAdd((unsigned long long*)&a.scal[inst * kScal + kNoMatch], (unsigned long long)nomatch);
      // the committee-order layout maps rank to index only when every validator matches
      if (nomatch && a.co_index)
        atomicOr((unsigned long long*)&a.scal[inst * kScal + kErrXl], (unsigned long long)kErrLayout);
      // The max active index needs an atomic only from a block that can hold it: the last
      // chunk, a block whose last validator is inactive, or one followed by an inactive
      // validator.  With every validator active only the last chunk adds one.
      const bool need = (V & 2) ? m != 0 : m && (bend == a.nval || m != a.val_offset + bend || !next_act);
      if (need) atomicMax((unsigned long long*)&a.scal[inst * kScal + kMaxIdx1], (unsigned long long)m);
      // CalculateRewards would panic on CheckBit(last bitfield, m-1) (incentives.go:23)
      if (m && a.kind == PZ_KIND_ACTIVE) {
        uint64_t L = 0;
        if (a.natt) {
          const uint64_t last = inst * a.natt + a.natt - 1;
          L = a.boffs[last + 1] - a.boffs[last];
        }
        if (a.natt == 0 || (m - 1) >= 8 * L)
          atomicAdd((unsigned long long*)&a.scal[inst * kScal + kErrRwd], 1ull);
      }
    }
    return;
  }

  {  // ---- popcount of this instance's bitfield bytes
    const uint64_t pb = b - g.nvb;
    const uint64_t inst = (uint32_t)pb / (uint32_t)g.pbpi, chunk = (uint32_t)pb - (uint32_t)inst * (uint32_t)g.pbpi;
    if (chunk == 0 && a.winner)  // winners are reset here; the winner pass runs after this launch
      for (uint32_t s = tid; s < a.nrec; s += kThreads) a.winner[inst * a.nrec + s] = 0xffffffffu;
    if (!g.do_pop || chunk % a.pop_world != a.pop_rank) return;
    const uint64_t beg = a.boffs[inst * a.natt], end = a.boffs[inst * a.natt + a.natt];
    const uint64_t cb = beg + chunk * kPopBytesPerBlock;
    if (cb >= end) return;
    const uint64_t ce = end < cb + kPopBytesPerBlock ? end : cb + kPopBytesPerBlock;
    uint64_t cnt = 0;
    const uint64_t u0 = cb & ~15ull;
    for (uint64_t u = u0 + 16ull * tid; u < ce; u += 16ull * kThreads) {
      if (u >= cb && u + 16 <= ce) {
        const uint4 q = *reinterpret_cast<const uint4*>(a.bits + u);
        cnt += __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
      } else {
        for (uint64_t k = u < cb ? cb : u; k < u + 16 && k < ce; ++k) cnt += __popc((uint32_t)a.bits[k]);
      }
    }
    uint64_t c = block_reduce<false>(cnt, sh);
    if (tid == 0 && c) atomicAdd((unsigned long long*)&a.scal[inst * kScal + kPop], (unsigned long long)c);
  }
}

#define PZ_COUNT_KERNEL(NAME, V) \
  extern "C" __global__ void __launch_bounds__(kThreads) NAME(EpochArgs a, CountGrid g) { count_body<V>(a, g, blockIdx.x); }
PZ_COUNT_KERNEL(pz_epoch_count_kernel, 0)
#undef PZ_COUNT_KERNEL

// ------------------------------------------------------------------------------------------
// Crosslink winners (core.go:549-555): the first attestation, in order, whose 3*vote >=
// 2*total and whose dynasty beats the shard's record wins that shard (atomicMin of index).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void winner_one(const EpochArgs& a, uint64_t ga) {
  const uint64_t inst = (uint32_t)ga / (uint32_t)a.natt;
  // the shard id loads beside the tallies (two dependent round trips per attestation, not three)
  const uint64_t v = a.vote[ga], t = a.total[ga];
  const uint32_t shard = a.att_shard[ga];
  asm volatile("" ::"v"(shard));  // keeps the compiler from sinking the load into the branch
  if (3ull * v >= 2ull * t) {  // uint64 wrap, as in Go
    if (shard >= a.nrec) {
      atomicAdd((unsigned long long*)&a.scal[inst * kScal + kErrXl], (unsigned long long)kErrShard);
      return;
    }
    if (a.dynasty[inst] > a.rec_dynasty[inst * a.nrec + shard])
      atomicMin(&a.winner[inst * a.nrec + shard], (uint32_t)(ga - inst * a.natt));
  }
}

extern "C" __global__ void __launch_bounds__(kThreads) pz_epoch_winner_kernel(EpochArgs a) {
  const uint64_t ga = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ga >= (uint64_t)a.ninst * a.natt) return;
  winner_one(a, ga);
}

// ------------------------------------------------------------------------------------------
// General rank path: compacted active list act_list[inst][rank] = global index.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void compact_block(const EpochArgs& a, uint64_t vbpi, int force, uint64_t blk) {
  __shared__ uint32_t wsum[kThreads / 64 * kValPerThread];
  __shared__ uint64_t base_off;
  const uint64_t inst = (uint32_t)blk / (uint32_t)vbpi, chunk = (uint32_t)blk - (uint32_t)inst * (uint32_t)vbpi;
  if (!force && a.scal[inst * kScal + kNoMatch] == 0) return;  // rank == index: nothing to compact
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    uint64_t s = 0;
    for (uint64_t c = 0; c < chunk; ++c) s += a.blk_cnt[inst * vbpi + c];
    base_off = s;
  }
  const uint64_t* mask = a.act_mask + inst * ((a.nval + 63) / 64);
  const uint64_t base = chunk * kValPerBlock;
  uint64_t words[kValPerThread];
#pragma unroll
  for (int j = 0; j < kValPerThread; ++j) {
    const uint64_t w = (base + (uint64_t)j * kThreads + wave * 64) >> 6;
    words[j] = (w << 6) < a.nval ? mask[w] : 0;  // wave-uniform
    if (lane == 0) wsum[j * (kThreads / 64) + wave] = (uint32_t)__popcll(words[j]);
  }
  __syncthreads();
  // element order inside the block is j-major then wave then lane == ascending index
  uint32_t* out = a.act_list + inst * a.nval_global;
#pragma unroll
  for (int j = 0; j < kValPerThread; ++j) {
    uint64_t off = base_off;
    for (int q = 0; q < j * (kThreads / 64) + wave; ++q) off += wsum[q];
    const uint64_t bits = words[j];
    if ((bits >> lane) & 1) {
      const uint64_t below = lane ? __popcll(bits & ((1ull << lane) - 1)) : 0;
      out[off + below] = (uint32_t)(a.val_offset + base + (uint64_t)j * kThreads + tid);
    }
  }
}

extern "C" __global__ void __launch_bounds__(kThreads)
pz_epoch_compact_kernel(EpochArgs a, uint64_t vbpi, int force) {
  compact_block(a, vbpi, force, blockIdx.x);
}

// Finish pass 1 of 2 in one launch: [winner threads | compaction blocks].
extern "C" __global__ void __launch_bounds__(kThreads)
pz_epoch_mid_kernel(EpochArgs a, uint64_t vbpi, uint64_t nwb, int do_compact) {
  if (blockIdx.x < nwb) {
    const uint64_t ga = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ga < (uint64_t)a.ninst * a.natt) winner_one(a, ga);
    return;
  }
  if (do_compact) compact_block(a, vbpi, 0, blockIdx.x - nwb);
}

// ------------------------------------------------------------------------------------------
// Multi-rank general rank path.  Each rank's count pass wrote the active bitmask of its own
// shard; an all-gather hands every rank the rank-major stack gmask[world][B][shard_words]
// (rank r owns global validators [r*64*shard_words, (r+1)*64*shard_words)).  From it every
// rank rebuilds the same global compacted list act_list[B][nval_global], which the reward
// pass reads by global rank position (incentives.go:22-23: validators[i] <- CheckBit(bf, a[i])).
// Both kernels: grid (chunks of 2048 global validators, B), one wave per block; an instance
// whose validators are all active (rank == index) is skipped.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t gmask_word(const uint64_t* gmask, uint32_t ninst, uint64_t sw, uint64_t inst,
                                               uint64_t w) {
  const uint64_t r = w / sw;
  return gmask[(r * ninst + inst) * sw + (w - r * sw)];
}

constexpr int kWordsPerChunk = (int)(kValPerBlock / 64);  // 32

extern "C" __global__ void __launch_bounds__(64)
pz_epoch_gcount_kernel(EpochArgs a, const uint64_t* __restrict__ gmask, uint64_t sw, uint32_t* gblk) {
  const uint64_t inst = blockIdx.y, chunk = blockIdx.x;
  if (a.scal[inst * kScal + kNoMatch] == 0) return;
  const int lane = threadIdx.x;
  const uint64_t nw = (a.nval_global + 63) / 64;
  const uint64_t w = chunk * kWordsPerChunk + lane;
  uint64_t c = (lane < kWordsPerChunk && w < nw) ? (uint64_t)__popcll(gmask_word(gmask, a.ninst, sw, inst, w)) : 0;
  c = wave_sum(c);
  if (lane == 0) gblk[inst * gridDim.x + chunk] = (uint32_t)c;
}

extern "C" __global__ void __launch_bounds__(64)
pz_epoch_gcompact_kernel(EpochArgs a, const uint64_t* __restrict__ gmask, uint64_t sw, const uint32_t* gblk) {
  const uint64_t inst = blockIdx.y, chunk = blockIdx.x;
  if (a.scal[inst * kScal + kNoMatch] == 0) return;
  const int lane = threadIdx.x;
  uint64_t base = 0;  // active validators in the chunks before this one
  for (uint64_t c = lane; c < chunk; c += 64) base += gblk[inst * gridDim.x + c];
  base = wave_sum(base);
  const uint64_t nw = (a.nval_global + 63) / 64;
  const uint64_t w = chunk * kWordsPerChunk + lane;
  uint64_t bits = (lane < kWordsPerChunk && w < nw) ? gmask_word(gmask, a.ninst, sw, inst, w) : 0;
  // exclusive prefix of the per-word counts across the wave (ascending word == ascending index)
  const uint32_t cnt = (uint32_t)__popcll(bits);
  uint32_t incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= o) incl += t;
  }
  uint64_t pos = base + incl - cnt;
  uint32_t* out = a.act_list + inst * a.nval_global;
  while (bits) {
    const int b = __ffsll((unsigned long long)bits) - 1;
    out[pos++] = (uint32_t)(w * 64 + b);
    bits &= bits - 1;
  }
}

hipError_t launch_epoch_gather_compact(const EpochArgs& a, const uint64_t* gmask, uint64_t sw, uint32_t* gblk,
                                       hipStream_t s) {
  const uint64_t chunks = vblocks_per_inst(a.nval_global);
  if (!chunks || !a.ninst) return hipSuccess;
  const dim3 grid((uint32_t)chunks, a.ninst);
  hipLaunchKernelGGL(pz_epoch_gcount_kernel, grid, dim3(64), 0, s, a, gmask, sw, gblk);
  hipLaunchKernelGGL(pz_epoch_gcompact_kernel, grid, dim3(64), 0, s, a, gmask, sw, gblk);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Pass 2: CalculateRewards (incentives.go:14-32) fused with the next-cycle balance sum
// (core.go:459-464).  Position p receives +-1 by CheckBit(last bitfield, active[p]).
// ------------------------------------------------------------------------------------------
// One validator position: +-1 at rank p from bit active[p] of the last bitfield, and the
// post-reward balance if p is active.
__device__ __forceinline__ uint64_t reward_one(uint64_t bal, uint64_t gp, bool applied, uint64_t nact,
                                               bool all_active, const uint32_t* list, const uint8_t* lastbf,
                                               bool* changed) {
  if (applied && gp < nact) {
    const uint64_t idx = all_active ? gp : list[gp];
    *changed = true;
    return bit_at(lastbf, idx) ? bal + PZ_ATTESTER_REWARD : bal - PZ_ATTESTER_REWARD;
  }
  return bal;
}

// MODE is an ablation knob for tools/epoch_parts.py only (0 in the product): bit 1 skips the
// last-bitfield loads, bit 2 skips the block reduction + atomic.  Results are wrong for MODE != 0.
// scal_ro / boffs_ro / tdep_ro alias a.scal / a.boffs / a.total_deposit but are only read
// (the slots written here, kApplied / kNextBal, are not the ones read), so they are
// declared __restrict__ at the kernel boundary: the compiler then reads them with s_load
// instead of vector loads that would queue behind, and reorder, the balance stream.
template <int MODE>
__device__ __forceinline__ void reward_body(EpochArgs a, uint64_t vbpi, int vec,
                                            const uint64_t* __restrict__ scal_ro,
                                            const uint64_t* __restrict__ boffs_ro,
                                            const uint64_t* __restrict__ tdep_ro, uint64_t inst_, uint64_t chunk_) {
  __shared__ uint64_t sh[kThreads / 64];
  // 2-D grid: x = instance, y = chunk (no per-block division).  The next
  // step's accumulators (scal_next) are zeroed at the END: a store ahead of the scalar reads
  // would stop the compiler from using s_load for them.
  if (vec) {  // 16 B per lane read-modify-write (nval even, arrays 16-B aligned)
    // instance-minor order (x = instance, y = chunk): the next-cycle-total atomics of one
    // instance never arrive in a burst (measured at 1M x 16: 39 us for the pass against 45 in
    // rounds of kGroup chunks and 45 instance-major; at 65,536 x 256 all three ~39-40 us)
    const uint64_t inst = inst_, chunk = chunk_;
    const int tid = threadIdx.x;
    uint64_t* B = a.balance + inst * a.nval;
    const uint64_t base = chunk * kValPerBlock;
    constexpr int kPairs = kValPerThread / 2;
    // phase 1: every 16-B balance load in flight BEFORE the per-instance scalars are
    // awaited (the scalar round trip would otherwise serialise in front of every block)
    uint4 q[kPairs];
#pragma unroll
    for (int j = 0; j < kPairs; ++j) {
      const uint64_t p = base + (uint64_t)j * (2 * kThreads) + 2 * tid;
      q[j] = *reinterpret_cast<const uint4*>(B + (p < a.nval ? p : 0));
    }
    const uint64_t* sc = scal_ro + inst * kScal;
    const uint64_t pop = sc[kPop], nact = a.nval_global - sc[kNoMatch];
    const uint64_t dep = pop * PZ_DEFAULT_BALANCE;
    const bool thr = (dep * 3ull) >= (tdep_ro[inst] * 2ull);  // uint64 wrap, incentives.go:18-20
    // Go panics in processCrosslinks or CalculateRewards: leave balances untouched.  A
    // predicate, not an early return, so the balance loads above cannot be sunk below it.
    const bool skip = sc[kErrXl] != 0 || (thr && nact > 0 && sc[kErrRwd] != 0);
    const bool applied = thr && !skip;
    const bool all_active = (nact == a.nval_global);
    const uint8_t* lastbf = a.natt ? a.bits + boffs_ro[inst * a.natt + a.natt - 1] : nullptr;
    const uint64_t* mask = a.act_mask ? a.act_mask + inst * ((a.nval + 63) / 64) : nullptr;
    const uint32_t* list = a.act_list ? a.act_list + inst * a.nval_global : nullptr;
    uint64_t sum = 0;
    // Fast bit path (all active, byte-aligned range): the wave needs 4 x 16 contiguous bytes
    // of the last bitfield (positions base + j*512 + wave*128 + [0,128)); one byte load per
    // lane fetches them and __shfl hands each lane its byte (one memory round trip instead
    // of one per element).
    const int lane = tid & 63, wave = tid >> 6;
    const uint64_t gbase = a.val_offset + base;
    const bool fastbits = (MODE & 1) == 0 && applied && all_active && lastbf && (gbase & 7) == 0 && !a.co_index;
    // committee order: position p holds validator co_index[p]; with every validator active its
    // rank is its index, so its reward bit is bit co_index[p] of the last bitfield (incentives.go:
    // 22-27); the index pair of each lane is loaded with the balances
    uint2 cix[kPairs];
    if (a.co_index && applied) {
#pragma unroll
      for (int j = 0; j < kPairs; ++j) {
        const uint64_t p = base + (uint64_t)j * (2 * kThreads) + 2 * tid;
        cix[j] = *reinterpret_cast<const uint2*>(a.co_index + (p < a.nval ? p : 0));
      }
    }
    uint32_t mybyte = 0;
    if (fastbits) {
      const uint64_t L = boffs_ro[inst * a.natt + a.natt] - boffs_ro[inst * a.natt + a.natt - 1];
      const uint64_t bi = (gbase >> 3) + (uint64_t)(lane >> 4) * 64 + wave * 16 + (lane & 15);
      mybyte = bi < L ? lastbf[bi] : 0u;
    }
    // phase 2: rewards + sums; phase 3: stores
#pragma unroll
    for (int j = 0; j < kPairs; ++j) {
      const uint64_t p = base + (uint64_t)j * (2 * kThreads) + 2 * tid;
      uint32_t byte_j = 0;
      if (fastbits) byte_j = (uint32_t)__shfl((int)mybyte, j * 16 + (lane >> 2), 64);
      if (p < a.nval) {
        const uint64_t gp = a.val_offset + p;
        bool changed = false;
        uint64_t b0, b1;
        if (MODE & 1) {
          b0 = pack64(q[j].x, q[j].y) + 1;
          b1 = pack64(q[j].z, q[j].w) - 1;
          changed = applied;
        } else if (a.co_index) {  // every validator active (the count pass checks): rank == index
          b0 = pack64(q[j].x, q[j].y);
          b1 = pack64(q[j].z, q[j].w);
          if (applied) {
            b0 = bit_at(lastbf, cix[j].x) ? b0 + PZ_ATTESTER_REWARD : b0 - PZ_ATTESTER_REWARD;
            b1 = bit_at(lastbf, cix[j].y) ? b1 + PZ_ATTESTER_REWARD : b1 - PZ_ATTESTER_REWARD;
            changed = true;
          }
        } else if (fastbits) {  // gp < nact for every p < nval here (all active)
          const uint32_t sh0 = 7u - (uint32_t)(gp & 7);
          b0 = pack64(q[j].x, q[j].y);
          b1 = pack64(q[j].z, q[j].w);
          b0 = ((byte_j >> sh0) & 1u) ? b0 + PZ_ATTESTER_REWARD : b0 - PZ_ATTESTER_REWARD;
          b1 = ((byte_j >> (sh0 - 1)) & 1u) ? b1 + PZ_ATTESTER_REWARD : b1 - PZ_ATTESTER_REWARD;
          changed = true;
        } else {
          b0 = reward_one(pack64(q[j].x, q[j].y), gp, applied, nact, all_active, list, lastbf, &changed);
          b1 = reward_one(pack64(q[j].z, q[j].w), gp + 1, applied, nact, all_active, list, lastbf, &changed);
        }
        if (changed) {
          *reinterpret_cast<uint4*>(B + p) =
              make_uint4((uint32_t)b0, (uint32_t)(b0 >> 32), (uint32_t)b1, (uint32_t)(b1 >> 32));
        }
        if (all_active) {
          sum += b0 + b1;
        } else {
          const uint64_t mw = mask[p >> 6];
          sum += ((mw >> (p & 63)) & 1) ? b0 : 0;
          sum += ((mw >> ((p + 1) & 63)) & 1) ? b1 : 0;
        }
      }
    }
    if (MODE & 2) {
      asm volatile("" ::"v"(sum));
      return;
    }
    uint64_t s = block_reduce<false>(sum, sh);
    if (tid == 0) {
      if (s && !skip) atomicAdd((unsigned long long*)&a.scal[inst * kScal + kNextBal], (unsigned long long)s);
      if (chunk == 0) {  // agent-scope (sc1) stores: a hand-off's last block reads them (below)
        __hip_atomic_store(&a.scal[inst * kScal + kApplied], (uint64_t)(applied ? 1 : 0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.scal[inst * kScal + kNact], nact, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (a.scal_next && chunk == 0 && tid < kScal) a.scal_next[inst * kScal + tid] = 0;
    return;
  }
  const uint64_t inst = inst_, chunk = chunk_;
  const int tid = threadIdx.x;
  const uint64_t* sc = a.scal + inst * kScal;
  const uint64_t pop = sc[kPop], nact = a.nval_global - sc[kNoMatch];
  const bool xl_err = sc[kErrXl] != 0;
  if (chunk == 0 && tid == 0) __hip_atomic_store(&a.scal[inst * kScal + kNact], nact, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t dep = pop * PZ_DEFAULT_BALANCE;                 // GetAttestersTotalDeposit
  const bool applied = (dep * 3ull) >= (a.total_deposit[inst] * 2ull);  // uint64 wrap
  const bool rwd_err = applied && nact > 0 && sc[kErrRwd] != 0;
  if (a.scal_next && chunk == 0 && tid < kScal) a.scal_next[inst * kScal + tid] = 0;
  if (xl_err || rwd_err) {  // Go panics before/while rewarding: leave balances untouched
    if (chunk == 0 && tid == 0) __hip_atomic_store(&a.scal[inst * kScal + kApplied], (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const bool all_active = (nact == a.nval_global);
  const uint8_t* lastbf = nullptr;
  if (a.natt) lastbf = a.bits + a.boffs[inst * a.natt + a.natt - 1];
  uint64_t* B = a.balance + inst * a.nval;
  const uint64_t* mask = a.act_mask ? a.act_mask + inst * ((a.nval + 63) / 64) : nullptr;
  const uint32_t* list = a.act_list ? a.act_list + inst * a.nval_global : nullptr;
  const uint64_t base = chunk * kValPerBlock;
  uint64_t sum = 0;
#pragma unroll
  for (int j = 0; j < kValPerThread; ++j) {
    const uint64_t p = base + (uint64_t)j * kThreads + tid;
    if (p >= a.nval) break;
    const uint64_t gp = a.val_offset + p;
    uint64_t bal = B[p];
    if (applied && gp < nact) {
      // committee order: the validator at p is co_index[p], rank == index (all active)
      const uint64_t idx = a.co_index ? a.co_index[p] : all_active ? gp : list[gp];
      bal = bit_at(lastbf, idx) ? bal + PZ_ATTESTER_REWARD : bal - PZ_ATTESTER_REWARD;
      B[p] = bal;
    }
    const bool act = all_active ? true : ((mask[p >> 6] >> (p & 63)) & 1);
    if (act) sum += bal;
  }
  uint64_t s = block_reduce<false>(sum, sh);
  if (tid == 0) {
    if (s) atomicAdd((unsigned long long*)&a.scal[inst * kScal + kNextBal], (unsigned long long)s);
    if (chunk == 0) __hip_atomic_store(&a.scal[inst * kScal + kApplied], (uint64_t)(applied ? 1 : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

#define PZ_REWARD_KERNEL(NAME, MODE)                                                            \
  extern "C" __global__ void __launch_bounds__(kThreads)                                         \
  NAME(EpochArgs a, uint64_t vbpi, int vec, const uint64_t* __restrict__ scal_ro,                \
       const uint64_t* __restrict__ boffs_ro, const uint64_t* __restrict__ tdep_ro) {            \
    reward_body<MODE>(a, vbpi, vec, scal_ro, boffs_ro, tdep_ro, blockIdx.x, blockIdx.y);          \
  }
PZ_REWARD_KERNEL(pz_epoch_reward_kernel, 0)
#undef PZ_REWARD_KERNEL

// The reward pass of ONE instance with its results handed to the host (EpochHandoff): the
// last block to finish copies the instance's scalars and the winners mid wrote into mapped
// pinned memory, zeroes the scalars for the next epoch's count, and writes the sequence word
// last behind a system-scope release -- so the host polls one word instead of a D2H, an event
// record and an event wait (three runtime calls per transition of the chain engine).
// Hand-off (MI355X_MICROARCH.md, the table's first row): every wave drains its stores and
// atomics (s_waitcnt vmcnt(0)) before the block barrier, one lane per block adds to ONE
// counter, the block whose add returns the last count reads with agent-scope (sc1) loads what
// the other blocks wrote by atomics or agent-scope stores (reward_body's scalar writes).
// nwb > 0: the crosslink winners of every attestation (the mid pass's winner threads) run as
// the grid's first nwb blocks, beside the reward blocks -- one launch less when no compaction is
// needed (every validator active: the reward pass reads no active list).  The winners read only
// the count pass's tallies; a winner's processCrosslinks panic (a shard >= nrec) is then raised
// with rewards already applied, which no caller reads (the chain is poisoned by the panic).
extern "C" __global__ void __launch_bounds__(kThreads)
pz_epoch_reward_handoff_kernel(EpochArgs a, uint64_t vbpi, int vec, const uint64_t* __restrict__ scal_ro,
                               const uint64_t* __restrict__ boffs_ro, const uint64_t* __restrict__ tdep_ro,
                               EpochHandoff h, uint32_t nwb) {
  if (blockIdx.x < nwb) {
    const uint64_t ga = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ga < (uint64_t)a.natt) winner_one(a, ga);
  } else {
    reward_body<0>(a, vbpi, vec, scal_ro, boffs_ro, tdep_ro, 0, blockIdx.x - nwb);
  }
  __shared__ uint32_t last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(h.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last) return;
  const uint32_t tid = threadIdx.x;
  if (tid < kScal) {
    h.out[tid] = __hip_atomic_load(&a.scal[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.scal[tid], (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  uint32_t* w = reinterpret_cast<uint32_t*>(h.out + kScal);
  for (uint32_t r = tid; r < h.nrec; r += kThreads)
    w[r] = __hip_atomic_load(&a.winner[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid == 0) __hip_atomic_store(h.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&h.out[kScal + (h.nrec + 1) / 2], h.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static bool vec_ok(const EpochArgs& a);
hipError_t launch_epoch_reward_handoff(const EpochArgs& a, const EpochHandoff& h, bool winners, hipStream_t s) {
  if (a.ninst != 1) return hipErrorInvalidValue;
  const uint64_t vbpi = std::max<uint64_t>(1, vblocks_per_inst(a.nval));
  const uint32_t nwb = winners ? (uint32_t)(((uint64_t)a.natt + kThreads - 1) / kThreads) : 0u;
  hipLaunchKernelGGL(pz_epoch_reward_handoff_kernel, dim3((uint32_t)(nwb + vbpi)), dim3(kThreads), 0, s, a, vbpi,
                     vec_ok(a) ? 1 : 0, a.scal, a.boffs, a.total_deposit, h, nwb);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// One-pass epoch (committee order, every validator active; epoch.h "one-pass epoch").
// ------------------------------------------------------------------------------------------
// Fused: one wave per committee piece (FusedArgs.items: <= 256 positions of one committee,
// pairs 16-B aligned), kFusedWaves pieces of one instance per block; grid (B, piece groups).
// A wave streams start, end, balance and co_index of its piece (16 B per lane per pair, every
// load issued before anything waits), adds the pre-reward balances into its committee's
// tallies (two wave sums, two atomics per attestation of the committee), then classifies,
// rewards, stores and sums; the block adds its next-cycle sum with one atomic.
constexpr int kFusedWaves = 8;

// MODE: an ablation knob for tools/ (0 in the product; results are wrong otherwise): bit 0 no
// crosslink tallies, bit 1 reward bit from the balance instead of the last bitfield, bit 2 no
// balance store, bit 3 no start/end loads (every validator taken as active), bit 4 start/end
// loads with the default cache policy, bit 5 instance-major grid; bit 8 (product when the
// state has FusedArgs.lastco) the reward bits read in position order instead of looked up.
//
// Measured choices (tools/fused_parts.py, 65,536 x 256 / 1M x 16 step, us): start/end loads
// nontemporal (read once per step: leaving the 256 MiB Infinity Cache to the balances, which
// are read and written) 142 -> 128 / 132 -> 122.  Grid order: instance-major won before the
// block-merged tally atomics (126 / 119 against 128 / 122); with them instance-minor is
// 2-5 us faster on every box measured since (107 / 100 against 110 / 103).  Staging the last
// bitfield in LDS (65,536 validators: 8 KiB per instance) measured 112 against 110: the block
// barrier costs more than the random L2 lookups it removes.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16_nt(const uint64_t* p) {
  const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(x.x, x.y, x.z, x.w);
}
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 ld8_nt(const uint32_t* p) {
  const v2u x = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
  return make_uint2(x.x, x.y);
}

template <int E = kFusedWaves>
__device__ __forceinline__ void fused_block_end(const EpochArgs& a, const FusedArgs& f, const uint32_t* xg,
                                                const uint64_t* xt, const uint64_t* xv, const uint64_t* xs,
                                                const uint64_t* xn, uint64_t inst, uint64_t grp, int lane,
                                                bool skip, bool applied, uint64_t pop, uint64_t ferr, bool rwd_err);
__device__ __forceinline__ void one_tail(const EpochArgs& a, const FusedArgs& f, int tid);

// FusedArgs.win_in_wave: attestation g's complete tallies (vote v, committee total t) are in
// this wave -- the winner rule of core.go:549-555 (the first attestation, in order, with
// 3*vote >= 2*total whose dynasty beats its shard's record) as an atomicMin over g, and g's
// next-step tallies zeroed.
// w = f.att_win[g]: {shard (< nrec: the host takes the one-launch step only then), its record's
// dynasty}.
template <bool PRO>
// d = a.dynasty[inst], loaded once by the caller (not behind the tallies).
__device__ __forceinline__ void one_win(const EpochArgs& a, const FusedArgs& f, uint64_t inst, uint32_t g, uint64_t v,
                                        uint64_t t, uint2 w, uint64_t d) {
  if (3ull * v >= 2ull * t && d > (uint64_t)w.y) atomicMin(&a.winner[inst * a.nrec + w.x], g);
  if (PRO) {  // (with a pre launch, pre zeroes the tallies)
    f.vote_next[inst * a.natt + g] = 0;
    f.total_next[inst * a.natt + g] = 0;
  }
}

template <int MODE>
__device__ __forceinline__ void fused_body(EpochArgs a, FusedArgs f, const uint64_t* __restrict__ pre_ro,
                                           const uint64_t* __restrict__ boffs_ro, const uint64_t* __restrict__ tdep_ro,
                                           const uint4* __restrict__ items_ro,
                                           const FusedCommittee* __restrict__ cinfo_ro,
                                           const uint32_t* __restrict__ catt_offs_ro,
                                           const uint32_t* __restrict__ catt_ro) {
  // per wave: {attestation of its committee (single-attestation committees), total, vote, next sum, nomatch}
  __shared__ uint64_t xt[kFusedWaves], xv[kFusedWaves], xs[kFusedWaves], xn[kFusedWaves];
  __shared__ uint32_t xg[kFusedWaves];
  constexpr bool ONE = (MODE & 512) != 0;  // single-launch step (launch_epoch_one)
  // single launch over B instances (launch_epoch_multi): ONE's per-block prologue, inst = blockIdx.x
  constexpr bool MULTI = (MODE & 2048) != 0;
  constexpr bool PRO = ONE || MULTI;  // each block counts its instance's bitfields itself
  // MODE & 4096: a 1-D grid mapped XCD-aware.  Blocks are dealt round-robin over the 8 XCDs
  // (MI355X_MICROARCH.md, "Workgroup dispatch"; for speed only, the map is a bijection either
  // way): block L runs on XCD L % 8, so the blocks of piece group y -- every instance's --
  // are given to XCD y % 8 and the group's co_index words (shared by the instances) are
  // fetched into one L2 instead of all eight.  Per XCD the order is group-major, instance-minor.
  uint64_t inst, grp;
  if (MODE & 4096) {
    const uint32_t L = blockIdx.x, j = L >> 3, B = (uint32_t)a.ninst;
    inst = j % B;
    grp = 8ull * (j / B) + (L & 7);
    if (grp * kFusedWaves >= f.nitems && grp != 0) return;  // the pad groups (group 0 always runs)
  } else {
    inst = (MODE & 32) ? blockIdx.y : blockIdx.x;
    grp = (MODE & 32) ? blockIdx.x : blockIdx.y;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t item = grp * kFusedWaves + wave;
  // MODE & (1 << 22) (A/B: tools/epoch_single.py): thread 0's wall clock at the start, when its
  // stream loads have landed, after the count's barrier, before the block's tail, at the end
  constexpr bool TRc = (MODE & (1 << 22)) != 0;
  uint64_t tst[5] = {0, 0, 0, 0, 0};
  if (TRc) tst[0] = __builtin_amdgcn_s_memrealtime();
  const uint64_t dyn = a.dynasty[inst];  // (the winner rule's, issued with the first loads)
  uint64_t pop = 0, ferr = 0;
  if (!PRO) {
    pop = pre_ro[inst * kPre];
    ferr = pre_ro[inst * kPre + 1];
  }
  const uint64_t lb = boffs_ro[inst * a.natt + a.natt - 1];
  const uint64_t L = boffs_ro[inst * a.natt + a.natt] - lb;
  const bool rwd_err = (a.nval_global - 1) >= 8 * L;  // CheckBit(last, N-1) panics (incentives.go:23)
  bool thr = (pop * PZ_DEFAULT_BALANCE * 3ull) >= (tdep_ro[inst] * 2ull);  // incentives.go:18-20
  bool skip = ferr != 0 || (thr && rwd_err);     // Go panics: balances stay untouched
  bool applied = thr && !skip;
  // ONE: this block's own bit count (GetAttestersTotalDeposit, validator.go:93-102) and
  // bitfield-length checks (core.go:538-541) over the whole instance, issued before the stream
  constexpr uint64_t kProBits = MULTI ? kMultiMaxBitBytes : kOneMaxBitBytes;
  constexpr uint32_t kProAtt = MULTI ? kMultiMaxAtt : kOneMaxAtt;
  constexpr int kOneLoads = PRO ? (int)((kProBits + 16) / (16 * 64 * kFusedWaves)) + 1 : 1;
  constexpr int kOneAtts = PRO ? (int)((kProAtt + 64 * kFusedWaves - 1) / (64 * kFusedWaves)) : 1;
  uint4 pq[kOneLoads];
  uint32_t ocs[kOneAtts];
  uint64_t ob0[kOneAtts], ob1[kOneAtts];
  // ONE: the instance's bitfield bytes [pbase, pend), staged in LDS by the loads above; the
  // reward bits are then looked up there (the last bitfield is the region's tail)
  __shared__ uint4 lbits[PRO ? kOneLoads * 64 * kFusedWaves : 1];
  const uint64_t pbeg = PRO ? boffs_ro[inst * a.natt] : 0, pend = PRO ? boffs_ro[inst * a.natt + a.natt] : 0,
                 pbase = pbeg & ~15ull;
  // (the rounds the instance's bytes need: block-uniform, so the unused rounds of the
  // capacity issue no loads)
  const uint32_t nlr = PRO ? (uint32_t)((pend - pbase + 16 * 64 * kFusedWaves - 1) / (16 * 64 * kFusedWaves)) : 0;
  if (PRO) {
#pragma unroll
    for (int k = 0; k < kOneLoads; ++k) {  // branch-free inside a round: the bitfield buffer is padded by 16 B
      const uint64_t u = pbase + 16ull * ((uint64_t)k * 64 * kFusedWaves + tid);
      pq[k] = (uint32_t)k < nlr ? *reinterpret_cast<const uint4*>(a.bits + (u < pend ? u : pbase)) : make_uint4(0, 0, 0, 0);
    }
    // (every round's loads issued, past natt at entry 0: a select on the round's use turned each
    // round's loads into a wait before the next round's -- the length check below skips g >= natt)
#pragma unroll
    for (int k = 0; k < kOneAtts; ++k) {
      const uint64_t g = (uint64_t)k * 64 * kFusedWaves + tid, gc = inst * a.natt + (g < a.natt ? g : 0);
      ocs[k] = f.att_csize[gc];
      ob0[k] = boffs_ro[gc];
      ob1[k] = boffs_ro[gc + 1];
    }
  }
  uint64_t sum = 0, nm = 0, ts = 0, vs = 0;
  uint32_t g1 = kNoAtt;  // the wave's single attestation, combined across the block below
  // every wave runs the body (a wave without a piece has no element in range)
  const bool have = item < f.nitems;
  if constexpr ((MODE & 32768) != 0) {
    // QUAD lanes (the multi-instance se/se16 kernels): lane l takes the 4 contiguous positions
    // p0 + 4l .. +3 of the piece (p0 the piece's window start, 4-aligned locally), so that every
    // column load is 16 B per lane -- balance 2 x 16 B, {start, end} 16 B (se16) or 2 x 16 B
    // (se), co_index 16 B -- where the pair layout read se16 and co_index 8 B per lane (an 8-B
    // access streams at 0.54-0.70 of the 16-B rate, MI355X_MICROARCH.md).
    static_assert(!PRO && (MODE & 1024), "quad lanes serve the multi-instance se/se16 kernels");
    static_assert(!(MODE & 524288) || (MODE & 32768), "u32 balance offsets on the quad lanes only");
    const uint4 it = have ? items_ro[item] : make_uint4((uint32_t)a.val_offset, 0, 0, (uint32_t)a.val_offset);
    const uint64_t ws = it.x, we = (uint64_t)it.x + it.y, cb = it.w;
    FusedCommittee ci;
    {
      const uint4 ic = have ? f.items_ci[inst * f.nitems + item] : make_uint4(0, 0, 0, kNoAtt);
      ci.boff = pack64(ic.x, ic.y);
      ci.nbits = ic.z;
      ci.ga = ic.w;
    }
    const bool wiw = f.win_fused != 0;
    const uint2 win1 = (wiw && ci.ga < kNoAtt) ? f.att_win[inst * a.natt + ci.ga] : make_uint2(0, 0);
    const uint64_t p0 = (ws - a.val_offset) & ~3ull;
    const uint64_t p = p0 + 4ull * lane, g = a.val_offset + p;
    bool v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = g + i >= ws && g + i < we;
    const uint64_t pp = (v[0] || v[1] || v[2] || v[3]) ? p : p0;
    constexpr bool B32 = (MODE & 524288) != 0;  // balances as u32 offsets (FusedArgs.bal32)
    uint64_t* Bal = a.balance + inst * f.vstride;
    uint32_t* Bal32 = B32 ? f.bal32 + inst * f.vstride : nullptr;
    uint4 qb0, qb1;
    if (B32) {
      qb0 = *reinterpret_cast<const uint4*>(Bal32 + pp);
      qb1 = make_uint4(0, 0, 0, 0);
    } else {
      qb0 = *reinterpret_cast<const uint4*>(Bal + pp);
      qb1 = *reinterpret_cast<const uint4*>(Bal + pp + 2);
    }
    const uint64_t bbase = B32 ? f.bal32_base[inst] : 0;
    uint32_t sv[4], ev[4];
    if (MODE & 8) {  // (ablation: no start/end loads, every validator taken as active)
#pragma unroll
      for (int i = 0; i < 4; ++i) sv[i] = 0, ev[i] = 0xFFFFFFFFu;
    } else if (MODE & 16384) {
      const uint4 w = ld16_nt(reinterpret_cast<const uint64_t*>(f.se16 + inst * f.vstride + pp));
      sv[0] = w.x & 0xFFFFu, ev[0] = w.x >> 16, sv[1] = w.y & 0xFFFFu, ev[1] = w.y >> 16;
      sv[2] = w.z & 0xFFFFu, ev[2] = w.z >> 16, sv[3] = w.w & 0xFFFFu, ev[3] = w.w >> 16;
    } else {
      const uint4 w0 = ld16_nt(reinterpret_cast<const uint64_t*>(f.se + inst * f.vstride + pp));
      const uint4 w1 = ld16_nt(reinterpret_cast<const uint64_t*>(f.se + inst * f.vstride + pp + 2));
      sv[0] = w0.x, ev[0] = w0.y, sv[1] = w0.z, ev[1] = w0.w, sv[2] = w1.x, ev[2] = w1.y, sv[3] = w1.z, ev[3] = w1.w;
    }
    uint32_t lcw = 0;
    uint4 cix = make_uint4(0, 0, 0, 0);
    if (MODE & 256)
      lcw = f.lastco[inst * f.lcw + (pp >> 5)];
    else if (!(MODE & 2))  // (ablation 2: no reward-bit lookups)
      cix = *reinterpret_cast<const uint4*>(a.co_index + pp);
    // the committee bitfield bytes holding the lane's positions (two at most), branch-free and
    // clamped to the bitfield: x = g + i - cb is position g + i's bit; lanes before the committee
    // start clamp to bit 0
    const int64_t qs = (int64_t)(g - cb);
    const int64_t last = (int64_t)ci.nbits - 1;
    const int64_t qlo = qs < 0 ? 0 : qs > last ? last : qs;
    const int64_t qhi = qs + 3 < 0 ? 0 : qs + 3 > last ? last : qs + 3;
    uint32_t byA = 0, byB = 0;
    if (!(MODE & 1) && ci.ga < kNoAtt && ci.nbits) {
      // the lane's (at most two) bytes in ONE 8-B load from the dword below them (the bitfield
      // buffer is padded by 16 B; bytes outside the bitfield are masked by x < nbits below)
      (void)qhi;
      const uint64_t bp = ci.boff + ((uint64_t)qlo >> 3), da = bp & ~3ull;
      uint64_t win;
      __builtin_memcpy(&win, __builtin_assume_aligned(a.bits + da, 4), 8);
      const uint32_t sh = (uint32_t)(bp - da) * 8;
      byA = (uint32_t)(win >> sh) & 0xFFu;
      byB = (uint32_t)(win >> (sh + 8)) & 0xFFu;
    }
    uint64_t b[4];
    if (B32) {  // u64 balance = base + offset, wrapping as Go's uint64 does
      b[0] = bbase + qb0.x, b[1] = bbase + qb0.y, b[2] = bbase + qb0.z, b[3] = bbase + qb0.w;
    } else {
      b[0] = pack64(qb0.x, qb0.y), b[1] = pack64(qb0.z, qb0.w), b[2] = pack64(qb1.x, qb1.y), b[3] = pack64(qb1.z, qb1.w);
    }
    // crosslink tallies on the pre-reward balances (core.go:533-545)
    if (!(MODE & 1) && ci.ga != kNoAtt) {
      uint64_t t = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) t += v[i] ? b[i] : 0;
      ts = wave_sum_dpp(t);
      if (ci.ga != kManyAtt) {
        uint64_t vv = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t x = qs + i;
          const uint32_t by = ((x >> 3) == (qlo >> 3)) ? byA : byB;
          if (v[i] && (uint64_t)x < (uint64_t)ci.nbits && ((by >> (7 - (uint32_t)(x & 7))) & 1)) vv += b[i];
        }
        vs = wave_sum_dpp(vv);
        g1 = ci.ga;
        if (wiw && lane == 0) one_win<false>(a, f, inst, ci.ga, vs, ts, win1, dyn);
      } else {  // several attestations of this committee: direct atomics per attestation
        const uint32_t* co = catt_offs_ro + inst * (f.ncomm + 1);
        for (uint32_t k = co[it.z]; k < co[it.z + 1]; ++k) {
          const uint64_t ga = catt_ro[inst * a.natt + k];
          const uint64_t boff = boffs_ro[inst * a.natt + ga];
          const uint64_t nbits = 8 * (boffs_ro[inst * a.natt + ga + 1] - boff);
          const uint8_t* bf = a.bits + boff;
          uint64_t vv = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint64_t x = (uint64_t)(qs + i);
            if (v[i] && x < nbits && bit_at(bf, x)) vv += b[i];
          }
          vv = wave_sum_dpp(vv);
          if (wiw && lane == 0) one_win<false>(a, f, inst, (uint32_t)ga, vv, ts, f.att_win[inst * a.natt + ga], dyn);
          if (lane < 2) {
            uint64_t* dst = (lane ? a.vote : a.total) + inst * a.natt + ga;
            const uint64_t xx = lane ? vv : ts;
            if (xx) atomicAdd((unsigned long long*)dst, (unsigned long long)xx);
          }
        }
      }
    }
    // classify (validator.go:45-53; the saturated bounds classify exactly: d is below the
    // saturation value), reward (incentives.go:22-27), store, sum (core.go:459-464)
    const uint64_t d = a.dynasty[inst];
    const uint8_t* lastbf = a.bits + lb;
    const uint32_t ci4[4] = {cix.x, cix.y, cix.z, cix.w};
    bool act[4], off[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      act[i] = (uint64_t)sv[i] <= d && d < (uint64_t)ev[i];
      off[i] = v[i] && !act[i];
    }
    nm = wave_count4(off);  // (wave-uniform: the block end reads lane 0's)
    if (applied) {  // every validator active: rank == index, the validator at p is co_index[p]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool r = (MODE & 2) ? (b[i] & 1)
                       : (MODE & 256) ? ((lcw >> ((p + i) & 31)) & 1) : bit_at(lastbf, v[i] ? ci4[i] : 0u);
        b[i] = r ? b[i] + PZ_ATTESTER_REWARD : b[i] - PZ_ATTESTER_REWARD;
      }
      if (MODE & 4) {  // (ablation: no balance store)
      } else if (B32) {  // the offsets back: (base + o +- 1) - base = o +- 1, inside u32 (the state's re-base bound)
        if (v[0] && v[1] && v[2] && v[3]) {
          *reinterpret_cast<uint4*>(Bal32 + p) = make_uint4((uint32_t)(b[0] - bbase), (uint32_t)(b[1] - bbase),
                                                            (uint32_t)(b[2] - bbase), (uint32_t)(b[3] - bbase));
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (v[i]) Bal32[p + i] = (uint32_t)(b[i] - bbase);
        }
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = 2 * h;
          if (v[i] && v[i + 1])
            *reinterpret_cast<uint4*>(Bal + p + i) =
                make_uint4((uint32_t)b[i], (uint32_t)(b[i] >> 32), (uint32_t)b[i + 1], (uint32_t)(b[i + 1] >> 32));
          else if (v[i])
            Bal[p + i] = b[i];
          else if (v[i + 1])
            Bal[p + i + 1] = b[i + 1];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) sum += (v[i] && act[i]) ? b[i] : 0;
    sum = wave_sum_dpp(sum);
  } else {
    // {first position, count, committee, committee start}
    // (ablation 64: the piece computed from its index -- 256 positions, wrong tallies -- so the
    // stream loads do not wait for the item load)
    const uint4 it = (MODE & 64) ? make_uint4((uint32_t)(a.val_offset + ((item * 256) % (a.nval & ~255ull ? a.nval & ~255ull : 256))),
                                              have ? 256u : 0u, 0, (uint32_t)a.val_offset)
                     : have ? items_ro[item] : make_uint4((uint32_t)a.val_offset, 0, 0, (uint32_t)a.val_offset);
    const uint64_t ws = it.x, we = (uint64_t)it.x + it.y, cb = it.w;
    FusedCommittee ci;  // loaded beside the item: no dependent hop before the stream loads
    {
      const uint4 ic = have ? f.items_ci[inst * f.nitems + item] : make_uint4(0, 0, 0, kNoAtt);
      ci.boff = pack64(ic.x, ic.y);
      ci.nbits = ic.z;
      ci.ga = ic.w;
    }
    // (one launch, winners in the waves: the single attestation's shard and record dynasty,
    // loaded with the stream below rather than after the tallies)
    const bool wiw = PRO ? f.win_in_wave != 0 : f.win_fused != 0;
    const uint2 win1 = (wiw && ci.ga < kNoAtt) ? f.att_win[inst * a.natt + ci.ga] : make_uint2(0, 0);
    // ONE, a committee with several attestations: the first two entries of its catt range
    // (FusedArgs.one_ck / one_cw) go out with the stream, the bitfields are read from LDS
    constexpr int kCk = 2;
    uint4 ck[kCk];
    uint2 cw[kCk];
    // (issued by every wave of the single launch, entry 0 when its committee has one: a load
    // under the branch would go out only after the count's barrier, a round trip late)
    const bool ckt = ONE && ci.ga == kManyAtt;  // (wave-uniform; the single launch always sets one_ck)
    const uint32_t ck0 = (uint32_t)ci.boff, ck1 = (uint32_t)(ci.boff >> 32);
#pragma unroll
    for (int u = 0; u < kCk; ++u) {
      const uint32_t k = ckt ? min(ck0 + (uint32_t)u, ck1 - 1) : 0u;
      ck[u] = ONE ? f.one_ck[k] : make_uint4(0, 0, 0, 0);
      cw[u] = ONE ? f.one_cw[k] : make_uint2(0, 0);
    }
    const uint64_t p0 = (ws - a.val_offset) & ~1ull;  // local and even: the 16-B pair of ws
    uint64_t* Bal = a.balance + inst * f.vstride;
    const uint64_t* S = a.start + inst * f.vstride;
    const uint64_t* E = a.end + inst * f.vstride;
    uint4 qb[2], qs[2], qe[2];
    uint2 cix[2];
    uint32_t lcw_[2];  // f.lastco: the words holding the pair's reward bits
    uint32_t by0[2], by1[2];  // the committee bitfield bytes holding each element's bit
    bool v0[2], v1[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint64_t p = p0 + (uint64_t)j * 128 + 2 * lane, g = a.val_offset + p;
      v0[j] = g >= ws && g < we;
      v1[j] = g + 1 >= ws && g + 1 < we;
      const uint64_t pp = (v0[j] || v1[j]) ? p : p0;
      qb[j] = *reinterpret_cast<const uint4*>(Bal + pp);
      if (MODE & 16384) {  // 16-bit saturated {start | end << 16}: one 8-B load for the pair
        const uint2 w = ld8_nt(f.se16 + inst * f.vstride + pp);
        qs[j] = make_uint4(w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16);
        qe[j] = make_uint4(0, 0, 0, 0);
      } else if (MODE & 1024) {  // {start, end} of the pair's two validators, 32-bit saturated: one 16-B load
        qs[j] = ld16_nt(reinterpret_cast<const uint64_t*>(f.se + inst * f.vstride + pp));
        qe[j] = make_uint4(0, 0, 0, 0);
      } else if (MODE & 8) {
        qs[j] = make_uint4(0, 0, 0, 0);
        qe[j] = make_uint4(~0u, ~0u, ~0u, ~0u);
      } else if (MODE & 16) {
        qs[j] = *reinterpret_cast<const uint4*>(S + pp);
        qe[j] = *reinterpret_cast<const uint4*>(E + pp);
      } else {
        qs[j] = ld16_nt(S + pp);
        qe[j] = ld16_nt(E + pp);
      }
      if (MODE & 256) {  // compile-time: a runtime branch here split the load batch
        lcw_[j] = f.lastco[inst * f.lcw + (pp >> 5)];
        cix[j] = make_uint2(0, 0);
      } else {
        lcw_[j] = 0;
        cix[j] = (MODE & 2) ? make_uint2(0, 0) : *reinterpret_cast<const uint2*>(a.co_index + pp);
      }
      // branch-free, clamped: issued with the stream loads (bits past the bitfield are masked
      // below; the pre pass has raised that panic)
      by0[j] = by1[j] = 0;
      if (!PRO && !(MODE & 1) && ci.ga < kNoAtt && ci.nbits) {  // (PRO: from LDS, below)
        const uint64_t q = g - cb, last = ci.nbits - 1;
        by0[j] = a.bits[ci.boff + ((q < last ? q : last) >> 3)];
        by1[j] = a.bits[ci.boff + ((q + 1 < last ? q + 1 : last) >> 3)];
      }
    }
    if (TRc) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tst[1] = __builtin_amdgcn_s_memrealtime();
    }
    if (PRO) {  // the block's bit count and length checks -> threshold (no other block involved)
      __shared__ uint64_t xp[kFusedWaves], xe[kFusedWaves];
      uint64_t c = 0, e = 0;
#pragma unroll
      for (int k = 0; k < kOneLoads; ++k) {
        const uint64_t u = pbase + 16ull * ((uint64_t)k * 64 * kFusedWaves + tid);
        if (u + 16 <= pbeg || u >= pend) continue;
        const uint32_t w[4] = {pq[k].x, pq[k].y, pq[k].z, pq[k].w};
        if (u >= pbeg && u + 16 <= pend) {  // (a chunk inside the region: no byte masks)
          c += __popc(w[0]) + __popc(w[1]) + __popc(w[2]) + __popc(w[3]);
          continue;
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) {  // bytes of [pbeg, pend) only
          uint32_t m = 0xFFFFFFFFu;
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const uint64_t at = u + 4 * d + b;
            if (at < pbeg || at >= pend) m &= ~(0xFFu << (8 * b));
          }
          c += __popc(w[d] & m);
        }
      }
#pragma unroll
      for (int k = 0; k < kOneAtts; ++k) {
        const uint64_t g = (uint64_t)k * 64 * kFusedWaves + tid;
        if (g < a.natt && ocs[k] > 8 * (ob1[k] - ob0[k])) e = 1;
      }
#pragma unroll
      for (int k = 0; k < kOneLoads; ++k)
        if ((uint32_t)k < nlr) lbits[k * 64 * kFusedWaves + tid] = pq[k];
      c = wave_sum_dpp(c);
      e = wave_sum_dpp(e);
      if (lane == 0) {
        xp[wave] = c;
        xe[wave] = e;
      }
      __syncthreads();
      if (TRc) tst[2] = __builtin_amdgcn_s_memrealtime();
      // (the several-attestation entries used here, on every path: their loads stay ahead of
      // the barrier -- left to the compiler they sank into the branch that reads them, one
      // round trip per attestation after it, 1.7 us for two)
      if (ONE)
        asm volatile("" ::"v"(ck[0].x), "v"(ck[0].y), "v"(ck[0].z), "v"(ck[1].x), "v"(ck[1].y), "v"(ck[1].z),
                     "v"(cw[0].x), "v"(cw[0].y), "v"(cw[1].x), "v"(cw[1].y));
      uint64_t pc = 0, pe = 0;
#pragma unroll
      for (int w = 0; w < kFusedWaves; ++w) {
        pc += xp[w];
        pe += xe[w];
      }
      pop = pc;
      ferr = pe ? (uint64_t)kErrBitfield : 0;
      thr = (pop * PZ_DEFAULT_BALANCE * 3ull) >= (tdep_ro[inst] * 2ull);
      skip = ferr != 0 || (thr && rwd_err);
      applied = thr && !skip;
      if (!(MODE & 1) && ci.ga < kNoAtt && ci.nbits) {  // the committee's bitfield bytes, staged above
        const uint8_t* lb8 = reinterpret_cast<const uint8_t*>(lbits) + (ci.boff - pbase);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const uint64_t q = a.val_offset + p0 + (uint64_t)j * 128 + 2 * lane - cb, last = ci.nbits - 1;
          by0[j] = lb8[(q < last ? q : last) >> 3];
          by1[j] = lb8[(q + 1 < last ? q + 1 : last) >> 3];
        }
      }
    }
    // crosslink tallies on the pre-reward balances (core.go:533-545): position g of the
    // committee is bit g - cb of each of its attestations' bitfields
    if (!(MODE & 1) && ci.ga != kNoAtt) {
      uint64_t t = 0;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        t += (v0[j] ? pack64(qb[j].x, qb[j].y) : 0) + (v1[j] ? pack64(qb[j].z, qb[j].w) : 0);
      ts = wave_sum_dpp(t);
      if (ci.ga != kManyAtt) {
        uint64_t v = 0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const uint64_t q = a.val_offset + p0 + (uint64_t)j * 128 + 2 * lane - cb;
          if (v0[j] && q < ci.nbits && ((by0[j] >> (7 - (uint32_t)(q & 7))) & 1)) v += pack64(qb[j].x, qb[j].y);
          if (v1[j] && q + 1 < ci.nbits && ((by1[j] >> (7 - (uint32_t)((q + 1) & 7))) & 1))
            v += pack64(qb[j].z, qb[j].w);
        }
        vs = wave_sum_dpp(v);
        g1 = ci.ga;
        if (wiw && lane == 0) one_win<PRO>(a, f, inst, ci.ga, vs, ts, win1, dyn);
      } else if (ckt) {  // several attestations, ONE: the table's entries, bitfields in LDS
        const uint8_t* l8 = reinterpret_cast<const uint8_t*>(lbits);
        const uint64_t tk0 = TRc ? __builtin_amdgcn_s_memrealtime() : 0;
        // the vote sums of attestation k: its bits from the block's LDS copy
        // (branch-free: every lane reads its bytes, clamped into the bitfield, then masks -- the
        // reads under the validity tests each waited alone)
        auto vote_of = [&](const uint4& e) {
          const uint8_t* bf = l8 + e.x;
          const uint64_t nbits = e.y, last = nbits ? nbits - 1 : 0;
          uint32_t b0[2], b1[2];
          uint64_t qj[2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            qj[j] = a.val_offset + p0 + (uint64_t)j * 128 + 2 * lane - cb;
            b0[j] = bf[(qj[j] < last ? qj[j] : last) >> 3];
            b1[j] = bf[(qj[j] + 1 < last ? qj[j] + 1 : last) >> 3];
          }
          uint64_t v = 0;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const uint64_t q = qj[j];
            const bool x0 = v0[j] && q < nbits && ((b0[j] >> (7 - (uint32_t)(q & 7))) & 1);
            const bool x1 = v1[j] && q + 1 < nbits && ((b1[j] >> (7 - (uint32_t)((q + 1) & 7))) & 1);
            v += (x0 ? pack64(qb[j].x, qb[j].y) : 0) + (x1 ? pack64(qb[j].z, qb[j].w) : 0);
          }
          return v;
        };
        auto tally_of = [&](const uint4& e, const uint2& wn, uint64_t v) {
          if (wiw && lane == 0) one_win<PRO>(a, f, inst, e.z, v, ts, wn, dyn);
          if (lane < 2) {  // one instruction: lane 0 the total, lane 1 the vote
            uint64_t* dst = (lane ? a.vote : a.total) + inst * a.natt + e.z;
            const uint64_t x = lane ? v : ts;
            if (x) atomicAdd((unsigned long long*)dst, (unsigned long long)x);
          }
        };
        // the two preloaded entries together (both sums in flight at once), then any others
        const bool two = ck1 - ck0 >= 2;  // (wave-uniform; a committee here has at least two)
        uint64_t va = vote_of(ck[0]), vb = two ? vote_of(ck[1]) : 0;
        va = wave_sum_dpp(va);
        vb = wave_sum_dpp(vb);
        if (TRc && lane == 0) f.trace[8 * (uint64_t)(blockIdx.x * gridDim.y + blockIdx.y) + 7] = __builtin_amdgcn_s_memrealtime() - tk0;
        tally_of(ck[0], cw[0], va);
        if (two) tally_of(ck[1], cw[1], vb);
        for (uint32_t k = ck0 + kCk; k < ck1; ++k) {  // (wave-uniform)
          const uint4 e = f.one_ck[k];
          tally_of(e, f.one_cw[k], wave_sum_dpp(vote_of(e)));
        }
        if (TRc && lane == 0) f.trace[8 * (uint64_t)(blockIdx.x * gridDim.y + blockIdx.y) + 6] = __builtin_amdgcn_s_memrealtime() - tk0;
      } else {  // several attestations of this committee: direct atomics per attestation
        const uint32_t* co = catt_offs_ro + inst * (f.ncomm + 1);
        for (uint32_t k = co[it.z]; k < co[it.z + 1]; ++k) {
          const uint64_t ga = catt_ro[inst * a.natt + k];
          const uint64_t boff = boffs_ro[inst * a.natt + ga];
          const uint64_t nbits = 8 * (boffs_ro[inst * a.natt + ga + 1] - boff);
          const uint8_t* bf = a.bits + boff;
          uint64_t v = 0;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const uint64_t q = a.val_offset + p0 + (uint64_t)j * 128 + 2 * lane - cb;
            if (v0[j] && q < nbits && bit_at(bf, q)) v += pack64(qb[j].x, qb[j].y);
            if (v1[j] && q + 1 < nbits && bit_at(bf, q + 1)) v += pack64(qb[j].z, qb[j].w);
          }
          v = wave_sum_dpp(v);
          if (wiw && lane == 0) one_win<PRO>(a, f, inst, (uint32_t)ga, v, ts, f.att_win[inst * a.natt + ga], dyn);
          if (lane < 2) {  // one instruction: lane 0 the total, lane 1 the vote
            uint64_t* dst = (lane ? a.vote : a.total) + inst * a.natt + ga;
            const uint64_t x = lane ? v : ts;
            if (x) atomicAdd((unsigned long long*)dst, (unsigned long long)x);
          }
        }
      }
    }
    // classify (validator.go:45-53), reward (incentives.go:22-27), store, sum (core.go:459-464)
    const uint64_t d = a.dynasty[inst];
    const uint8_t* lastbf = PRO ? reinterpret_cast<const uint8_t*>(lbits) + (lb - pbase) : a.bits + lb;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint64_t p = p0 + (uint64_t)j * 128 + 2 * lane;
      uint64_t b0 = pack64(qb[j].x, qb[j].y), b1 = pack64(qb[j].z, qb[j].w);
      // (MODE & 1024: d < 2^32 - 1, so the saturated 32-bit bounds classify exactly)
      const bool a0 = (MODE & 1024) ? ((uint64_t)qs[j].x <= d && d < (uint64_t)qs[j].y)
                                    : (pack64(qs[j].x, qs[j].y) <= d && d < pack64(qe[j].x, qe[j].y));
      const bool a1 = (MODE & 1024) ? ((uint64_t)qs[j].z <= d && d < (uint64_t)qs[j].w)
                                    : (pack64(qs[j].z, qs[j].w) <= d && d < pack64(qe[j].z, qe[j].w));
      nm += (v0[j] && !a0 ? 1 : 0) + (v1[j] && !a1 ? 1 : 0);
      if (applied) {  // every validator active: rank == index, the validator at p is co_index[p]
        // an element outside the piece looks up bit 0 (its co_index may be a row's pad)
        const bool r0 = (MODE & 2) ? (b0 & 1)
                        : (MODE & 256) ? ((lcw_[j] >> (p & 31)) & 1)
                                       : bit_at(lastbf, v0[j] ? cix[j].x : 0u);
        const bool r1 = (MODE & 2) ? (b1 & 1)
                        : (MODE & 256) ? ((lcw_[j] >> ((p + 1) & 31)) & 1)
                                       : bit_at(lastbf, v1[j] ? cix[j].y : 0u);
        b0 = r0 ? b0 + PZ_ATTESTER_REWARD : b0 - PZ_ATTESTER_REWARD;
        b1 = r1 ? b1 + PZ_ATTESTER_REWARD : b1 - PZ_ATTESTER_REWARD;
        if (MODE & 4)
          ;
        else if (v0[j] && v1[j])
          *reinterpret_cast<uint4*>(Bal + p) =
              make_uint4((uint32_t)b0, (uint32_t)(b0 >> 32), (uint32_t)b1, (uint32_t)(b1 >> 32));
        else if (v0[j])
          Bal[p] = b0;
        else if (v1[j])
          Bal[p + 1] = b1;
      }
      sum += (v0[j] && a0 ? b0 : 0) + (v1[j] && a1 ? b1 : 0);
    }
  }
  if constexpr ((MODE & 32768) == 0) {  // (the quad path summed them above)
    sum = wave_sum_dpp(sum);
    nm = wave_sum_dpp(nm);
  }
  if (lane == 0) {
    xg[wave] = g1;
    xt[wave] = ts;
    xv[wave] = vs;
    xs[wave] = sum;
    xn[wave] = nm;
  }
  __syncthreads();
  if (TRc) tst[3] = __builtin_amdgcn_s_memrealtime();
  if (!PRO && wave != 0) return;
  if (wave == 0) fused_block_end(a, f, xg, xt, xv, xs, xn, inst, grp, lane, skip, applied, pop, ferr, rwd_err);
  if (PRO && f.win_in_wave) {  // the next step's winners start empty (this step's are in a.winner)
    for (uint32_t r = (uint32_t)(grp * blockDim.x) + tid; r < a.nrec; r += gridDim.y * blockDim.x)
      f.winner_next[inst * a.nrec + r] = 0xFFFFFFFFu;
  } else if (ONE) {
    one_tail(a, f, tid);
  }
  if (TRc && tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tst[4] = __builtin_amdgcn_s_memrealtime();
    uint64_t* t = f.trace + 8 * (uint64_t)(blockIdx.x * gridDim.y + blockIdx.y);
    for (int k = 0; k < 5; ++k) t[k] = tst[k];
    t[5] = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // XCC_ID
  }
}

// Wave 0 of a fused block: the block's tallies, next-cycle sum and per-instance scalars.
// E: the block's tally entries, in piece order (one per wave, or two for the two-piece waves).
template <int E>
__device__ __forceinline__ void fused_block_end(const EpochArgs& a, const FusedArgs& f, const uint32_t* xg,
                                                const uint64_t* xt, const uint64_t* xv, const uint64_t* xs,
                                                const uint64_t* xn, uint64_t inst, uint64_t grp, int lane,
                                                bool skip, bool applied, uint64_t pop, uint64_t ferr, bool rwd_err) {
  // Wave 0 adds the block's tallies: consecutive pieces of one committee are merged, and one
  // atomic instruction carries every total (lanes 0 .. E-1) and vote (lanes E .. 2E-1).
  static_assert((E & (E - 1)) == 0 && 2 * E <= 64, "entries: a power of two, two per lane at most");
  if (lane < 2 * E) {
    const int e = lane & (E - 1);
    const uint32_t g = xg[e];
    if (g < kNoAtt && (e == 0 || xg[e - 1] != g)) {  // head of a run of equal attestations
      uint64_t x = 0;
      for (int k = e; k < E && xg[k] == g; ++k) x += lane < E ? xt[k] : xv[k];
      uint64_t* dst = (lane < E ? a.total : a.vote) + inst * a.natt + g;
      if (x) atomicAdd((unsigned long long*)dst, (unsigned long long)x);
    }
  }
  uint64_t* sc = a.scal + inst * kScal;
  if (lane == 0) {
    uint64_t s = 0, nmt = 0;
    for (int w = 0; w < kFusedWaves; ++w) {
      s += xs[w];
      nmt += xn[w];
    }
    if (s && !skip) atomicAdd((unsigned long long*)&sc[kNextBal], (unsigned long long)s);
    if (nmt) {  // the layout's rank == index premise is broken (the state never allows it)
      atomicAdd((unsigned long long*)&sc[kNoMatch], (unsigned long long)nmt);
      atomicOr((unsigned long long*)&sc[kErrXl], (unsigned long long)kErrLayout);
    }
    if (grp == 0 && f.rank0) {
      sc[kPop] = pop;
      sc[kApplied] = applied ? 1 : 0;
      sc[kNact] = a.nval_global;
      sc[kMaxIdx1] = a.nval_global;
      sc[kErrRwd] = rwd_err ? 1 : 0;
      if (ferr) atomicAdd((unsigned long long*)&sc[kErrXl], (unsigned long long)ferr);
    }
  }
  if (grp == 0) {
    if (a.scal_next && lane < kScal) a.scal_next[inst * kScal + lane] = 0;
    if (lane < kPre) f.pre_next[inst * kPre + lane] = 0;
  }
}

// ONE: the arrival ticket, and in the last block to arrive the crosslink winners of the one
// instance (core.go:549-555: the first attestation, in order, whose 3*vote >= 2*total and whose
// dynasty beats the shard's record), formed in LDS from the complete tallies.  Hand-off
// (MI355X_MICROARCH.md, the table's first row): every wave drains its tally atomics
// (s_waitcnt vmcnt(0)) before the block barrier, one lane adds to ONE counter, the block whose
// add returns the last count reads the tallies with agent-scope (sc1) loads; the tallies are
// only ever written by agent-scope atomics and sc1 stores, so no L2 holds a stale copy.
__device__ __forceinline__ void one_tail(const EpochArgs& a, const FusedArgs& f, int tid) {
  __shared__ uint32_t last, wl[kOneMaxRec];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const uint32_t t = __hip_atomic_fetch_add(f.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x * gridDim.y - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last) return;
  const int nt = (int)blockDim.x;
  for (uint32_t r = tid; r < a.nrec; r += nt) wl[r] = 0xFFFFFFFFu;
  __syncthreads();
  const uint64_t d = a.dynasty[0];
  for (uint32_t g = tid; g < a.natt; g += nt) {
    const uint64_t v = __hip_atomic_load(&a.vote[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t = __hip_atomic_load(&a.total[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t shard = a.att_shard[g];  // < nrec: the host takes the one-pass step only then
    if (3ull * v >= 2ull * t && d > a.rec_dynasty[shard]) atomicMin(&wl[shard], g);
  }
  for (uint32_t g = tid; g < a.natt; g += nt) {  // the next step's tallies start from zero
    __hip_atomic_store(&f.vote_next[g], (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&f.total_next[g], (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  for (uint32_t r = tid; r < a.nrec; r += nt) a.winner[r] = wl[r];
  if (tid == 0) __hip_atomic_store(f.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The single-launch step (one instance): no occupancy target (a few dozen blocks), so the
// bit-count loads the prologue holds do not spill.
extern "C" __global__ void __launch_bounds__(64 * kFusedWaves)
pz_epoch_one_kernel(EpochArgs a, FusedArgs f, const uint64_t* __restrict__ boffs_ro,
                    const uint64_t* __restrict__ tdep_ro, const uint4* __restrict__ items_ro,
                    const FusedCommittee* __restrict__ cinfo_ro, const uint32_t* __restrict__ catt_offs_ro,
                    const uint32_t* __restrict__ catt_ro) {
  fused_body<512>(a, f, nullptr, boffs_ro, tdep_ro, items_ro, cinfo_ro, catt_offs_ro, catt_ro);
}
extern "C" __global__ void __launch_bounds__(64 * kFusedWaves)
pz_epoch_one_se_kernel(EpochArgs a, FusedArgs f, const uint64_t* __restrict__ boffs_ro,
                       const uint64_t* __restrict__ tdep_ro, const uint4* __restrict__ items_ro,
                       const FusedCommittee* __restrict__ cinfo_ro, const uint32_t* __restrict__ catt_offs_ro,
                       const uint32_t* __restrict__ catt_ro) {
  fused_body<512 + 1024>(a, f, nullptr, boffs_ro, tdep_ro, items_ro, cinfo_ro, catt_offs_ro, catt_ro);
}
extern "C" __global__ void __launch_bounds__(64 * kFusedWaves)
pz_epoch_one_se16_kernel(EpochArgs a, FusedArgs f, const uint64_t* __restrict__ boffs_ro,
                         const uint64_t* __restrict__ tdep_ro, const uint4* __restrict__ items_ro,
                         const FusedCommittee* __restrict__ cinfo_ro, const uint32_t* __restrict__ catt_offs_ro,
                         const uint32_t* __restrict__ catt_ro) {
  fused_body<512 + 1024 + 16384>(a, f, nullptr, boffs_ro, tdep_ro, items_ro, cinfo_ro, catt_offs_ro, catt_ro);
}
#ifdef PZ_AB_BUILD
// the same with phase stamps (FusedArgs.trace; tools/epoch_single.py)
extern "C" __global__ void __launch_bounds__(64 * kFusedWaves)
pz_epoch_one_se16_trace_kernel(EpochArgs a, FusedArgs f, const uint64_t* __restrict__ boffs_ro,
                               const uint64_t* __restrict__ tdep_ro, const uint4* __restrict__ items_ro,
                               const FusedCommittee* __restrict__ cinfo_ro, const uint32_t* __restrict__ catt_offs_ro,
                               const uint32_t* __restrict__ catt_ro) {
  fused_body<512 + 1024 + 16384 + (1 << 22)>(a, f, nullptr, boffs_ro, tdep_ro, items_ro, cinfo_ro, catt_offs_ro,
                                             catt_ro);
}
static uint64_t* g_one_trace = nullptr;
extern "C" void pz_debug_set_one_trace(uint64_t* d_trace) { g_one_trace = d_trace; }
#endif

// ---- launchers ---------------------------------------------------------------------------
static bool vec_ok(const EpochArgs& a) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return (a.nval % 2 == 0) && al(a.start) && al(a.end) && al(a.balance);
}

static CountGrid count_grid(const EpochArgs& a, bool do_val, bool do_pop, bool do_xl) {
  CountGrid g;
  g.vbpi = vblocks_per_inst(a.nval);
  g.nvb = do_val ? (uint64_t)a.ninst * g.vbpi : 0;
  g.pbpi = (a.max_inst_bytes + kPopBytesPerBlock - 1) / kPopBytesPerBlock;
  // The popcount range also resets the crosslink winners (chunk 0 of each instance), so it
  // keeps one block per instance whenever winners will be computed -- even when no bitfield
  // has a byte (every pending attestation names an empty committee, nval < 64) or when this
  // launch counts nothing but crosslinks.
  const bool reset = do_xl && a.winner && a.natt;
  if (reset && g.pbpi == 0) g.pbpi = 1;
  g.do_pop = do_pop ? 1 : 0;
  g.npb = ((do_pop || reset) && a.natt) ? (uint64_t)a.ninst * g.pbpi : 0;
  g.vec = vec_ok(a) ? 1 : 0;
  g.xl_j = ((uint64_t)a.natt + 3) / 4;
  g.xl_affine = a.ninst >= 8 ? 1 : 0;
  const uint64_t xl_inst = g.xl_affine ? ((uint64_t)a.ninst + 7) / 8 * 8 : a.ninst;
  g.nxb = (do_xl && a.natt) ? xl_inst * g.xl_j : 0;
  return g;
}

hipError_t launch_epoch_count(const EpochArgs& a, bool do_val, bool do_pop, bool do_xl, hipStream_t s) {
  const CountGrid g = count_grid(a, do_val, do_pop, do_xl);
  const uint64_t blocks = g.nvb + g.npb + g.nxb;
  if (!blocks) return hipSuccess;
  const dim3 grid((uint32_t)blocks);
  hipLaunchKernelGGL(pz_epoch_count_kernel, grid, dim3(kThreads), 0, s, a, g);
  return hipGetLastError();
}

#ifdef PZ_AB_BUILD
// A stateRecalc's vote-cache tally and its epoch's count pass in ONE launch (the chain
// engine, one rank): blocks [0, ntb) are the voter-major tally (votes_dev.h), the rest the
// count pass's blocks.  The two read the same pre-reward balances and write disjoint buffers; the
// tally blocks come first, so the walk's wait (their gathered totals) is not behind the count.
static_assert(kVoteWordThreads == kThreads, "one block shape for both parts");
extern "C" __global__ void __launch_bounds__(kThreads)
pz_vote_words_count_kernel(VoteWordArgs v, uint32_t ntb, EpochArgs a, CountGrid g) {
  if (blockIdx.x < ntb)
    vote_words_body(v, ntb, blockIdx.x);
  else
    count_body<0>(a, g, blockIdx.x - ntb);
}

hipError_t launch_vote_words_count(const VoteWordArgs& v, const EpochArgs& a, hipStream_t s) {
  const CountGrid g = count_grid(a, true, true, true);
  const uint32_t ntb = v.natt ? vote_word_blocks(v) : 0;
  const uint64_t blocks = ntb + g.nvb + g.npb + g.nxb;
  if (!blocks) return hipSuccess;
  hipLaunchKernelGGL(pz_vote_words_count_kernel, dim3((uint32_t)blocks), dim3(kThreads), 0, s, v, ntb, a, g);
  return hipGetLastError();
}

#endif

hipError_t launch_epoch_winners(const EpochArgs& a, hipStream_t s) {
  const uint64_t n = (uint64_t)a.ninst * a.natt;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(pz_epoch_winner_kernel, dim3((uint32_t)((n + kThreads - 1) / kThreads)), dim3(kThreads),
                     0, s, a);
  return hipGetLastError();
}

hipError_t launch_epoch_compact(const EpochArgs& a, bool force, hipStream_t s) {
  const uint64_t vbpi = vblocks_per_inst(a.nval);
  const uint64_t blocks = (uint64_t)a.ninst * vbpi;
  if (!blocks) return hipSuccess;
  hipLaunchKernelGGL(pz_epoch_compact_kernel, dim3((uint32_t)blocks), dim3(kThreads), 0, s, a, vbpi,
                     force ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_epoch_reward(const EpochArgs& a, hipStream_t s) {
  // at least one chunk per instance: chunk 0 also writes the per-instance scalars (applied,
  // active count) and zeroes the next step's, even for a rank whose range is empty
  const uint64_t vbpi = std::max<uint64_t>(1, vblocks_per_inst(a.nval));
  const uint64_t blocks = (uint64_t)a.ninst * vbpi;
  if (!blocks) return hipSuccess;
  hipLaunchKernelGGL(pz_epoch_reward_kernel, dim3(a.ninst, (uint32_t)vbpi), dim3(kThreads), 0, s, a, vbpi,
                     vec_ok(a) ? 1 : 0, a.scal, a.boffs, a.total_deposit);
  return hipGetLastError();
}

// The one-pass stream loads 16-B pairs at even local indices: the arrays must be 16-B aligned
// (an odd range's last pair reads the allocation's padding, and stores only its own element).
bool fused_ok(const EpochArgs& a) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return al(a.start) && al(a.end) && al(a.balance) && a.co_index && a.natt &&
         (reinterpret_cast<uintptr_t>(a.co_index) & 7) == 0;
}

bool epoch_one_enabled(const FusedArgs& f) { return f.one != 0; }

hipError_t launch_epoch_one(const EpochArgs& a, const FusedArgs& f, hipStream_t s) {
  const uint64_t groups = std::max<uint64_t>(1, (f.nitems + kFusedWaves - 1) / kFusedWaves);
#ifdef PZ_AB_BUILD
  if (g_one_trace && f.se16) {
    FusedArgs ft = f;
    ft.trace = g_one_trace;
    hipLaunchKernelGGL(pz_epoch_one_se16_trace_kernel, dim3(1, (uint32_t)groups), dim3(64 * kFusedWaves), 0, s, a, ft,
                       a.boffs, a.total_deposit, f.items, f.cinfo, f.catt_offs, f.catt);
    return hipGetLastError();
  }
#endif
  if (f.se16)
    hipLaunchKernelGGL(pz_epoch_one_se16_kernel, dim3(1, (uint32_t)groups), dim3(64 * kFusedWaves), 0, s, a, f,
                       a.boffs, a.total_deposit, f.items, f.cinfo, f.catt_offs, f.catt);
  else if (f.se)
    hipLaunchKernelGGL(pz_epoch_one_se_kernel, dim3(1, (uint32_t)groups), dim3(64 * kFusedWaves), 0, s, a, f, a.boffs,
                       a.total_deposit, f.items, f.cinfo, f.catt_offs, f.catt);
  else
    hipLaunchKernelGGL(pz_epoch_one_kernel, dim3(1, (uint32_t)groups), dim3(64 * kFusedWaves), 0, s, a, f, a.boffs,
                       a.total_deposit, f.items, f.cinfo, f.catt_offs, f.catt);
  return hipGetLastError();
}

hipError_t launch_epoch_mid(const EpochArgs& a, bool winners, bool compact, hipStream_t s) {
  const uint64_t vbpi = vblocks_per_inst(a.nval);
  const uint64_t n = winners ? (uint64_t)a.ninst * a.natt : 0;
  const uint64_t nwb = (n + kThreads - 1) / kThreads;
  const uint64_t ncb = compact ? (uint64_t)a.ninst * vbpi : 0;
  if (!(nwb + ncb)) return hipSuccess;
  hipLaunchKernelGGL(pz_epoch_mid_kernel, dim3((uint32_t)(nwb + ncb)), dim3(kThreads), 0, s, a, vbpi, nwb,
                     compact ? 1 : 0);
  return hipGetLastError();
}

}  // namespace pz
