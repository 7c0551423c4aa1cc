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

#include "../../include/prysm_hip.h"
#include "epoch.h"

namespace pz {

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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
struct CountGrid {
  uint64_t vbpi, nvb, pbpi, npb, nxb;
  uint64_t xl_j;      // crosslink blocks per instance (4 attestations per block)
  int xl_affine;      // 1: crosslink blocks of instance i land on XCD i % 8 (>= 8 instances)
};

// Crosslink tally for one attestation, one wave (core.go:533-545).  Members are processed
// 256 at a time with every committee load, then every balance gather, in flight together
// (two dependent round trips per 256 members instead of two per 64).
__device__ __forceinline__ void crosslink_wave(const EpochArgs& a, uint64_t ga, int lane) {
  const uint64_t inst = ga / a.natt;
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
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t i = r0 + j * 64 + lane;
      byte[j] = (i < k && i < 8 * blen) ? bf[i >> 3] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t i = r0 + j * 64 + lane;
      const uint64_t local = (uint64_t)mem[j] - a.val_offset;  // wraps huge when mem < val_offset
      const bool own = i < k && mem[j] < a.nval_global && local < a.nval;
      bal[j] = own ? B[local] : 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t i = r0 + j * 64 + lane;
      if (i < k) {
        e_mem |= mem[j] >= a.nval_global;
        e_bf |= i >= 8 * blen;
        tot += bal[j];
        vote += ((byte[j] >> (7 - (uint32_t)(i & 7))) & 1u) ? bal[j] : 0;
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

extern "C" __global__ void __launch_bounds__(kThreads)
pz_epoch_count_kernel(EpochArgs a, CountGrid g) {
  __shared__ uint64_t sh[kThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // Grid order: [crosslink blocks | validator blocks | popcount blocks].  The latency-bound
  // gathers start first and overlap the streaming blocks behind them.
  if (blockIdx.x < g.nxb) {
    const uint64_t x = blockIdx.x;
    uint64_t inst, j;
    if (g.xl_affine) {  // blocks x and x+8 share an XCD: keep one instance's balances in one L2
      const uint64_t qj = x >> 3;
      inst = (qj / g.xl_j) * 8 + (x & 7);
      j = qj % g.xl_j;
    } else {
      inst = x / g.xl_j;
      j = x % g.xl_j;
    }
    const uint64_t att = j * (kThreads / 64) + wave;
    if (inst >= a.ninst || att >= a.natt) return;
    crosslink_wave(a, inst * a.natt + att, lane);
    return;
  }
  const uint64_t b = blockIdx.x - g.nxb;

  if (b < g.nvb) {  // ---- classify + count + active mask + max active index
    const uint64_t inst = b / g.vbpi, chunk = b % g.vbpi;
    const uint64_t base = chunk * kValPerBlock;
    const uint64_t d = a.dynasty[inst];
    const uint64_t* S = a.start + inst * a.nval;
    const uint64_t* E = a.end + inst * a.nval;
    uint64_t* mask = a.act_mask ? a.act_mask + inst * ((a.nval + 63) / 64) : nullptr;
    uint32_t cnt = 0;
    uint64_t maxi1 = 0;
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
    uint64_t c = block_reduce<false>(lane == 0 ? cnt : 0, sh);
    uint64_t m = block_reduce<true>(maxi1, sh);
    if (tid == 0) {
      if (a.blk_cnt) a.blk_cnt[inst * g.vbpi + chunk] = (uint32_t)c;
      if (c) atomicAdd((unsigned long long*)&a.scal[inst * kScal + kNact], (unsigned long long)c);
      if (m) atomicMax((unsigned long long*)&a.scal[inst * kScal + kMaxIdx1], (unsigned long long)m);
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
    const uint64_t inst = pb / g.pbpi, chunk = pb % g.pbpi;
    if (chunk % a.pop_world != a.pop_rank) return;
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

// ------------------------------------------------------------------------------------------
// Crosslink winners (core.go:549-555): the first attestation, in order, whose 3*vote >=
// 2*total and whose dynasty beats the shard's record wins that shard (atomicMin of index).
// ------------------------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(kThreads) pz_epoch_winner_kernel(EpochArgs a) {
  const uint64_t ga = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ga >= (uint64_t)a.ninst * a.natt) return;
  const uint64_t inst = ga / a.natt;
  const uint64_t v = a.vote[ga], t = a.total[ga];
  if (3ull * v >= 2ull * t) {  // uint64 wrap, as in Go
    const uint32_t shard = a.att_shard[ga];
    if (shard >= a.nrec) {
      atomicAdd((unsigned long long*)&a.scal[inst * kScal + kErrXl], (unsigned long long)kErrShard);
      return;
    }
    if (a.dynasty[inst] > a.rec_dynasty[inst * a.nrec + shard])
      atomicMin(&a.winner[inst * a.nrec + shard], (uint32_t)(ga - inst * a.natt));
  }
}

// ------------------------------------------------------------------------------------------
// General rank path: compacted active list act_list[inst][rank] = global index.
// ------------------------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(kThreads)
pz_epoch_compact_kernel(EpochArgs a, uint64_t vbpi, int force) {
  __shared__ uint32_t wsum[kThreads / 64 * kValPerThread];
  __shared__ uint64_t base_off;
  const uint64_t inst = blockIdx.x / vbpi, chunk = blockIdx.x % vbpi;
  const uint64_t nact = a.scal[inst * kScal + kNact];
  if (!force && nact == a.nval) return;  // rank == index: nothing to compact
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

// ------------------------------------------------------------------------------------------
// Pass 2: CalculateRewards (incentives.go:14-32) fused with the next-cycle balance sum
// (core.go:459-464).  Position p receives +-1 by CheckBit(last bitfield, active[p]).
// ------------------------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(kThreads) pz_epoch_reward_kernel(EpochArgs a, uint64_t vbpi) {
  __shared__ uint64_t sh[kThreads / 64];
  const uint64_t inst = blockIdx.x / vbpi, chunk = blockIdx.x % vbpi;
  const int tid = threadIdx.x;
  const uint64_t* sc = a.scal + inst * kScal;
  const uint64_t pop = sc[kPop], nact = sc[kNact];
  const bool xl_err = sc[kErrXl] != 0;
  const uint64_t dep = pop * PZ_DEFAULT_BALANCE;                 // GetAttestersTotalDeposit
  const bool applied = (dep * 3ull) >= (a.total_deposit[inst] * 2ull);  // uint64 wrap
  const bool rwd_err = applied && nact > 0 && sc[kErrRwd] != 0;
  if (xl_err || rwd_err) {  // Go panics before/while rewarding: leave balances untouched
    if (blockIdx.x % vbpi == 0 && tid == 0) a.scal[inst * kScal + kApplied] = 0;
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
      const uint64_t idx = all_active ? gp : list[gp];
      bal = bit_at(lastbf, idx) ? bal + PZ_ATTESTER_REWARD : bal - PZ_ATTESTER_REWARD;
      B[p] = bal;
    }
    const bool act = all_active ? true : ((mask[p >> 6] >> (p & 63)) & 1);
    if (act) sum += bal;
  }
  uint64_t s = block_reduce<false>(sum, sh);
  if (tid == 0) {
    if (s) atomicAdd((unsigned long long*)&a.scal[inst * kScal + kNextBal], (unsigned long long)s);
    if (chunk == 0) a.scal[inst * kScal + kApplied] = applied ? 1 : 0;
  }
}

// ---- launchers ---------------------------------------------------------------------------
hipError_t launch_epoch_count(const EpochArgs& a, bool do_val, bool do_pop, bool do_xl, hipStream_t s) {
  CountGrid g;
  g.vbpi = vblocks_per_inst(a.nval);
  g.nvb = do_val ? (uint64_t)a.ninst * g.vbpi : 0;
  g.pbpi = (a.max_inst_bytes + kPopBytesPerBlock - 1) / kPopBytesPerBlock;
  g.npb = (do_pop && a.natt) ? (uint64_t)a.ninst * g.pbpi : 0;
  g.xl_j = ((uint64_t)a.natt + 3) / 4;
  g.xl_affine = a.ninst >= 8 ? 1 : 0;
  const uint64_t xl_inst = g.xl_affine ? ((uint64_t)a.ninst + 7) / 8 * 8 : a.ninst;
  g.nxb = (do_xl && a.natt) ? xl_inst * g.xl_j : 0;
  const uint64_t blocks = g.nvb + g.npb + g.nxb;
  if (!blocks) return hipSuccess;
  hipLaunchKernelGGL(pz_epoch_count_kernel, dim3((uint32_t)blocks), dim3(kThreads), 0, s, a, g);
  return hipGetLastError();
}

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
  const uint64_t vbpi = vblocks_per_inst(a.nval);
  const uint64_t blocks = (uint64_t)a.ninst * vbpi;
  if (!blocks) return hipSuccess;
  hipLaunchKernelGGL(pz_epoch_reward_kernel, dim3((uint32_t)blocks), dim3(kThreads), 0, s, a, vbpi);
  return hipGetLastError();
}

}  // namespace pz
