// Block vote-cache tally (blockchain/core.go:300-345 calculateBlockVoteCache) for gfx950.
//
// The reference keeps, per signed parent hash h, the list of validators that voted for h
// (deduplicated by a linear scan, O(k^2)) and VoteTotalDeposit += balance of each newly
// seen voter.  Here each hash h has a dense slot id (assigned by the host) owning an
// nval-bit dedup bitmap in HBM.  Work item = (attestation, slot): one wave walks the
// attestation's committee; a set bitfield bit does atomicOr on the voter's bitmap word and
// the lanes whose bit was newly set add the voter's balance.  Set union and uint64 sums
// commute, so a whole cycle of blocks is one launch and the totals are bit-exact with the
// sequential Go loop (VoterIndices' insertion order is never serialized).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "../../include/prysm_hip.h"
#include "votes.h"
#include "votes_dev.h"

namespace pz {

extern "C" __global__ void __launch_bounds__(256)
pz_vote_tally_kernel(VoteArgs a) {
  const uint64_t item = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (item >= a.nitems) return;
  const uint32_t att = a.item_att[item];
  const uint32_t slot = a.item_slot[item];
  const uint64_t bb = a.boffs[att];
  tally_item(a.committee, a.coffs, a.att_comm[att], a.bits + bb, a.boffs[att + 1] - bb, a.balance, a.nval,
             a.bitmaps + (uint64_t)slot * a.words_per_slot, a.totals + slot, a.err, a.val_offset, a.nval_global);
}

// The block engine's form (votes.h VoteWordArgs): voter-major, one wave per (attestation,
// 256-member chunk), every signed parent hash of the attestation in one pass.  Round 3's form
// (an item per (attestation, parent): a union pass ORing each item's bitfield into its (slot,
// committee) group, then a leader pass tallying each group with one atomic per voter and
// parent) took 7.6 + 22 us per stateRecalc flush at 65,536 validators
// (profiles/r04/replay_kernels_r4h.txt), 64 atomics per voter where this takes one or two.
extern "C" __global__ void __launch_bounds__(kVoteWordMaxThreads)
pz_vote_words_kernel(VoteWordArgs a) { vote_words_body(a, gridDim.x, blockIdx.x); }

// Waves per block of the per-attestation form (16: more of the flush's totals summed in LDS
// before the device atomics; 4, 8 and 16 measured level, profiles/r04/replay_ab_vote_waves_r4u.txt).
static uint32_t vote_word_threads() { return 16 * 64; }

hipError_t launch_vote_words(const VoteWordArgs& a, hipStream_t s) {
  if (!a.natt) return hipSuccess;
  const uint32_t t = a.ngroups ? kVoteWordThreads : vote_word_threads();
  hipLaunchKernelGGL(pz_vote_words_kernel, dim3(vote_word_blocks(a, t)), dim3(t), 0, s, a);
  return hipGetLastError();
}

#ifdef PZ_AB_BUILD
extern "C" __global__ void __launch_bounds__(kVoteWordMaxThreads)
pz_vote_words_traced_kernel(VoteWordArgs a, uint64_t* tr) { vote_words_body(a, gridDim.x, blockIdx.x, tr); }

hipError_t launch_vote_words_traced(const VoteWordArgs& a, uint64_t* tr, hipStream_t s) {
  if (!a.natt) return hipSuccess;
  const uint32_t t = a.ngroups ? kVoteWordThreads : vote_word_threads();
  hipLaunchKernelGGL(pz_vote_words_traced_kernel, dim3(vote_word_blocks(a, t)), dim3(t), 0, s, a, tr);
  return hipGetLastError();
}

#endif

extern "C" __global__ void __launch_bounds__(256)
pz_stage_h2d_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

#ifdef PZ_AB_BUILD
// Several segments in one launch: block y copies segment y (grid-stride over x).
extern "C" __global__ void __launch_bounds__(256)
pz_stage_h2d_segs_kernel(StageSegs g) {
  const StageSeg& sg = g.seg[blockIdx.y];
  const uint4* __restrict__ src = static_cast<const uint4*>(sg.src);
  uint4* __restrict__ dst = static_cast<uint4*>(sg.dst);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < sg.n16; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

hipError_t launch_stage_h2d_segs(const StageSegs& g, hipStream_t s) {
  uint64_t mx = 0;
  for (int k = 0; k < g.nseg; ++k) mx = std::max(mx, g.seg[k].n16);
  if (!mx || !g.nseg) return hipSuccess;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((mx + 255) / 256, 256);
  hipLaunchKernelGGL(pz_stage_h2d_segs_kernel, dim3(blocks, (uint32_t)g.nseg), dim3(256), 0, s, g);
  return hipGetLastError();
}

#endif

hipError_t launch_stage_h2d(const void* host_mapped, void* dev, uint64_t bytes, hipStream_t s) {
  const uint64_t n16 = bytes / 16;
  if (!n16) return hipSuccess;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((n16 + 255) / 256, 1024);
  hipLaunchKernelGGL(pz_stage_h2d_kernel, dim3(blocks), dim3(256), 0, s, static_cast<const uint4*>(host_mapped),
                     static_cast<uint4*>(dev), n16);
  return hipGetLastError();
}

extern "C" __global__ void __launch_bounds__(64)
pz_vote_gather_kernel(const uint64_t* __restrict__ totals, VoteGatherSlots q, const uint64_t* __restrict__ err,
                      uint64_t* __restrict__ out) {
  const int j = threadIdx.x;
  const uint32_t sl = q.slot[j];
  out[j] = sl == 0xFFFFFFFFu ? 0 : totals[sl];
  if (j == 0) out[kJustifySlots] = err ? *err : 0;
}

hipError_t launch_vote_gather(const uint64_t* totals, VoteGatherSlots slots, const uint64_t* err, uint64_t* out,
                              hipStream_t s) {
  hipLaunchKernelGGL(pz_vote_gather_kernel, dim3(1), dim3(kJustifySlots), 0, s, totals, slots, err, out);
  return hipGetLastError();
}

hipError_t launch_vote_tally(const VoteArgs& a, hipStream_t s) {
  if (!a.nitems) return hipSuccess;
  const uint64_t threads = a.nitems * 64;
  hipLaunchKernelGGL(pz_vote_tally_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace pz
