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

#include "../../include/prysm_hip.h"
#include "votes.h"

namespace pz {

__device__ __forceinline__ uint64_t wsum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

extern "C" __global__ void __launch_bounds__(256)
pz_vote_tally_kernel(VoteArgs a) {
  const int lane = threadIdx.x & 63;
  const uint64_t item = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (item >= a.nitems) return;
  const uint32_t att = a.item_att[item];
  const uint32_t slot = a.item_slot[item];
  const uint32_t c = a.att_comm[att];
  const uint64_t cb = a.coffs[c], k = a.coffs[c + 1] - cb;
  const uint64_t bb = a.boffs[att], blen = a.boffs[att + 1] - bb;
  const uint8_t* bf = a.bits + bb;
  uint32_t* bm = a.bitmaps + (uint64_t)slot * a.words_per_slot;
  uint64_t add = 0, err = 0;
  for (uint64_t i = lane; i < k; i += 64) {
    if (i >= 8 * blen) { err |= PZ_XLERR_BITFIELD; continue; }  // CheckBit would panic
    if (!((bf[i >> 3] >> (7 - (uint32_t)(i & 7))) & 1u)) continue;
    const uint32_t v = a.committee[cb + i];
    if (v >= a.nval) { err |= PZ_XLERR_MEMBER; continue; }
    const uint32_t m = 1u << (v & 31);
    // Voter bits only ever get set, so a plain read that already shows the bit is final;
    // a stale 0 (another XCD's L2) just falls through to the atomic, which decides.  After
    // the first attestation of a committee most voters are set: the atomics mostly vanish.
    if (bm[v >> 5] & m) continue;
    const uint32_t old = atomicOr(&bm[v >> 5], m);
    if (!(old & m)) add += a.balance[v];
  }
  add = wsum64(add);
  const uint64_t e1 = __ballot(err != 0);
  if (lane == 0) {
    if (add) atomicAdd((unsigned long long*)&a.totals[slot], (unsigned long long)add);
    if (e1) atomicOr((unsigned long long*)a.err, 1ull);
  }
}

hipError_t launch_vote_tally(const VoteArgs& a, hipStream_t s) {
  if (!a.nitems) return hipSuccess;
  const uint64_t threads = a.nitems * 64;
  hipLaunchKernelGGL(pz_vote_tally_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace pz
