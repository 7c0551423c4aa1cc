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

// The block engine's form: work item (attestation, j) for each of its 64 signed parent
// hashes, read from the hash log ids the walk recorded; the vote-cache slot of every id is
// resolved by the host when the id is logged.  No host-side grouping: pass 1 ORs each item's
// bitfield into the union bitfield of its (slot, committee) group -- dedup makes the union
// exact -- and elects the group's first item as its leader; pass 2 lets each leader tally the
// union once and clear it.  (Tallying every item directly made up to 64 waves race on the
// same voter words with atomics: 100 us per cycle instead of ~25.)
// kUnionLanes lanes per item (a committee bitfield is at most a few words): 8 items a wave.
constexpr uint32_t kUnionLanes = 8;
extern "C" __global__ void __launch_bounds__(256)
pz_vote_union_kernel(VoteIdArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t item = t / kUnionLanes;
  const uint32_t sub = (uint32_t)(t % kUnionLanes);
  const uint64_t att = item >> 6;
  if (att >= a.natt) return;
  // every load that depends only on the item first (one round trip), the skip test after
  const uint64_t sk = a.skip[att];
  const uint32_t slot = a.slots[item];
  const uint32_t c = a.att_comm[att];
  const uint64_t bb = a.boffs[att], nbytes = a.boffs[att + 1] - bb;  // the queue holds ceil(k/8) bytes
  if ((sk >> (item & 63)) & 1) return;  // an oblique parent hash (core.go:313-320) is skipped
  const uint64_t grp = (uint64_t)slot * a.ncomm + c;
  const uint64_t cb = a.coffs[c], ce = a.coffs[c + 1];  // (with the bit loads below)
  uint32_t* u = a.ubits + grp * a.cwords;
  for (uint64_t w = sub; 4 * w < nbytes; w += kUnionLanes) {
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * w + q < nbytes) x |= (uint32_t)a.bits[bb + 4 * w + q] << (8 * q);
    if (x) atomicOr(&u[w], x);
  }
  if (sub == 0) {
    a.present[slot] = 1;  // the map entry exists (core.go:322-326)
    // the leader's record carries what its pass needs, so that pass starts at the committee
    if (atomicOr(&a.uflag[grp], 1u) == 0)
      a.leader[atomicAdd(a.nlead, 1u)] = make_uint4(slot, c, (uint32_t)cb, (uint32_t)(ce - cb));
  }
}

// A fixed grid of kLeaderWaves waves walks the compact leader list of pass 1.
extern "C" __global__ void __launch_bounds__(256)
pz_vote_leader_kernel(VoteIdArgs a) { vote_leader_body(a, gridDim.x, blockIdx.x); }

// Pass 1 without a staging copy: the queue is read where the walk wrote it (pinned host memory,
// mapped), one wave per attestation, so its bytes cross the host link once -- the 64 parent
// slots (one coalesced 256-B load), the scalars, then the bitfield bytes (one byte per lane) --
// instead of once into a device copy that 64 items then re-read.  Lane j ORs the bitfield into
// the union of parent j's (slot, committee) group and elects the group's leader.
extern "C" __global__ void __launch_bounds__(256)
pz_vote_union_att_kernel(VoteIdArgs a) {
  const uint64_t att = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (att >= a.natt) return;
  const uint64_t sk = a.skip[att];
  const uint32_t c = a.att_comm[att];
  const uint64_t bb = a.boffs[att], nbytes = a.boffs[att + 1] - bb;
  const uint32_t slot = a.slots[att * 64 + lane];
  const uint64_t cb = a.coffs[c], ce = a.coffs[c + 1];
  // an oblique parent hash (core.go:313-320) is skipped
  const bool mine = !((sk >> lane) & 1) && slot != 0xFFFFFFFFu;
  const uint64_t grp = (uint64_t)slot * a.ncomm + c;
  uint32_t* u = a.ubits + grp * a.cwords;
  for (uint64_t base = 0; base < nbytes; base += 64) {
    const uint32_t byte = base + lane < nbytes ? (uint32_t)a.bits[bb + base + lane] : 0u;
    const uint64_t nw = (std::min<uint64_t>(64, nbytes - base) + 3) / 4;
    for (uint64_t w = 0; w < nw; ++w) {  // word w of this chunk: bytes 4w..4w+3, little-endian
      const uint32_t x = (uint32_t)__shfl(byte, (int)(4 * w)) | ((uint32_t)__shfl(byte, (int)(4 * w + 1)) << 8) |
                         ((uint32_t)__shfl(byte, (int)(4 * w + 2)) << 16) |
                         ((uint32_t)__shfl(byte, (int)(4 * w + 3)) << 24);
      if (mine && x) atomicOr(&u[base / 4 + w], x);
    }
  }
  if (mine) {
    a.present[slot] = 1;  // the map entry exists (core.go:322-326)
    if (atomicOr(&a.uflag[grp], 1u) == 0)
      a.leader[atomicAdd(a.nlead, 1u)] = make_uint4(slot, c, (uint32_t)cb, (uint32_t)(ce - cb));
  }
}

hipError_t launch_vote_ids_att(const VoteIdArgs& a, hipStream_t s);
hipError_t launch_vote_ids_direct(const VoteIdArgs& a, hipStream_t s) { return launch_vote_ids_att(a, s); }

hipError_t launch_vote_union(const VoteIdArgs& a, hipStream_t s) {
  if (!a.natt) return hipSuccess;
  const uint64_t uthreads = a.natt * 64 * kUnionLanes;
  hipLaunchKernelGGL(pz_vote_union_kernel, dim3((uint32_t)((uthreads + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_vote_ids(const VoteIdArgs& a, hipStream_t s) {
  if (!a.natt) return hipSuccess;
  const uint64_t uthreads = a.natt * 64 * kUnionLanes;
  hipLaunchKernelGGL(pz_vote_union_kernel, dim3((uint32_t)((uthreads + 255) / 256)), dim3(256), 0, s, a);
  static const uint32_t lw = [] {  // tools/ A/B knob for the leader grid
    const char* e = std::getenv("PZ_LEADER_WAVES");
    return e ? (uint32_t)std::max(4L, std::atol(e)) : kLeaderWaves;
  }();
  hipLaunchKernelGGL(pz_vote_leader_kernel, dim3(lw / 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

extern "C" __global__ void __launch_bounds__(256)
pz_stage_h2d_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

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

hipError_t launch_vote_ids_att(const VoteIdArgs& a, hipStream_t s) {
  if (!a.natt) return hipSuccess;
  const uint64_t threads = a.natt * 64;
  hipLaunchKernelGGL(pz_vote_union_att_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(pz_vote_leader_kernel, dim3(kLeaderWaves / 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

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
