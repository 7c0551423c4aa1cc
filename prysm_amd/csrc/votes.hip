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

// tally_item for a committee of at most 256 members (the chain's leaders): a lane's four
// members go through each step together -- bits and member ids, then the voter words, then the
// atomics, then the balances -- so a wave waits out four round trips, not four per member.
// (The loop form waited them out member after member: 20 us per transition's leader pass.)
__device__ __forceinline__ void tally_item_x4(const uint32_t* __restrict__ committee, uint64_t cb, uint64_t k,
                                              const uint8_t* bf, uint64_t blen, const uint64_t* __restrict__ balance,
                                              uint64_t nval, uint32_t* bm, uint64_t* total, uint64_t* errp,
                                              uint64_t lo, uint64_t nval_global) {
  if (!nval_global) nval_global = nval;
  const int lane = threadIdx.x & 63;
  uint32_t v[4], word[4];
  uint64_t bal[4];
  bool on[4];
  uint64_t err = 0, add = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // bits and member ids
    const uint64_t i = lane + 64 * q;
    on[q] = false;
    v[q] = 0;
    if (i < k) {
      if (i >= 8 * blen) {
        err |= PZ_XLERR_BITFIELD;  // CheckBit would panic
      } else if ((bf[i >> 3] >> (7 - (uint32_t)(i & 7))) & 1u) {
        on[q] = true;
        v[q] = committee[cb + i];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // range checks, then the voter words
    if (on[q] && v[q] >= nval_global) {
      err |= PZ_XLERR_MEMBER;
      on[q] = false;
    }
    const uint64_t lv = (uint64_t)v[q] - lo;
    if (on[q] && lv >= nval) on[q] = false;  // another rank's validator
    word[q] = on[q] ? bm[lv >> 5] : 0xFFFFFFFFu;
    bal[q] = on[q] ? balance[lv] : 0;  // issued with the word: used only if the atomic sets the bit
  }
  uint32_t old[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // a bit already set is final; the atomic decides the rest
    const uint64_t lv = (uint64_t)v[q] - lo;
    const uint32_t m = 1u << (lv & 31);
    old[q] = 0xFFFFFFFFu;
    if (on[q] && !(word[q] & m)) old[q] = atomicOr(&bm[lv >> 5], m);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint64_t lv = (uint64_t)v[q] - lo;
    if (on[q] && !(old[q] & (1u << (lv & 31)))) add += bal[q];
  }
  add = wsum64(add);
  const uint64_t e1 = __ballot(err != 0);
  if (lane == 0) {
    if (add) atomicAdd((unsigned long long*)total, (unsigned long long)add);
    if (e1) atomicOr((unsigned long long*)errp, 1ull);
  }
}

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
constexpr uint32_t kLeaderWaves = 4096;  // 2048 / 4096 / 8192 A/B: profiles/r03/replay_leader_waves_r3m.txt
extern "C" __global__ void __launch_bounds__(256)
pz_vote_leader_kernel(VoteIdArgs a) {
  const uint32_t n = *a.nlead;
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.nlead_next = 0;  // (no wave of this flush reads it)
  const uint32_t waves = gridDim.x * (blockDim.x >> 6);
  for (uint32_t li = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; li < n; li += waves) {
    const uint4 rec = a.leader[li];  // {slot, committee, its first member, its size}
    const uint32_t slot = rec.x, c = rec.y;
    const uint64_t grp = (uint64_t)slot * a.ncomm + c;
    uint32_t* u = a.ubits + grp * a.cwords;
    const uint64_t cb = rec.z, k = rec.w;
    if (k <= 256)
      tally_item_x4(a.committee, cb, k, reinterpret_cast<const uint8_t*>(u), (k + 7) / 8, a.balance, a.nval,
                    a.bitmaps + (uint64_t)slot * a.words_per_slot, a.totals + slot, a.err, a.val_offset, a.nval_global);
    else
      tally_item(a.committee, a.coffs, c, reinterpret_cast<const uint8_t*>(u), (k + 7) / 8, a.balance, a.nval,
                 a.bitmaps + (uint64_t)slot * a.words_per_slot, a.totals + slot, a.err, a.val_offset, a.nval_global);
    // leave the group empty for the next flush
    for (uint64_t w = threadIdx.x & 63; w < a.cwords; w += 64) u[w] = 0;
    if ((threadIdx.x & 63) == 0) a.uflag[grp] = 0;
  }
  if (!a.gather_out) return;
  // The fused gather (MI355X_MICROARCH.md's last-block hand-off): every wave drains its tally
  // atomics before the block barrier, one lane per block takes a ticket, and the block that
  // takes the last one reads the complete totals with agent-scope loads (they are only written
  // by device-scope atomics) into the pinned output.  Only the blocks that had a leader take
  // a ticket (wave w takes leaders w, w + waves, ...): 1,024 arrivals on one counter cost
  // ~10 us, a transition's ~160 about 2 (the fan-in row of the guide's price list).
  const uint32_t busy = n ? min(gridDim.x, (n + (blockDim.x >> 6) - 1) / (blockDim.x >> 6)) : 1u;
  if (blockIdx.x >= busy) return;
  __shared__ uint32_t last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == busy - 1 ? 1u : 0u;
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
}

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

hipError_t launch_vote_ids_direct(const VoteIdArgs& a, hipStream_t s) {
  if (!a.natt) return hipSuccess;
  const uint64_t threads = a.natt * 64;
  hipLaunchKernelGGL(pz_vote_union_att_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(pz_vote_leader_kernel, dim3(kLeaderWaves / 4), dim3(256), 0, s, a);
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
