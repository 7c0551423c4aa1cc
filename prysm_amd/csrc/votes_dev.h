// Device code of the vote-cache tally shared by votes.hip and epoch.hip (the leader pass also
// runs inside pz_vote_leader_count_kernel, beside a stateRecalc's epoch count blocks).
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

// A fixed grid of kLeaderWaves waves walks the compact leader list of pass 1.
constexpr uint32_t kLeaderWaves = 4096;  // 2048 / 4096 / 8192 A/B: profiles/r03/replay_leader_waves_r3m.txt
// The leader pass over nblk blocks of 256 threads, as block `bid` (a kernel of its own, or the
// first nblk blocks of a launch shared with other work: pz_vote_leader_count_kernel).
__device__ __forceinline__ void vote_leader_body(const VoteIdArgs& a, uint32_t nblk, uint32_t bid) {
  const uint32_t n = *a.nlead;
  if (bid == 0 && threadIdx.x == 0) *a.nlead_next = 0;  // (no wave of this flush reads it)
  const uint32_t waves = nblk * (blockDim.x >> 6);
  for (uint32_t li = ((uint64_t)bid * blockDim.x + threadIdx.x) >> 6; li < n; li += waves) {
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
  const uint32_t busy = n ? min(nblk, (n + (blockDim.x >> 6) - 1) / (blockDim.x >> 6)) : 1u;
  if (bid >= busy) return;
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

}  // namespace pz
