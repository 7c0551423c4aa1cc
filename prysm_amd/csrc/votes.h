// Vote-cache tally kernel arguments and launcher (votes.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/prysm_hip.h"

namespace pz {
typedef pz_vote_batch VoteArgs;
hipError_t launch_vote_tally(const VoteArgs& a, hipStream_t s);

// The 64 totals a stateRecalc's justification loop reads (blockchain/core.go:413-418) and the
// sticky tally panic flag, gathered into out[0..64] (slot UINT32_MAX: no map entry, total 0):
// one small D2H (or one 65-word all-reduce of a validator-range-sharded cache) per transition.
constexpr int kJustifySlots = 64;
struct VoteGatherSlots {
  uint32_t slot[kJustifySlots];
};

// The block engine's tally (chain.hip), voter-major: bit j of bm[w * nval + v] says validator
// lo + v has voted for the hash of vote-cache id 64 w + j.  An attestation's 64 signed parent
// hashes fall in a handful of such words (the recent window's ids are consecutive), so one
// 64-bit atomicOr per voter and word records its votes for all of those parents at once.
//
// One queued attestation is one 64-B record, so that the wave tallying it reads all it needs
// from the walk's pinned queue in ONE host-link request (round 4: a 16-B record, a 256-B id row
// and the bitfield bytes were ~9 requests per wave, and the flush's waves queued on them).
// The ids of its 64 signed parent hashes (UINT32_MAX where a parent is not tallied: skipped, or
// none) are, for the usual attestation, a run: the recent window's ids are assigned in the order
// the hashes first appear, a skipped slot repeating its predecessor's hash.  So a record gives
// them as s0 (the first tallied parent's id) + step (bit j: parent j's id is the previous tallied
// parent's + 1, else the same) + absent (bit j: parent j not tallied); any other attestation
// keeps an explicit 64-id row and names it (kVoteIdsRow, s0 = the row).
constexpr uint32_t kVoteIdsRow = 1;  // VoteRec.form: ids in slots[64 * s0, 64 * s0 + 64)
struct alignas(64) VoteRec {
  uint32_t cb, k;    // the committee's first member offset (CSR), its size
  uint32_t s0;       // the first tallied parent's id (kVoteIdsRow: the id row)
  uint32_t form;     // 0 or kVoteIdsRow
  uint64_t step;     // (form 0) bit j: id(j) = id(previous tallied parent) + 1, else the same
  uint64_t absent;   // (form 0) bit j: parent j not tallied
  uint32_t bits[8];  // VoteWordArgs.bits == null: the bitfield's first 32 bytes (k <= 256), zero-padded
};
static_assert(sizeof(VoteRec) == 64, "one 64-B request per record");
constexpr uint32_t kVoteInlineBits = 256;  // committees up to this size keep their bitfield inline

// The grouped form of a flush (VoteWordArgs.ngroups > 0): its attestations grouped by committee.
// A committee's attestations in one flush (one per block that carries it: 64 per transition on
// the configs[4] chain) share their voters, so a wave per (group, 64 members) ORs each voter's
// parents over the group's attestations in registers and then makes ONE 64-bit atomicOr per
// voter and id word, where the per-attestation form made one per attestation (the same voter
// words hit 64 times a flush: 131 k serialising atomics per transition at 65,536 validators).
// Needs every record in the run form (the id set of a run is the range [s0, s0 + popcount(step)])
// with its bitfield inline; a group spans at most kVoteGroupWords id words.
constexpr int kVoteMaxGroups = 64;  // (kernel arguments: 2 KB of the 4 KB limit)
constexpr int kVoteGroupWords = 4;
struct VoteGroup {
  uint32_t cb, k;      // the committee
  uint32_t first, n;   // its n attestations (below)
  uint32_t wlo, nw;    // the id words its parents span: [wlo, wlo + nw), nw <= kVoteGroupWords
  uint32_t wave0;      // its first unit (max(1, ceil(k / 64)) units of 64 members per group)
  uint32_t stride;     // its records are first + stride * t (0: perm[first + t])
};

struct VoteWordArgs {
  const uint32_t* committee;  // ShardAndCommittee member lists (CSR, global validator indices)
  const VoteRec* rec;         // natt records
  const uint32_t* slots;      // the explicit id rows (kVoteIdsRow records)
  const uint8_t* bits;        // null: every bitfield inline (every committee <= kVoteInlineBits);
                              //   else every bitfield here, ceil(k / 8) bytes, attestation a's at
                              //   a * bstride (a multiple of 4 >= every committee's ceil(k / 8):
                              //   the bytes load beside the record, not behind it)
  uint32_t bstride;
  uint64_t natt;
  uint32_t chunks;            // waves per attestation: max over the flush of ceil(k / 256), >= 1
  const uint64_t* balance;
  uint64_t nval;              // a validator-range shard: balance and bm columns hold [val_offset,
  uint64_t val_offset;        //   val_offset + nval) of nval_global validators
  uint64_t nval_global;
  uint64_t* bm;
  uint64_t* totals;           // per id: VoteTotalDeposit
  uint8_t* present;           // per id: the Go map has an entry
  uint64_t* err;
  // non-null: the last tally block to finish gathers the 64 justification totals and the panic
  // flag into gather_out (pinned), then writes gather_out[kJustifySlots + 1] = gather_seq behind
  // a system-scope release; `ticket` is a zero device word, left zero
  uint64_t* gather_out;
  uint32_t* ticket;
  VoteGatherSlots gq;
  uint64_t gather_seq;
  // the grouped form (0 groups: one wave per (attestation, 256 members)): nwaves units, each
  // one block of kVoteWordThreads
  uint32_t ngroups, nwaves;
  const uint32_t* perm;  // the records' indices, group by group
  VoteGroup groups[kVoteMaxGroups];
};
constexpr uint32_t kVoteWordThreads = 256;    // the tally blocks beside an epoch count pass
constexpr uint32_t kVoteWordMaxThreads = 1024;  // pz_vote_words_kernel's blocks (PZ_VOTE_WAVES per block)
// Blocks of the tally part of a launch (threads / 64 waves each).
inline uint32_t vote_word_blocks(const VoteWordArgs& a, uint32_t threads = kVoteWordThreads) {
  if (a.ngroups) return a.nwaves;  // (one block of kVoteWordThreads per unit)
  const uint64_t wpb = threads / 64, waves = a.natt * a.chunks;
  return (uint32_t)((waves + wpb - 1) / wpb);
}
hipError_t launch_vote_words(const VoteWordArgs& a, hipStream_t s);
// (tools/ only) the same with per-wave phase stamps into tr[wave][8] (null: none)
#ifdef PZ_AB_BUILD  // the A/B library only
hipError_t launch_vote_words_traced(const VoteWordArgs& a, uint64_t* tr, hipStream_t s);
#endif
// Up to 6 copies from mapped pinned memory to device memory in ONE launch (16 B per lane; the
// sources may be read up to 15 bytes past their ends, so a source buffer's capacity must cover
// ceil16 of its bytes).
struct StageSeg {
  const void* src;
  void* dst;
  uint64_t n16;
};
struct StageSegs {
  StageSeg seg[6];
  int nseg;
};
#ifdef PZ_AB_BUILD  // the A/B library only
hipError_t launch_stage_h2d_segs(const StageSegs& g, hipStream_t s);
#endif
// Copy `bytes` (a multiple of 16) from mapped pinned host memory to device memory in a kernel on
// stream s: 16 B per lane, so the bytes cross PCIe in one round trip of coalesced reads.
hipError_t launch_stage_h2d(const void* host_mapped, void* dev, uint64_t bytes, hipStream_t s);

hipError_t launch_vote_gather(const uint64_t* totals, VoteGatherSlots slots, const uint64_t* err, uint64_t* out,
                              hipStream_t s);
}  // namespace pz
