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
struct VoteWordArgs {
  const uint32_t* committee;  // ShardAndCommittee member lists (CSR, global validator indices)
  const uint4* rec;           // natt: {committee's first member offset, its size k, 0, 0}
  const uint32_t* slots;      // natt x 64: the vote-cache id of each signed parent hash, or
                              //   UINT32_MAX where the parent is not tallied (skipped, none)
  const uint8_t* bits;        // the bitfields, ceil(k / 8) bytes each, attestation a's at a * bstride
  uint32_t bstride;           //   (a multiple of 4 >= every committee's ceil(k / 8): the bytes load
                              //   beside the record, not behind it)
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
};
constexpr uint32_t kVoteWordThreads = 256;
// Blocks of the tally part of a launch (4 waves each).
inline uint32_t vote_word_blocks(const VoteWordArgs& a) {
  return (uint32_t)((a.natt * a.chunks + 3) / 4);
}
hipError_t launch_vote_words(const VoteWordArgs& a, hipStream_t s);
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
hipError_t launch_stage_h2d_segs(const StageSegs& g, hipStream_t s);
// Copy `bytes` (a multiple of 16) from mapped pinned host memory to device memory in a kernel on
// stream s: 16 B per lane, so the bytes cross PCIe in one round trip of coalesced reads.
hipError_t launch_stage_h2d(const void* host_mapped, void* dev, uint64_t bytes, hipStream_t s);

hipError_t launch_vote_gather(const uint64_t* totals, VoteGatherSlots slots, const uint64_t* err, uint64_t* out,
                              hipStream_t s);
}  // namespace pz
