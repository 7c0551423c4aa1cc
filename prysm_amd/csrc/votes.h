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

// The block engine's tally (chain.hip): natt attestations x their 64 signed parent hashes.
struct VoteIdArgs {
  const uint32_t* committee;
  const uint64_t* coffs;
  const uint32_t* att_comm;  // natt
  const uint8_t* bits;       // CSR bitfields
  const uint64_t* boffs;     // natt+1
  const uint32_t* slots;     // natt x 64 vote-cache slots of the signed parent hashes
  const uint64_t* skip;      // natt: bit j set = parent j equals an oblique parent hash
  uint64_t natt;
  const uint64_t* balance;
  uint64_t nval;
  uint32_t* bitmaps;
  uint64_t words_per_slot;
  uint64_t* totals;
  uint8_t* present;  // per slot: the Go map has an entry
  uint64_t* err;
  uint32_t* ubits;   // per (slot, committee) group: union bitfield, cwords words (zero between flushes)
  uint32_t* uflag;   // per group: touched in this flush (zero between flushes)
  uint4* leader;     // the groups to tally (compact list, *nlead entries): {slot, committee,
                     //   committee's first member offset, committee size}
  uint32_t* nlead;       // zero when the flush starts (the previous flush's leader pass zeroed it)
  uint32_t* nlead_next;  // the other counter: zeroed here for the next flush
  uint64_t ncomm, cwords;
  uint64_t val_offset;   // a validator-range shard: balance and bitmaps hold [val_offset, val_offset + nval)
  uint64_t nval_global;  // of nval_global validators (0: nval, unsharded)
  // non-null: the leader pass's last block to finish also does launch_vote_gather's work into
  // gather_out (a stateRecalc's flush: one kernel boundary less on the walk's wait); `ticket`
  // is a zero device word, left zero
  uint64_t* gather_out;
  uint32_t* ticket;
  VoteGatherSlots gq;
  // gather_out[kJustifySlots + 1] is set to gather_seq last, behind a system-scope release, so
  // that the host can poll the pinned words instead of sleeping in an event wait
  uint64_t gather_seq;
};
hipError_t launch_vote_ids(const VoteIdArgs& a, hipStream_t s);
// Pass 1 alone (the per-item union); pass 2 then runs as launch_vote_leader_count (epoch.h).
hipError_t launch_vote_union(const VoteIdArgs& a, hipStream_t s);
// The same two passes with the queue arrays (att_comm, bits, boffs, slots, skip) in mapped
// pinned host memory, read in place by a per-attestation union pass (no staging copy).
hipError_t launch_vote_ids_direct(const VoteIdArgs& a, hipStream_t s);
// The per-attestation union pass (as launch_vote_ids_direct) over device copies of the queue.
hipError_t launch_vote_ids_att(const VoteIdArgs& a, hipStream_t s);
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
