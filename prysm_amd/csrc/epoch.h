// Epoch-transition (T/R) kernels: device-side argument block and launchers (epoch.hip).
//
// One launch sequence processes B independent epoch instances ("throughput mode"); B = 1
// is the Go drop-in.  Validator arrays are instance-major [B][nval]; pending attestations
// are CSR bitfields over all B*natt attestations; committees are a CSR shared by all
// instances.  A multi-GPU rank holds validators [val_offset, val_offset+nval) of each
// instance and combines the partial sums in `scal`/`vote`/`total` with one RCCL all-reduce.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/prysm_hip.h"

namespace pz {

enum : int {
  kPop = PZ_SCAL_POP, kNact = PZ_SCAL_NACT, kErrXl = PZ_SCAL_ERR_XL, kErrRwd = PZ_SCAL_ERR_RWD,
  kApplied = PZ_SCAL_APPLIED, kNextBal = PZ_SCAL_NEXT_BAL, kMaxIdx1 = PZ_SCAL_MAXIDX1,
  kNoMatch = PZ_SCAL_NOMATCH, kScal = PZ_SCAL_COUNT
};
enum : uint64_t {
  kErrMember = PZ_XLERR_MEMBER, kErrBitfield = PZ_XLERR_BITFIELD, kErrShard = PZ_XLERR_SHARD,
  kErrLayout = PZ_XLERR_LAYOUT
};

typedef pz_epoch_batch EpochArgs;

constexpr int kValPerThread = 8;
constexpr int kThreads = 256;
constexpr uint64_t kValPerBlock = (uint64_t)kValPerThread * kThreads;  // 2048
constexpr uint64_t kPopBytesPerBlock = 16ull * kThreads * 4;            // 16 KiB

inline uint64_t vblocks_per_inst(uint64_t nval) { return (nval + kValPerBlock - 1) / kValPerBlock; }

// Pass 1: classify/count validators (+active mask), popcount bitfields, crosslink tallies.
hipError_t launch_epoch_count(const EpochArgs& a, bool do_val, bool do_pop, bool do_xl,
                              hipStream_t s);
// Crosslink winner rule on the (all-reduced) tallies: first qualifying attestation per shard.
hipError_t launch_epoch_winners(const EpochArgs& a, hipStream_t s);
// General rank path: scan per-block counts and compact the active list (no-op per instance
// when every validator is active).  Single-rank only (multi-rank gathers lists itself).
hipError_t launch_epoch_compact(const EpochArgs& a, bool force, hipStream_t s);
// Multi-rank general rank path: global active list from the all-gathered shard masks
// gmask[world][B][sw] (gblk: scratch [B][vblocks_per_inst(nval_global)]).
hipError_t launch_epoch_gather_compact(const EpochArgs& a, const uint64_t* gmask, uint64_t sw, uint32_t* gblk,
                                       hipStream_t s);
// Winners + compaction in one launch (the device-resident finish path).
hipError_t launch_epoch_mid(const EpochArgs& a, bool winners, bool compact, hipStream_t s);
// Pass 2: rewards (in place) + post-reward active balance sum.
hipError_t launch_epoch_reward(const EpochArgs& a, hipStream_t s);

}  // namespace pz
