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
// ONE instance's reward pass whose last block hands the results to the host: out (mapped pinned)
// receives the kScal scalars, then the nrec u32 winners, then -- last, behind a system-scope
// release -- `seq` in the u64 at index kScal + (nrec + 1) / 2; the scalars are zeroed for the
// next count and `ticket` (a zero device word) is left zero.
struct EpochHandoff {
  uint32_t* ticket;
  uint64_t* out;
  uint32_t nrec;
  uint64_t seq;
};
// The vote-cache tally (votes_dev.h, voter-major) and this one-instance epoch's count pass (all
// three ranges) in ONE launch, tally blocks first (the chain engine's stateRecalc, one rank).
struct VoteWordArgs;
#ifdef PZ_AB_BUILD  // the A/B library only
hipError_t launch_vote_words_count(const VoteWordArgs& v, const EpochArgs& a, hipStream_t s);
#endif
// winners: the mid pass's crosslink winners run in the same launch (only when no compaction is
// needed: every validator active).
hipError_t launch_epoch_reward_handoff(const EpochArgs& a, const EpochHandoff& h, bool winners, hipStream_t s);

// ---- one-pass epoch (committee-order layout, every validator active) ----------------------
// GetAttestersTotalDeposit depends on the bitfields only and CalculateRewards' reward bit of
// the validator at rank i == index i (every validator active) is bit co_index[p] of the last
// bitfield, so once the bit count is known one stream over the validators classifies them,
// adds their PRE-reward balances into the crosslink tallies of their committee, applies the
// reward and sums the post-reward balances: 32 B per validator-epoch instead of 40.
//   pre   : bitfield popcount -> pre[inst].pop, zero vote/total, bitfield-length panics
//   fused : the stream above (partial sums at N > 1: all-reduce {scal, vote, total} after)
//   mid   : winners on the (reduced) tallies
// The host enables it only when no attestation names a shard >= nrec (that panic depends on
// the tallies, i.e. on balances the fused pass has already rewarded).
constexpr uint64_t kLastCoMaxBytes = 16384;  // last bitfields up to 131,072 validators
constexpr uint64_t kLastCoPos = 8192;         // positions per gathering block (one word per thread)
constexpr uint32_t kNoAtt = 0xFFFFFFFEu, kManyAtt = 0xFFFFFFFFu;  // a committee's attestation: none / several
constexpr int kPre = 2;  // pre[inst]: {bit count, PZ_XLERR_BITFIELD if a bitfield is short}
struct FusedCommittee {        // per (instance, committee)
  uint64_t boff;              // bits offset of its single attestation's bitfield
  uint32_t nbits;             // 8 * that bitfield's length
  uint32_t ga;                // that attestation's index in the instance; 0xFFFFFFFE: no
                              // attestation; 0xFFFFFFFF: several (catt / catt_offs list them)
};
struct FusedArgs {
  const uint4* items;         // [nitems] committee pieces of this rank: {first global position,
                              // count <= 256, committee, committee's first position}; a piece
                              // lies in [a + 256k, a + 256(k+1)) with a = the committee's first
                              // position & ~1, so its 16-B pairs span <= 256 positions
  uint64_t nitems;
  const FusedCommittee* cinfo;  // [B][ncomm]
  const uint32_t* catt_offs;  // [B][ncomm + 1] attestations of committee c: catt[catt_offs[c] ..)
  const uint32_t* catt;       // [B][natt] attestation index within its instance, by committee
  uint64_t ncomm;
  uint64_t* pre;              // [B][kPre], zero before `pre`
  uint64_t* pre_next;         // [B][kPre] zeroed by `fused` for the next step (ping-pong)
  int rank0;                  // 1: this rank writes the per-instance scalars (bit count, flags,
                              //    applied, nact, max index) that the all-reduce must not multiply
  uint64_t vstride;           // row stride of balance/start/end (>= nval, even)
  uint32_t* lastco;           // [B][lcw] or NULL: the reward bit of every position p (bit co_index[p]
  uint64_t lcw;               //   of the instance's last bitfield), LSB-first, gathered by `pre`
                              //   through LDS when the last bitfield fits kLastCoMaxBytes
  int own_only;               // sharded: winners proposed only for the attestations whose
                              //    committee this rank holds (pz_epoch_fwin_kernel)
  // single-launch step (one instance, one rank: the latency path, pz_epoch_one_kernel)
  int one;                    // 1: launch_epoch_one replaces pre + fused + mid
  uint32_t* ticket;           // blocks done this step (the last one forms the winners; reset by it)
  uint64_t* vote_next;        // [natt] the next step's tallies, zeroed by this step's last block
  uint64_t* total_next;
  const uint32_t* att_csize;  // [natt] the size of each attestation's committee (a layout of the
                              //   inputs made at upload, so the length check needs no coffs hop)
  const uint4* items_ci;      // [B][nitems] each piece's FusedCommittee {boff lo, boff hi, nbits,
                              //   ga} per instance, read beside its item (no items -> cinfo hop)
  // single-launch step, every attested committee one piece (so one wave holds each
  // attestation's complete tallies): that wave proposes the attestation as its shard's winner
  // (atomicMin) and zeroes its next-step tallies; no last-block pass.  The winners ping-pong:
  // this step resets winner_next (all 0xFFFFFFFF) for the next one.
  int win_in_wave;
  uint32_t* winner_next;
  // the multi-instance step (pre + fused), one rank, every attested committee one piece: the
  // fused waves form the winners the same way (pre resets them), and mid is not launched
  int win_fused;
  // the single launch over B instances (pz_epoch_multi_kernel): each block counts its
  // instance's bitfields (within kMultiMaxBitBytes, at most kMultiMaxAtt attestations); needs
  // win_in_wave (winners ping-pong per instance) and att_csize [B][natt]
  int multi;
  // [B][vstride] {start, end} dynasty of each position, saturated to 32 bits (set only when
  // every instance's CurrentDynasty is below 2^32 - 1, which makes the saturated bounds classify
  // exactly): the stream reads 8 B of them per validator instead of 16
  const uint2* se;
  // [B][vstride] the same bounds saturated to 16 bits, {start | end << 16} (set instead of `se`
  // when every instance's CurrentDynasty is below 0xFFFF): 4 B per validator
  const uint32_t* se16;
  uint64_t last_max;          // the largest last bitfield (bytes) of the instances (the LDS streaming pass)
  const uint2* att_win;       // [B][natt] {shard, record dynasty of that shard} per attestation (an
                              //   upload-time layout: loaded beside the stream, no shard -> record hop)
  // [B][vstride] the balances as u32 offsets from a per-instance u64 base (bal32_base[B]):
  // balance = base + offset (mod 2^64).  Set instead of EpochArgs.balance (which is then stale)
  // when every instance's balances lie within 2^30 of each other; a step moves an offset by at
  // most PZ_ATTESTER_REWARD, so the offsets stay inside u32 for 2^30 steps, and the state
  // re-bases them well before (epoch_state.hip).  The stream reads and writes 4 B of balance per
  // validator instead of 8, and every sum is taken on the reconstructed u64 values.
  uint32_t* bal32;
  const uint64_t* bal32_base;
  uint64_t* trace;  // (A/B library, the single launch's phase stamps: [blocks][8], or NULL)
  // single launch: each attestation of a committee with several, in catt order (the piece's
  // items_ci holds its catt range {k0, k1} then): {bitfield offset from the instance's 16-B
  // aligned bits start, 8 x its length, attestation, 0} and its att_win entry -- the bitfield
  // bytes are read from the block's LDS copy of the instance's bitfields, no global hop
  const uint4* one_ck;
  const uint2* one_cw;
};
// ---- the window pass (epoch_window.hip): the one-pass step of B instances in ONE launch ------
// Block (instance, range): a range is a run of this rank's committees (local ids [cr0, cr1)),
// so every committee's tallies complete inside one block.
constexpr int kWinThreads = 1024, kWinDepth = 2, kWinDepth16 = 2;  // (pieces in flight per wave: 3 measured slower, r5f)
constexpr uint32_t kWinKargR = 32;  // ranges whose descriptors ride in the kernel arguments (WinArgs.rdk)
// the straight-line DMA counts the product kernel is instantiated for (65,536 / 131,072 /
// 262,144 / 524,288 / 1,048,576-bit last bitfields, each + up to 15 B of alignment)
constexpr uint32_t kWinDmaK[] = {1, 2, 3, 5, 9};
struct WinArgs {
  const uint4* rdesc;         // [R] {cr0, cr1, first piece, pieces}
  uint32_t R;                 // ranges per instance (grid: B x R blocks)
  // R <= kWinKargR: rdesc's entries again, in the kernel arguments, so a block's first piece
  // descriptors depend on nothing but the kernarg segment (one dependent round trip less)
  uint4 rdk[kWinKargR];
  // [B][ptot][2] per instance and piece (<= 256 positions of one committee, from its first
  // position rounded down to 4): {first position, positions, committee - cr0, kind (0 no
  // attestation, 1 one, 2 several)}, {its first catt index, the bit of the first position in
  // the single attestation's bitfield counted from the instance's bitfields (kind 1; kind 2:
  // the committee's first position), vote bits present from the first position, 0}
  const uint4* pinfo;
  uint32_t ptot;
  const uint2* rk;            // [B][R] {the range's first catt index, its attestations}
  uint32_t cg0;               // the rank's first committee (global id)
  const uint32_t* catt;       // [B][natt] attestation indices grouped by committee (committee order)
  const uint32_t* att_csize;  // [B][natt] the size of each attestation's committee
  const uint4* cq;            // [B][natt] by catt index, for the epilogue: {attestation, its committee -
                              //   the range's cr0, shard, its record's dynasty saturated to 32 bits}
  const uint32_t* cqh;        // a dynasty >= 2^32 - 1 in the part: [B][natt] the record dynasty's high
                              //   word (cq.w its low word), else NULL
  const uint2* ckb;           // [B][natt] by catt index: {bitfield's first byte from the instance's
                              //   16-B-aligned bitfields start, its bits} (kind-2 pieces)
  uint32_t* bal32;            // [B][vstride] u32 balance offsets (or NULL: EpochArgs.balance)
  const uint64_t* bal32_base; // [B]
  const uint32_t* se16;       // [B][vstride] {start | end << 16} saturated (or NULL)
  const uint2* se;            // [B][vstride] {start, end} saturated to 32 bits (or NULL: start/end)
  uint64_t vstride;
  uint32_t* winner_next;      // [B][nrec] reset to 0xFFFFFFFF for the next step (ping-pong)
  uint64_t* vote_next;        // world > 1: [B][natt] the next step's tallies zeroed (non-owned
  uint64_t* total_next;       //   attestations stay zero for pz_epoch_state_tallies' sum), else NULL
  int rank0;                  // this rank writes the per-instance scalars
  // LDS plan: last-bitfield bytes (0: reward bits from L2), most committees / attestations of a range
  uint32_t lds_lbf, lds_maxc, lds_maxk;
  // > 0: every instance's last bitfield copy is at most dma_k x kWinThreads 16-B chunks and
  // lds_lbf holds that many (padding included), so the product kernel issues exactly dma_k DMA
  // instructions per wave, straight-line, before its first wait (kWinDmaK); 0: the copy's loop
  uint32_t dma_k;
  // every instance's u32 offsets within kTallySpan of kTallyFloor (the state keeps them there by
  // re-basing every kNarrowPeriod steps): each committee's tallies are two 32-bit wave sums of
  // (offset - floor) instead of four (epoch_window.hip)
  uint32_t narrow;
  uint64_t* trace;            // A/B library only: [blocks][4] phase stamps (s_memrealtime), else NULL
  // A/B form (epoch_window.hip AB & 16), R > 1: the R blocks of an instance each count 1/R of
  // its bitfields and meet in one 64-bit word per instance, {arrivals << 48 | length-panic
  // blocks << 39 | bits}, this step's pacc and the next step's pacc_next (zeroed by the r == 0
  // blocks; the two swap every step).  A block whose partners have not all arrived within
  // kCoopSpinTicks counts everything itself.
  uint64_t* pacc;
  uint64_t* pacc_next;
};
constexpr uint32_t kTallyFloor = (1u << 30) - (1u << 22);  // offsets start in [2^30, 2^30 + spread)
constexpr uint64_t kNarrowSpread = 1ull << 21, kNarrowPeriod = 1ull << 21;  // -> [floor, floor + 2^23)
constexpr uint64_t kCoopSpinTicks = 5000;  // s_memrealtime ticks (100 MHz): 50 us
size_t window_lds_bytes(const WinArgs& w);
hipError_t launch_epoch_window(const EpochArgs& a, const WinArgs& w, hipStream_t s);

// The single-launch step's limits: every block counts the instance's bitfields itself and the
// last block keeps one LDS word per crosslink record.
constexpr uint64_t kOneMaxBitBytes = 32768;
constexpr uint32_t kOneMaxAtt = 2048;
constexpr uint32_t kOneMaxRec = 4096;
constexpr uint64_t kMultiMaxBitBytes = 16384;
constexpr uint32_t kMultiMaxAtt = 512;
// One instance, one rank, in ONE launch (f.one): every block counts the bitfields and checks
// their lengths itself (no pre pass), streams its committee pieces as `fused` does, and the
// last block to finish (an arrival ticket) forms the winners in LDS (no mid pass).
hipError_t launch_epoch_one(const EpochArgs& a, const FusedArgs& f, hipStream_t s);
bool epoch_one_enabled(const FusedArgs& f);  // f.one
bool fused_ok(const EpochArgs& a);  // 16-B vector path available (16-B aligned validator rows)

}  // namespace pz
