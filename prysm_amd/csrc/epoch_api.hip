// C-ABI entry points for the T/R part of the hot path (include/prysm_hip.h): host-pointer
// drop-ins for the casper / blockchain Go functions, the device-resident batched epoch API,
// and the host-resident ShuffleIndices.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "epoch.h"
#include "runtime.h"
#include "votes.h"

namespace pz {
namespace {

EpochArgs blank_args() {
  EpochArgs a;
  std::memset(&a, 0, sizeof a);
  a.ninst = 1;
  a.pop_world = 1;
  return a;
}

// casper/validator.go:21-26: every active validator below DefaultBalance/2 exits.
extern "C" __global__ void __launch_bounds__(256)
pz_rotate_exit_kernel(const uint64_t* __restrict__ balance, const uint64_t* __restrict__ start, uint64_t* end,
                      uint64_t n, uint64_t dynasty) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (start[i] <= dynasty && dynasty < end[i] && balance[i] < PZ_DEFAULT_BALANCE / 2) end[i] = dynasty;
}

// casper/validator.go:33-39: the first k queued validators (ascending index) start now.
extern "C" __global__ void __launch_bounds__(256)
pz_rotate_induct_kernel(const uint32_t* __restrict__ queued, uint64_t k, uint64_t* start, uint64_t dynasty) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < k) start[queued[j]] = dynasty;
}

}  // namespace
}  // namespace pz

using namespace pz;

extern "C" {

int pz_validator_indices(const uint64_t* start, const uint64_t* end, uint64_t n, uint64_t dynasty,
                         int kind, uint32_t* out, uint64_t* count) {
  if (!count) return fail(PZ_EINVAL, "count is null");
  if (kind < PZ_KIND_ACTIVE || kind > PZ_KIND_QUEUED) return fail(PZ_EINVAL, "bad kind %d", kind);
  *count = 0;
  if (n == 0) return PZ_OK;
  if (!start || !end || !out) return fail(PZ_EINVAL, "null pointer");
  DeviceCtx* c;
  int rc = acquire(&c);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = c->ensure_stream())) return rc;
  Stager st{c, c->stream};
  EpochArgs a = blank_args();
  a.nval = a.nval_global = n;
  a.kind = kind;
  a.start = st.up(start, n);
  a.end = st.up(end, n);
  a.dynasty = st.up(&dynasty, 1);
  a.scal = st.zeros<uint64_t>(kScal);
  a.act_mask = st.zeros<uint64_t>((n + 63) / 64);
  a.blk_cnt = st.zeros<uint32_t>(vblocks_per_inst(n));
  a.act_list = st.zeros<uint32_t>(n);
  if (st.rc) return st.rc;
  st.check(launch_epoch_count(a, true, false, false, st.s), "pz_epoch_count_kernel");
  st.check(launch_epoch_compact(a, true, st.s), "pz_epoch_compact_kernel");
  uint64_t scal[kScal];
  st.down(scal, a.scal, kScal);
  if (st.sync()) return st.rc;
  *count = n - scal[kNoMatch];  // pass 1 counts the validators that do not match
  st.down(out, a.act_list, *count);
  return st.sync();
}

int pz_attesters_total_deposit(const uint8_t* bits, uint64_t nbytes, uint64_t* out) {
  if (!out) return fail(PZ_EINVAL, "out is null");
  *out = 0;
  if (nbytes == 0) return PZ_OK;
  if (!bits) return fail(PZ_EINVAL, "bits is null");
  DeviceCtx* c;
  int rc = acquire(&c);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = c->ensure_stream())) return rc;
  Stager st{c, c->stream};
  EpochArgs a = blank_args();
  const uint64_t offs[2] = {0, nbytes};
  a.natt = 1;
  a.bits = st.up(bits, nbytes);
  a.boffs = st.up(offs, 2);
  a.max_inst_bytes = nbytes;
  a.scal = st.zeros<uint64_t>(kScal);
  if (st.rc) return st.rc;
  st.check(launch_epoch_count(a, false, true, false, st.s), "pz_epoch_count_kernel");
  uint64_t scal[kScal];
  st.down(scal, a.scal, kScal);
  if (st.sync()) return st.rc;
  *out = scal[kPop] * PZ_DEFAULT_BALANCE;  // uint64 wrap, casper/validator.go:101
  return PZ_OK;
}

int pz_calculate_rewards(uint64_t* balance, const uint64_t* start, const uint64_t* end, uint64_t n,
                         uint64_t dynasty, uint64_t total_deposit, const uint8_t* bits,
                         const uint64_t* boffs, uint64_t natt, int* applied) {
  if (applied) *applied = 0;
  if (n && (!balance || !start || !end)) return fail(PZ_EINVAL, "null validator arrays");
  if (natt) {
    int rc0 = check_csr(boffs, natt, "bitfield");
    if (rc0) return rc0;
  }
  if (natt > 0xffffffffull) return fail(PZ_EINVAL, "too many attestations");
  DeviceCtx* c;
  int rc = acquire(&c);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = c->ensure_stream())) return rc;
  Stager st{c, c->stream};
  EpochArgs a = blank_args();
  a.nval = a.nval_global = n;
  a.kind = PZ_KIND_ACTIVE;
  a.balance = st.up(balance, n);
  a.start = st.up(start, n);
  a.end = st.up(end, n);
  a.dynasty = st.up(&dynasty, 1);
  a.total_deposit = st.up(&total_deposit, 1);
  a.natt = (uint32_t)natt;
  std::vector<uint64_t> rb;
  if (natt) {
    rb = rebase(boffs, natt);
    a.bits = st.up(bits ? bits + boffs[0] : bits, rb[natt]);
    a.boffs = st.up(rb.data(), natt + 1);
    a.max_inst_bytes = rb[natt];
  }
  a.scal = st.zeros<uint64_t>(kScal);
  a.act_mask = st.zeros<uint64_t>((n + 63) / 64);
  a.blk_cnt = st.zeros<uint32_t>(vblocks_per_inst(n));
  a.act_list = st.zeros<uint32_t>(n ? n : 1);
  if (st.rc) return st.rc;
  if (natt && rb[natt] && !bits) return fail(PZ_EINVAL, "bits is null");
  st.check(launch_epoch_count(a, true, true, false, st.s), "pz_epoch_count_kernel");
  st.check(launch_epoch_compact(a, false, st.s), "pz_epoch_compact_kernel");
  st.check(launch_epoch_reward(a, st.s), "pz_epoch_reward_kernel");
  uint64_t scal[kScal];
  st.down(scal, a.scal, kScal);
  if (st.sync()) return st.rc;
  const uint64_t dep = scal[kPop] * PZ_DEFAULT_BALANCE;
  const bool thr = dep * 3ull >= total_deposit * 2ull;
  if (thr && scal[kNact] > 0 && scal[kErrRwd])
    return fail(PZ_EINDEX, natt ? "CheckBit index out of range (incentives.go:23)"
                                : "index out of range [-1]: no attestations (incentives.go:23)");
  if (applied) *applied = scal[kApplied] ? 1 : 0;
  if (scal[kApplied]) {
    st.down(balance, a.balance, n);
    return st.sync();
  }
  return PZ_OK;
}

static int xl_common(const uint32_t* committee, const uint64_t* coffs, uint64_t ncomm,
                     const uint32_t* att_committee, const uint32_t* att_shard, const uint8_t* bits,
                     const uint64_t* boffs, uint64_t natt, const uint64_t* balance, uint64_t nval,
                     const uint64_t* rec_dynasty, uint64_t nrec, uint64_t dynasty, uint32_t* winner,
                     uint64_t* vote_out, uint64_t* total_out) {
  if (natt == 0) {
    for (uint64_t s = 0; winner && s < nrec; ++s) winner[s] = 0xffffffffu;
    return PZ_OK;
  }
  if (!att_committee || !vote_out || !total_out) return fail(PZ_EINVAL, "null pointer");
  if (natt > 0xffffffffull || nrec > 0xffffffffull) return fail(PZ_EINVAL, "sizes exceed 32 bits");
  int rc;
  if ((rc = check_csr(coffs, ncomm, "committee"))) return rc;
  if ((rc = check_csr(boffs, natt, "bitfield"))) return rc;
  for (uint64_t i = 0; i < natt; ++i)
    if (att_committee[i] >= ncomm) return fail(PZ_EINVAL, "attestation %llu names committee %u of %llu",
                                               (unsigned long long)i, att_committee[i], (unsigned long long)ncomm);
  DeviceCtx* c;
  if ((rc = acquire(&c))) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = c->ensure_stream())) return rc;
  Stager st{c, c->stream};
  EpochArgs a = blank_args();
  a.nval = a.nval_global = nval;
  a.balance = st.up(const_cast<uint64_t*>(balance), nval);
  a.natt = (uint32_t)natt;
  std::vector<uint64_t> rb = rebase(boffs, natt), rc_ = rebase(coffs, ncomm);
  a.bits = st.up(bits ? bits + boffs[0] : bits, rb[natt]);
  a.boffs = st.up(rb.data(), natt + 1);
  a.max_inst_bytes = rb[natt];
  a.committee = st.up(committee ? committee + coffs[0] : committee, rc_[ncomm]);
  a.coffs = st.up(rc_.data(), ncomm + 1);
  a.att_comm = st.up(att_committee, natt);
  a.vote = st.zeros<uint64_t>(natt);
  a.total = st.zeros<uint64_t>(natt);
  a.scal = st.zeros<uint64_t>(kScal);
  if (winner) {
    a.att_shard = st.up(att_shard, natt);
    a.nrec = (uint32_t)nrec;
    a.rec_dynasty = st.up(rec_dynasty, nrec);
    a.winner = st.zeros<uint32_t>(nrec, 0xff);
    std::vector<uint64_t> dyn(1, dynasty);
    a.dynasty = st.up(dyn.data(), 1);
    if (st.rc) return st.rc;
    if (!att_shard || (nrec && !rec_dynasty)) return fail(PZ_EINVAL, "null crosslink record arrays");
  }
  if (st.rc) return st.rc;
  st.check(launch_epoch_count(a, false, false, true, st.s), "pz_epoch_count_kernel");
  if (winner) st.check(launch_epoch_winners(a, st.s), "pz_epoch_winner_kernel");
  uint64_t scal[kScal];
  st.down(scal, a.scal, kScal);
  st.down(vote_out, a.vote, natt);
  st.down(total_out, a.total, natt);
  if (winner) st.down(winner, a.winner, nrec);
  if (st.sync()) return st.rc;
  if (scal[kErrXl]) {
    const uint64_t e = scal[kErrXl];
    return fail(PZ_EINDEX, "processCrosslinks would panic:%s%s%s",
                (e & kErrMember) ? " committee member >= len(validators)" : "",
                (e & kErrBitfield) ? " bitfield shorter than committee (CheckBit)" : "",
                (e & kErrShard) ? " shard id >= len(crosslinkRecords)" : "");
  }
  return PZ_OK;
}

int pz_crosslink_tally(const uint32_t* committee, const uint64_t* coffs, uint64_t ncomm,
                       const uint32_t* att_committee, const uint8_t* bits, const uint64_t* boffs,
                       uint64_t natt, const uint64_t* balance, uint64_t nval, uint64_t* vote_out,
                       uint64_t* total_out) {
  return xl_common(committee, coffs, ncomm, att_committee, nullptr, bits, boffs, natt, balance, nval,
                   nullptr, 0, 0, nullptr, vote_out, total_out);
}

int pz_process_crosslinks(const uint32_t* committee, const uint64_t* coffs, uint64_t ncomm,
                          const uint32_t* att_committee, const uint32_t* att_shard,
                          const uint8_t* bits, const uint64_t* boffs, uint64_t natt,
                          const uint64_t* balance, uint64_t nval, const uint64_t* rec_dynasty,
                          uint64_t nrec, uint64_t dynasty, uint32_t* winner, uint64_t* vote_out,
                          uint64_t* total_out) {
  if (!winner) return fail(PZ_EINVAL, "winner is null");
  return xl_common(committee, coffs, ncomm, att_committee, att_shard, bits, boffs, natt, balance, nval,
                   rec_dynasty, nrec, dynasty, winner, vote_out, total_out);
}

// ---- device-resident batched epoch -------------------------------------------------------
static int check_batch(const pz_epoch_batch* b) {
  if (!b) return fail(PZ_EINVAL, "batch is null");
  if (!b->ninst || !b->scal || !b->dynasty || !b->start || !b->end || !b->balance)
    return fail(PZ_EINVAL, "batch: missing validator arrays / scal");
  if (b->nval_global < b->val_offset + b->nval) return fail(PZ_EINVAL, "batch: shard exceeds nval_global");
  if (b->natt && (!b->bits || !b->boffs)) return fail(PZ_EINVAL, "batch: missing bitfields");
  if (b->committee && b->natt && (!b->coffs || !b->att_comm || !b->vote || !b->total))
    return fail(PZ_EINVAL, "batch: missing committee arrays");
  if (b->pop_world == 0 || b->pop_rank >= b->pop_world) return fail(PZ_EINVAL, "batch: bad pop split");
  if (b->ninst > 65535 || (uint64_t)b->ninst * b->natt >= (1ull << 32) || b->nval >= (1ull << 32))
    return fail(PZ_EINVAL, "batch: more than 65535 instances, 2^32 attestations or 2^32 validators");
  return PZ_OK;
}

int pz_dev_epoch_count(const pz_epoch_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  hipError_t e = launch_epoch_count(*b, true, true, b->committee != nullptr, (hipStream_t)stream);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_epoch_count_kernel");
}

int pz_dev_epoch_finish(const pz_epoch_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  if (!b->total_deposit) return fail(PZ_EINVAL, "batch: total_deposit is null");
  hipStream_t s = (hipStream_t)stream;
  const bool winners = b->committee && b->natt && b->nrec && b->winner && b->att_shard && b->rec_dynasty;
  const bool compact = b->nval == b->nval_global && b->act_mask && b->blk_cnt && b->act_list;
  hipError_t e = launch_epoch_mid(*b, winners, compact, s);  // one launch: winners + compaction
  if (e == hipSuccess) e = launch_epoch_reward(*b, s);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "epoch finish");
}

int pz_dev_epoch_gather_compact(const pz_epoch_batch* b, const uint64_t* gathered_mask, uint32_t world,
                                uint64_t shard_words, uint32_t* gblk, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  if (!gathered_mask || !gblk || !b->act_list) return fail(PZ_EINVAL, "gather_compact: null pointer");
  if (!world || !shard_words || b->val_offset % (64 * shard_words) ||
      (uint64_t)world * 64 * shard_words < b->nval_global || b->nval > 64 * shard_words)
    return fail(PZ_EINVAL, "gather_compact: shards must be %llu-validator aligned ranges covering nval_global",
                (unsigned long long)(64 * shard_words));
  hipError_t e = launch_epoch_gather_compact(*b, gathered_mask, shard_words, gblk, (hipStream_t)stream);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_epoch_gcompact_kernel");
}

// ---- vote-cache tally ----------------------------------------------------------------------
int pz_dev_vote_tally(const pz_vote_batch* b, void* stream) {
  if (!b) return fail(PZ_EINVAL, "batch is null");
  if (!b->nitems) return PZ_OK;
  if (!b->committee || !b->coffs || !b->att_comm || !b->bits || !b->boffs || !b->item_att || !b->item_slot ||
      !b->balance || !b->bitmaps || !b->totals || !b->err)
    return fail(PZ_EINVAL, "vote batch: null pointer");
  if (b->words_per_slot * 32 < b->nval) return fail(PZ_EINVAL, "vote batch: words_per_slot too small");
  hipError_t e = launch_vote_tally(*b, (hipStream_t)stream);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_vote_tally_kernel");
}

int pz_vote_tally(const uint32_t* committee, const uint64_t* coffs, uint64_t ncomm, const uint32_t* att_comm,
                  const uint8_t* bits, const uint64_t* boffs, uint64_t natt, const uint32_t* item_att,
                  const uint32_t* item_slot, uint64_t nitems, const uint64_t* balance, uint64_t nval,
                  uint32_t* bitmaps, uint64_t nslots, uint64_t words_per_slot, uint64_t* totals) {
  if (!nitems) return PZ_OK;
  int rc;
  if ((rc = check_csr(coffs, ncomm, "committee"))) return rc;
  if ((rc = check_csr(boffs, natt, "bitfield"))) return rc;
  if (!item_att || !item_slot || !att_comm || !bitmaps || !totals) return fail(PZ_EINVAL, "null pointer");
  if (words_per_slot * 32 < nval) return fail(PZ_EINVAL, "words_per_slot too small");
  for (uint64_t i = 0; i < nitems; ++i) {
    if (item_att[i] >= natt || item_slot[i] >= nslots)
      return fail(PZ_EINVAL, "work item %llu out of range", (unsigned long long)i);
  }
  for (uint64_t a = 0; a < natt; ++a)
    if (att_comm[a] >= ncomm) return fail(PZ_EINVAL, "attestation %llu names a missing committee", (unsigned long long)a);
  DeviceCtx* c;
  if ((rc = acquire(&c))) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = c->ensure_stream())) return rc;
  Stager st{c, c->stream};
  std::vector<uint64_t> rb = rebase(boffs, natt), rc_ = rebase(coffs, ncomm);
  pz_vote_batch v;
  std::memset(&v, 0, sizeof v);
  v.committee = st.up(committee ? committee + coffs[0] : committee, rc_[ncomm]);
  v.coffs = st.up(rc_.data(), ncomm + 1);
  v.att_comm = st.up(att_comm, natt);
  v.bits = st.up(bits ? bits + boffs[0] : bits, rb[natt]);
  v.boffs = st.up(rb.data(), natt + 1);
  v.item_att = st.up(item_att, nitems);
  v.item_slot = st.up(item_slot, nitems);
  v.nitems = nitems;
  v.balance = st.up(balance, nval);
  v.nval = nval;
  v.bitmaps = st.up(bitmaps, nslots * words_per_slot);
  v.words_per_slot = words_per_slot;
  v.totals = st.up(totals, nslots);
  v.err = st.zeros<uint64_t>(1);
  if (st.rc) return st.rc;
  st.check(launch_vote_tally(v, st.s), "pz_vote_tally_kernel");
  uint64_t err = 0;
  st.down(&err, v.err, 1);
  st.down(bitmaps, v.bitmaps, nslots * words_per_slot);
  st.down(totals, v.totals, nslots);
  if (st.sync()) return st.rc;
  if (err) return fail(PZ_EINDEX, "calculateBlockVoteCache would panic (short bitfield or voter >= len(validators))");
  return PZ_OK;
}

// ---- host-resident shuffle ---------------------------------------------------------------
int pz_shuffle_indices(const uint8_t seed[32], uint32_t* list, uint64_t n) {
  if (n > PZ_MAX_VALIDATORS) return fail(PZ_ETOOMANY, "Validator count has exceeded MaxValidator Count");
  if (!seed) return fail(PZ_EINVAL, "seed is null");
  if (n && !list) return fail(PZ_EINVAL, "list is null");
  uint8_t hs[64];
  const uint64_t offs[2] = {0, 32};
  int rc = pz_blake2b512_batch(seed, offs, 1, hs, 64);  // utils/shuffle.go:19 (on the GPU)
  if (rc) return rc;
  uint32_t sw[21];  // utils/shuffle.go:25-26: byte-wrapped sum of 3 seed bytes, j = 0,3,..,60
  for (int j = 0, k = 0; j + 3 < 64; j += 3, ++k) sw[k] = (uint8_t)(hs[j] + hs[j + 1] + hs[j + 2]);
  // utils/shuffle.go:28-31: swap(i, sw[k] % (n - i) + i) for k = 0..20, i = 0..n-2.  Every
  // sw[k] is a byte, so while n - i > 255 the modulo is the identity and the targets are the
  // fixed offsets i + sw[k]: the 21 swaps of step i touch only the 256-entry window at i (L1
  // resident, no division).  Only the last 255 steps need the modulo.
  // (An offset of 0 swaps list[i] with itself: a no-op, dropped from the list.)
  uint32_t off[21];
  int noff = 0;
  for (int k = 0; k < 21; ++k)
    if (sw[k]) off[noff++] = sw[k];
  const uint64_t fast = n > 256 ? n - 256 : 0;
  uint32_t* L = list;
  for (uint64_t i = 0; i < fast; ++i) {
    uint32_t vi = L[i];  // list[i] stays in a register across its swaps
    for (int k = 0; k < noff; ++k) {
      uint32_t* q = L + i + off[k];
      const uint32_t t = *q;
      *q = vi;
      vi = t;
    }
    L[i] = vi;
  }
  for (uint64_t i = fast; i + 1 < n; ++i) {
    const uint64_t rem = n - i;
    for (int k = 0; k < 21; ++k) {
      const uint64_t p = sw[k] % rem + i;
      const uint32_t t = list[i];
      list[i] = list[p];
      list[p] = t;
    }
  }
  return PZ_OK;
}

int pz_rotate_validator_set(const uint64_t* balance, uint64_t* start, uint64_t* end, uint64_t n, uint64_t dynasty) {
  if (n == 0) return PZ_OK;
  if (!balance || !start || !end) return fail(PZ_EINVAL, "null pointer");
  DeviceCtx* c;
  int rc = acquire(&c);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = c->ensure_stream())) return rc;
  Stager st{c, c->stream};
  uint64_t* d_start = st.up(start, n);
  uint64_t* d_end = st.up(end, n);
  const uint64_t* d_bal = st.up(balance, n);
  const uint64_t* d_dyn = st.up(&dynasty, 1);
  // upperbound = len(ActiveValidatorIndices)/30 + 1, counted before the exits (validator.go:18)
  EpochArgs a = blank_args();
  a.nval = a.nval_global = n;
  a.kind = PZ_KIND_ACTIVE;
  a.start = d_start;
  a.end = d_end;
  a.dynasty = d_dyn;
  a.scal = st.zeros<uint64_t>(kScal);
  a.act_mask = st.zeros<uint64_t>((n + 63) / 64);
  a.blk_cnt = st.zeros<uint32_t>(vblocks_per_inst(n));
  a.act_list = st.zeros<uint32_t>(n);
  EpochArgs q = a;  // QueuedValidatorIndices after the exits (their start is untouched)
  q.kind = PZ_KIND_QUEUED;
  q.scal = st.zeros<uint64_t>(kScal);
  if (st.rc) return st.rc;
  st.check(launch_epoch_count(a, true, false, false, st.s), "pz_epoch_count_kernel");
  const dim3 grid((uint32_t)((n + 255) / 256));
  hipLaunchKernelGGL(pz_rotate_exit_kernel, grid, dim3(256), 0, st.s, d_bal, d_start, d_end, n, dynasty);
  st.check(hipGetLastError(), "pz_rotate_exit_kernel");
  st.check(launch_epoch_count(q, true, false, false, st.s), "pz_epoch_count_kernel");
  st.check(launch_epoch_compact(q, true, st.s), "pz_epoch_compact_kernel");
  uint64_t sa[kScal], sq[kScal];
  st.down(sa, a.scal, kScal);
  st.down(sq, q.scal, kScal);
  if (st.sync()) return st.rc;
  const uint64_t k = std::min<uint64_t>((n - sa[kNoMatch]) / 30 + 1, n - sq[kNoMatch]);
  if (k) {
    hipLaunchKernelGGL(pz_rotate_induct_kernel, dim3((uint32_t)((k + 255) / 256)), dim3(256), 0, st.s, q.act_list, k,
                       d_start, dynasty);
    st.check(hipGetLastError(), "pz_rotate_induct_kernel");
  }
  st.down(start, d_start, n);
  st.down(end, d_end, n);
  return st.sync();
}

int pz_shuffle_validators_to_committees(const uint8_t seed[32], const uint64_t* start, const uint64_t* end,
                                        uint64_t n, uint64_t dynasty, uint64_t crosslink_start_shard,
                                        uint32_t* members, uint64_t* coffs, uint64_t* shard_id, uint64_t* slot_offs,
                                        uint64_t cap_comm, uint64_t* ncomm) {
  if (!ncomm || !slot_offs) return fail(PZ_EINVAL, "null pointer");
  *ncomm = 0;
  // ActiveValidatorIndices on the device, then the host swap chain (sharding.go:12-16)
  std::vector<uint32_t> idx(n ? n : 1);
  uint64_t na = 0;
  int rc = pz_validator_indices(start, end, n, dynasty, PZ_KIND_ACTIVE, idx.data(), &na);
  if (rc) return rc;
  if ((rc = pz_shuffle_indices(seed, idx.data(), na))) return rc;
  // getCommitteeParams (sharding.go:60-73)
  const uint64_t cyc = PZ_CYCLE_LENGTH;
  uint64_t cps = 1, spc = 1;
  if (na >= cyc * PZ_MIN_COMMITTEE_SIZE) {
    cps = na / (cyc * PZ_MIN_COMMITTEE_SIZE * 2) + 1;
  } else {
    while (na * spc < PZ_MIN_COMMITTEE_SIZE * cyc && spc < cyc) spc *= 2;
  }
  if (cap_comm < cyc * cps) {
    *ncomm = cyc * cps;
    return fail(PZ_ERANGE, "need room for %llu committees", (unsigned long long)(cyc * cps));
  }
  if (!coffs || !shard_id || (na && !members)) return fail(PZ_EINVAL, "null pointer");
  // splitBySlotShard (sharding.go:27-53): SplitIndices into 64 slots, each into cps committees
  uint64_t c = 0;
  coffs[0] = 0;
  for (uint64_t i = 0; i < cyc; ++i) {
    slot_offs[i] = c;
    const uint64_t s0 = na * i / cyc, s1 = na * (i + 1) / cyc, len = s1 - s0;
    const uint64_t shard_start = crosslink_start_shard + i * cps / spc;
    for (uint64_t j = 0; j < cps; ++j, ++c) {
      const uint64_t c0 = s0 + len * j / cps, c1 = s0 + len * (j + 1) / cps;
      shard_id[c] = (shard_start + j) % PZ_SHARD_COUNT;
      std::memcpy(members + coffs[c], idx.data() + c0, (c1 - c0) * 4);
      coffs[c + 1] = coffs[c] + (c1 - c0);
    }
  }
  slot_offs[cyc] = c;
  *ncomm = c;
  return PZ_OK;
}

}  // extern "C"

#ifdef PZ_AB_BUILD  // the A/B library only (tools/epoch_parts.py)
// Internal: launch pass 1 with a subset of its block ranges (per-part timing in tools/).
extern "C" int pz_debug_epoch_count(const pz_epoch_batch* b, int do_val, int do_pop, int do_xl, void* stream) {
  hipError_t e = pz::launch_epoch_count(*b, do_val != 0, do_pop != 0, do_xl != 0, (hipStream_t)stream);
  return e == hipSuccess ? PZ_OK : pz::hip_fail(e, "pz_epoch_count_kernel");
}
extern "C" int pz_debug_epoch_reward(const pz_epoch_batch* b, void* stream) {
  hipError_t e = pz::launch_epoch_reward(*b, (hipStream_t)stream);
  return e == hipSuccess ? PZ_OK : pz::hip_fail(e, "pz_epoch_reward_kernel");
}
#endif
