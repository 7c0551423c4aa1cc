// pz_state: a device-resident mirror of one CrystallizedState's validator set (SoA balance /
// start / end in HBM), owned by the library, with explicit upload / download (SURVEY.md §8b
// "Ownership").  The casper drop-ins on the mirror run the same kernels as the host-pointer
// entry points of epoch_api.hip but never re-pack or re-copy the validator set per call: a
// cgo shim syncs the Go []*pb.ValidatorRecord with the mirror when it changes (rewards in
// stateRecalc, rotation) instead of on every ActiveValidatorIndices / CalculateRewards call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "epoch.h"
#include "runtime.h"

using namespace pz;

struct pz_state {
  int device = 0;
  uint64_t n = 0;
  std::mutex mu;
  hipStream_t s = nullptr;
  DevBuf balance, start, end;           // [n] u64 each: the mirror
  DevBuf scal, mask, blk, list, aux[8];  // kernel scratch
  ~pz_state() {
    (void)hipSetDevice(device);
    if (s) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
    for (DevBuf* b : {&balance, &start, &end, &scal, &mask, &blk, &list}) b->release();
    for (DevBuf& b : aux) b.release();
  }
};

namespace {

// Scratch for one filter / reward pass over the mirror (zeroed where the kernels accumulate).
int prepare(pz_state* st, EpochArgs& a, int kind) {
  std::memset(&a, 0, sizeof a);
  a.ninst = 1;
  a.pop_world = 1;
  a.nval = a.nval_global = st->n;
  a.kind = kind;
  a.balance = (uint64_t*)st->balance.ptr;
  a.start = (const uint64_t*)st->start.ptr;
  a.end = (const uint64_t*)st->end.ptr;
  int rc;
  if ((rc = st->scal.reserve(kScal * 8 + 32)) || (rc = st->mask.reserve(((st->n + 63) / 64 + 1) * 8)) ||
      (rc = st->blk.reserve((vblocks_per_inst(st->n) + 1) * 4)) || (rc = st->list.reserve((st->n + 1) * 4)))
    return rc;
  hipError_t e = hipMemsetAsync(st->scal.ptr, 0, kScal * 8 + 32, st->s);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
  a.scal = (uint64_t*)st->scal.ptr;
  a.dynasty = (const uint64_t*)st->scal.ptr + kScal;        // one u64 written per call
  a.total_deposit = (const uint64_t*)st->scal.ptr + kScal + 1;
  a.act_mask = (uint64_t*)st->mask.ptr;
  a.blk_cnt = (uint32_t*)st->blk.ptr;
  a.act_list = (uint32_t*)st->list.ptr;
  return PZ_OK;
}

int set_scalars(pz_state* st, uint64_t dynasty, uint64_t total_deposit) {
  const uint64_t v[2] = {dynasty, total_deposit};
  hipError_t e = hipMemcpyAsync((uint64_t*)st->scal.ptr + kScal, v, sizeof v, hipMemcpyHostToDevice, st->s);
  if (e == hipSuccess) e = hipStreamSynchronize(st->s);  // v is on the stack
  return e == hipSuccess ? PZ_OK : hip_fail(e, "scalars H2D");
}

int lock(pz_state* st) {
  if (!st) return fail(PZ_EINVAL, "state is null");
  hipError_t e = hipSetDevice(st->device);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "hipSetDevice");
}

}  // namespace

extern "C" {

int pz_state_new(uint64_t n, int device, pz_state** out) {
  if (!out) return fail(PZ_EINVAL, "out is null");
  *out = nullptr;
  if (n > PZ_MAX_VALIDATORS) return fail(PZ_ETOOMANY, "validator count %llu above MaxValidators", (unsigned long long)n);
  DeviceCtx* dc;
  int rc = device_ctx(device, &dc);
  if (rc) return rc;
  auto* st = new pz_state();
  st->device = device;
  st->n = n;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&st->s, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete st;
    return hip_fail(e, "hipStreamCreate");
  }
  if ((rc = st->balance.reserve(n * 8 + 16)) || (rc = st->start.reserve(n * 8 + 16)) ||
      (rc = st->end.reserve(n * 8 + 16))) {
    delete st;
    return rc;
  }
  *out = st;
  return PZ_OK;
}

int pz_state_upload(pz_state* st, const uint64_t* balance, const uint64_t* start, const uint64_t* end) {
  int rc = lock(st);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(st->mu);
  const size_t bytes = st->n * 8;
  hipError_t e = hipSuccess;
  if (balance && bytes) e = hipMemcpyAsync(st->balance.ptr, balance, bytes, hipMemcpyHostToDevice, st->s);
  if (e == hipSuccess && start && bytes) e = hipMemcpyAsync(st->start.ptr, start, bytes, hipMemcpyHostToDevice, st->s);
  if (e == hipSuccess && end && bytes) e = hipMemcpyAsync(st->end.ptr, end, bytes, hipMemcpyHostToDevice, st->s);
  if (e == hipSuccess) e = hipStreamSynchronize(st->s);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_state_upload");
}

int pz_state_download(pz_state* st, uint64_t* balance, uint64_t* start, uint64_t* end) {
  int rc = lock(st);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(st->mu);
  const size_t bytes = st->n * 8;
  hipError_t e = hipSuccess;
  if (balance && bytes) e = hipMemcpyAsync(balance, st->balance.ptr, bytes, hipMemcpyDeviceToHost, st->s);
  if (e == hipSuccess && start && bytes) e = hipMemcpyAsync(start, st->start.ptr, bytes, hipMemcpyDeviceToHost, st->s);
  if (e == hipSuccess && end && bytes) e = hipMemcpyAsync(end, st->end.ptr, bytes, hipMemcpyDeviceToHost, st->s);
  if (e == hipSuccess) e = hipStreamSynchronize(st->s);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_state_download");
}

/* casper/validator.go:45-77 on the mirror (see pz_validator_indices). */
int pz_state_validator_indices(pz_state* st, uint64_t dynasty, int kind, uint32_t* out, uint64_t* count) {
  if (!count) return fail(PZ_EINVAL, "count is null");
  if (kind < PZ_KIND_ACTIVE || kind > PZ_KIND_QUEUED) return fail(PZ_EINVAL, "bad kind %d", kind);
  *count = 0;
  int rc = lock(st);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(st->mu);
  if (!st->n) return PZ_OK;
  if (!out) return fail(PZ_EINVAL, "out is null");
  EpochArgs a;
  if ((rc = prepare(st, a, kind)) || (rc = set_scalars(st, dynasty, 0))) return rc;
  hipError_t e = launch_epoch_count(a, true, false, false, st->s);
  if (e == hipSuccess) e = launch_epoch_compact(a, true, st->s);
  uint64_t scal[kScal];
  if (e == hipSuccess) e = hipMemcpyAsync(scal, a.scal, sizeof scal, hipMemcpyDeviceToHost, st->s);
  if (e == hipSuccess) e = hipStreamSynchronize(st->s);
  if (e != hipSuccess) return hip_fail(e, "pz_state_validator_indices");
  *count = st->n - scal[kNoMatch];
  e = hipMemcpyAsync(out, a.act_list, *count * 4, hipMemcpyDeviceToHost, st->s);
  if (e == hipSuccess) e = hipStreamSynchronize(st->s);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "D2H indices");
}

/* casper/incentives.go:14-32 on the mirror's balances, in place (see pz_calculate_rewards);
 * only the pending attestations' bitfields cross PCIe. */
int pz_state_calculate_rewards(pz_state* st, uint64_t dynasty, uint64_t total_deposit, const uint8_t* bits,
                               const uint64_t* boffs, uint64_t natt, int* applied) {
  if (applied) *applied = 0;
  int rc = lock(st);
  if (rc) return rc;
  if (natt && (rc = check_csr(boffs, natt, "bitfield"))) return rc;
  if (natt > 0xffffffffull) return fail(PZ_EINVAL, "too many attestations");
  std::lock_guard<std::mutex> lk(st->mu);
  EpochArgs a;
  if ((rc = prepare(st, a, PZ_KIND_ACTIVE)) || (rc = set_scalars(st, dynasty, total_deposit))) return rc;
  std::vector<uint64_t> rb;
  hipError_t e = hipSuccess;
  if (natt) {
    rb = rebase(boffs, natt);
    if (rb[natt] && !bits) return fail(PZ_EINVAL, "bits is null");
    if ((rc = st->aux[0].reserve(rb[natt] + 16)) || (rc = st->aux[1].reserve((natt + 1) * 8))) return rc;
    if (rb[natt]) e = hipMemcpyAsync(st->aux[0].ptr, bits + boffs[0], rb[natt], hipMemcpyHostToDevice, st->s);
    if (e == hipSuccess) e = hipMemcpyAsync(st->aux[1].ptr, rb.data(), (natt + 1) * 8, hipMemcpyHostToDevice, st->s);
    a.natt = (uint32_t)natt;
    a.bits = (const uint8_t*)st->aux[0].ptr;
    a.boffs = (const uint64_t*)st->aux[1].ptr;
    a.max_inst_bytes = rb[natt];
  }
  if (e == hipSuccess) e = launch_epoch_count(a, true, true, false, st->s);
  if (e == hipSuccess) e = launch_epoch_compact(a, false, st->s);
  // rewards only when no panic: the reward kernel itself leaves balances untouched then
  if (e == hipSuccess) e = launch_epoch_reward(a, st->s);
  uint64_t scal[kScal];
  if (e == hipSuccess) e = hipMemcpyAsync(scal, a.scal, sizeof scal, hipMemcpyDeviceToHost, st->s);
  if (e == hipSuccess) e = hipStreamSynchronize(st->s);  // rb and scal are host locals
  if (e != hipSuccess) return hip_fail(e, "pz_state_calculate_rewards");
  const uint64_t dep = scal[kPop] * PZ_DEFAULT_BALANCE;
  const bool thr = dep * 3ull >= total_deposit * 2ull;
  if (thr && scal[kNact] > 0 && scal[kErrRwd])
    return fail(PZ_EINDEX, natt ? "CheckBit index out of range (incentives.go:23)"
                                : "index out of range [-1]: no attestations (incentives.go:23)");
  if (applied) *applied = scal[kApplied] ? 1 : 0;
  return PZ_OK;
}

/* blockchain/core.go:459-464 on the mirror: the total balance of the active validators. */
int pz_state_active_balance(pz_state* st, uint64_t dynasty, uint64_t* total) {
  if (!total) return fail(PZ_EINVAL, "total is null");
  *total = 0;
  int rc = lock(st);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(st->mu);
  if (!st->n) return PZ_OK;
  EpochArgs a;
  // a reward pass whose threshold cannot hold (total_deposit = 2^63 + 1: 2 * it wraps to 2,
  // and pop 0 gives 0 >= 2 false) adds nothing and sums the active balances
  if ((rc = prepare(st, a, PZ_KIND_ACTIVE)) || (rc = set_scalars(st, dynasty, (1ull << 63) + 1))) return rc;
  hipError_t e = launch_epoch_count(a, true, false, false, st->s);
  if (e == hipSuccess) e = launch_epoch_compact(a, false, st->s);
  if (e == hipSuccess) e = launch_epoch_reward(a, st->s);
  uint64_t scal[kScal];
  if (e == hipSuccess) e = hipMemcpyAsync(scal, a.scal, sizeof scal, hipMemcpyDeviceToHost, st->s);
  if (e == hipSuccess) e = hipStreamSynchronize(st->s);
  if (e != hipSuccess) return hip_fail(e, "pz_state_active_balance");
  *total = scal[kNextBal];
  return PZ_OK;
}

void pz_state_free(pz_state* st) { delete st; }

}  // extern "C"
