// pz_epoch_state: the device-resident, validator-range-sharded epoch transition behind the
// C ABI (include/prysm_hip.h, "multi-GPU").  B independent instances of the data-parallel
// part of stateRecalc (blockchain/core.go:433-464): processCrosslinks tallies + winners
// (:502-558), GetAttestersTotalDeposit (casper/validator.go:93-102), CalculateRewards
// (casper/incentives.go:14-32) and the next-cycle total (core.go:459-464).
//
// Each rank of the communicator owns the 64-aligned validator range [lo, hi) of every
// instance (SoA, instance-major, in its GPU's HBM) and the committee members that fall in it,
// each with its position in the full committee (its bitfield bit).  A step is
//
//   count (local partial sums)  -> all-reduce {scal, vote, total}            (RCCL, u64 sum)
//   [some validator inactive: all-gather the active masks -> global compacted list]
//   finish (winners, rewards on the local range, partial next-cycle total)
//                               -> all-reduce of the next-cycle totals
//
// and the B instances are split in two parts so that one part's collectives run on the
// collective stream while the other part's kernels run on the compute stream.  Integer sums
// mod 2^64 commute, so every result is bit-exact for any reduction order.  The same code runs
// every world size; at world 1 the collectives are skipped.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "comm.h"
#include "epoch.h"
#include "runtime.h"

using namespace pz;

namespace {

struct Part {
  uint32_t i0 = 0, B = 0;
  uint64_t* red[2] = {nullptr, nullptr};  // ping-pong {scal[B][8], vote[B*natt], total[B*natt]}
  int cur = 0;
  uint64_t* results = nullptr;            // the red buffer of the last completed step
  uint32_t* win_results = nullptr;        // FusedArgs.win_in_wave: the winners of the last step
  uint64_t* mask_send = nullptr;          // [B][sw]
  uint64_t* gmask = nullptr;              // [world][B][sw]
  uint32_t* gblk = nullptr;               // [B][vblocks(N)]
  uint64_t* nb = nullptr;                 // [B] next-cycle totals, contiguous for the all-reduce
  hipEvent_t ev_red = nullptr, ev_gather = nullptr, ev_nb = nullptr;
  EpochArgs a;
  FusedArgs f;                            // one-pass step, one instance (pz_epoch_one_kernel)
  bool window = false;                    // one-pass step, the window pass (epoch_window.hip)
  WinArgs w;
};

struct Shard {
  int dev = 0, grank = 0;
  hipStream_t s = nullptr;    // where steps are enqueued: own, or a caller's (bind_stream)
  hipStream_t own = nullptr;  // created and destroyed by the state
  uint64_t lo = 0, hi = 0, n = 0, wl = 0;
  uint64_t np = 0;  // row stride of the validator arrays: n, or n rounded up to even for the
                    // one-pass step (its 16-B pairs start at even local indices of every row)
  std::vector<void*> allocs;
  Part part[2];
};

}  // namespace

struct pz_epoch_state {
  pz_comm* comm = nullptr;  // null: one device, world 1
  int world = 1;
  uint32_t B = 0, natt = 0, nrec = 0, nparts = 1;
  uint64_t N = 0, sw = 0, ncomm = 0;
  bool general = false, all_active = true;
  bool co = false;                 // committee-order layout (see pz_epoch_batch.co_index)
  bool fused = false;              // one-pass step (epoch.h "one-pass epoch") on that layout
  std::vector<uint32_t> co_inv;    // storage position -> validator index (committee order)
  uint64_t steps = 0;
  uint64_t tallied = ~0ull;        // the step whose vote/total pz_epoch_state_tallies completed
  // FusedArgs.bal32 (some part holds its balances as u32 offsets): steps left before the
  // offsets are re-based (each step moves an offset by at most 1; see kBal32Window)
  bool b32 = false;
  uint64_t b32_left = 0;
  pz_epoch_options opts{};
  std::vector<Shard> sh;
  ~pz_epoch_state();
};

namespace {

template <typename T>
int dalloc(Shard& s, T** p, size_t count, bool zero = true) {
  const size_t bytes = (count ? count : 1) * sizeof(T) + 16;
  hipError_t e = hipMalloc((void**)p, bytes);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc (epoch state)");
  s.allocs.push_back(*p);
  if (zero && (e = hipMemset(*p, 0, bytes)) != hipSuccess) return hip_fail(e, "hipMemset (epoch state)");
  return PZ_OK;
}

template <typename T>
int upload(Shard& s, T** p, const T* host, size_t count) {
  int rc = dalloc(s, p, count, false);
  if (rc || !count) return rc;
  hipError_t e = hipMemcpy(*p, host, count * sizeof(T), hipMemcpyHostToDevice);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "hipMemcpy H2D (epoch state)");
}

int upload_into(uint8_t* d, const uint8_t* host, size_t bytes) {
  if (!bytes) return PZ_OK;
  hipError_t e = hipMemcpy(d, host, bytes, hipMemcpyHostToDevice);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "hipMemcpy H2D (epoch state)");
}

// Rows [0, B) x columns [lo, hi) of a host [B][N] u64 array -> device [B][hi-lo].
int upload_range(Shard& s, uint64_t** p, const uint64_t* host, uint32_t B, uint64_t N) {
  int rc = dalloc(s, p, (size_t)B * s.n, false);
  if (rc || !s.n) return rc;
  hipError_t e = hipMemcpy2D(*p, s.n * 8, host + s.lo, N * 8, s.n * 8, B, hipMemcpyHostToDevice);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "hipMemcpy2D H2D (epoch state)");
}

// Committee order: rows [0, B) of a host [B][N] array, the validators stored at positions
// [lo, hi) (inv[p] = the validator at position p) -> device [B][hi-lo].
int upload_perm(Shard& s, uint64_t** p, const uint64_t* host, uint32_t B, uint64_t N, const uint32_t* inv) {
  int rc = dalloc(s, p, (size_t)B * s.np, false);
  if (rc || !s.n) return rc;
  std::vector<uint64_t> tmp((size_t)B * s.np, 0);  // rows of np (the pad element stays 0)
  for (uint64_t b = 0; b < B; ++b)
    for (uint64_t q = 0; q < s.n; ++q) tmp[b * s.np + q] = host[b * N + inv[s.lo + q]];
  hipError_t e = hipMemcpy(*p, tmp.data(), tmp.size() * 8, hipMemcpyHostToDevice);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "hipMemcpy H2D (epoch state)");
}

// The one-pass stream's {start, end} column (FusedArgs.se): rows of np, the positions [lo, hi)
// of committee order, each bound saturated to 32 bits (pad elements: {0, 0}).
int upload_se(Shard& s, uint2** p, const uint64_t* start, const uint64_t* end, uint32_t B, uint64_t N,
              const uint32_t* inv) {
  int rc = dalloc(s, p, (size_t)B * s.np, false);
  if (rc || !s.n) return rc;
  auto sat = [](uint64_t x) { return (uint32_t)std::min<uint64_t>(x, 0xFFFFFFFFull); };
  std::vector<uint2> tmp((size_t)B * s.np, make_uint2(0, 0));
  for (uint64_t b = 0; b < B; ++b)
    for (uint64_t q = 0; q < s.n; ++q) {
      const uint64_t v = b * N + inv[s.lo + q];
      tmp[b * s.np + q] = make_uint2(sat(start[v]), sat(end[v]));
    }
  hipError_t e = hipMemcpy(*p, tmp.data(), tmp.size() * 8, hipMemcpyHostToDevice);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "hipMemcpy H2D (epoch state)");
}

// FusedArgs.se16: the same positions, each bound saturated to 16 bits, {start | end << 16}.
int upload_se16(Shard& s, uint32_t** p, const uint64_t* start, const uint64_t* end, uint32_t B, uint64_t N,
                const uint32_t* inv) {
  int rc = dalloc(s, p, (size_t)B * s.np, false);
  if (rc || !s.n) return rc;
  auto sat = [](uint64_t x) { return (uint32_t)std::min<uint64_t>(x, 0xFFFFull); };
  std::vector<uint32_t> tmp((size_t)B * s.np, 0u);
  for (uint64_t b = 0; b < B; ++b)
    for (uint64_t q = 0; q < s.n; ++q) {
      const uint64_t v = b * N + inv[s.lo + q];
      tmp[b * s.np + q] = sat(start[v]) | (sat(end[v]) << 16);
    }
  hipError_t e = hipMemcpy(*p, tmp.data(), tmp.size() * 4, hipMemcpyHostToDevice);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "hipMemcpy H2D (epoch state)");
}

// FusedArgs.bal32: an instance's balances are held as u32 offsets from base = min - 2^30 when
// max - min < 2^30, so every offset starts in [2^30, 2^31).  A step adds or subtracts
// PZ_ATTESTER_REWARD (1) at most, so after kBal32Period steps the offsets are still inside
// [2^30 - 2^29, 2^31 + 2^29), well inside u32, and the state re-bases them then (bal32_rebase).
// Arithmetic is mod 2^64 throughout (base + offset), so a balance that wraps below zero, as
// Go's uint64 does, stays exact; the re-base then finds the spread too wide and returns that
// part to the u64 column.
constexpr uint64_t kBal32Window = 1ull << 30;
constexpr uint64_t kBal32Period = 1ull << 29;
static uint64_t bal32_period(uint64_t opt, bool narrow) {  // pz_epoch_options.rebase_period (tests: the re-base)
  const uint64_t cap = narrow ? kNarrowPeriod : kBal32Period;  // (narrow tallies: epoch.h WinArgs.narrow)
  return opt && opt < cap ? opt : cap;
}

static bool any_narrow(const pz_epoch_state* st);

// The base of every instance of [i0, i0 + Bp) over the values vals(b, q), q < n; false if some
// instance's spread is kBal32Window or more.
template <typename F>
static bool bal32_bases(uint64_t Bp, uint64_t n, F vals, std::vector<uint64_t>& base, uint64_t* spread = nullptr) {
  base.assign(Bp, 0);
  uint64_t sp = 0;
  for (uint64_t b = 0; b < Bp; ++b) {
    uint64_t lo = ~0ull, hi = 0;
    for (uint64_t q = 0; q < n; ++q) {
      const uint64_t v = vals(b, q);
      lo = std::min(lo, v);
      hi = std::max(hi, v);
    }
    if (n && hi - lo >= kBal32Window) return false;
    base[b] = (n ? lo : 0) - kBal32Window;
    sp = std::max(sp, n ? hi - lo : 0);
  }
  if (spread) *spread = sp;
  return true;
}

// Upload the offsets [Bp][np] (pad positions 0) and bases of one part.
template <typename F>
static int bal32_upload(Shard& s, Part& q, F vals, const std::vector<uint64_t>& base, bool alloc) {
  std::vector<uint32_t> off((size_t)q.B * s.np, 0u);
  for (uint64_t b = 0; b < q.B; ++b)
    for (uint64_t p = 0; p < s.n; ++p) off[b * s.np + p] = (uint32_t)(vals(b, p) - base[b]);
  if (alloc) {
    uint64_t* d_base = nullptr;
    int rc = dalloc(s, &q.f.bal32, off.size(), false);
    if (!rc) rc = dalloc(s, &d_base, q.B, false);
    if (rc) return rc;
    q.f.bal32_base = d_base;
  }
  hipError_t e = hipMemcpy(q.f.bal32, off.data(), off.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(const_cast<uint64_t*>(q.f.bal32_base), base.data(), base.size() * 8, hipMemcpyHostToDevice);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "hipMemcpy H2D (epoch state, u32 balances)");
}

// The part's balances as u64 [Bp][n] on the host (from the offsets or the u64 column).
static int part_balances(const Shard& s, const Part& q, uint64_t* out, uint64_t ld) {
  hipError_t e;
  if (!q.f.bal32) {
    e = hipMemcpy2D(out, ld * 8, q.a.balance, s.np * 8, s.n * 8, q.B, hipMemcpyDeviceToHost);
    return e == hipSuccess ? PZ_OK : hip_fail(e, "epoch state results D2H");
  }
  std::vector<uint32_t> off((size_t)q.B * s.np);
  std::vector<uint64_t> base(q.B);
  e = hipMemcpy(off.data(), q.f.bal32, off.size() * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(base.data(), q.f.bal32_base, base.size() * 8, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(e, "epoch state results D2H (u32 balances)");
  for (uint64_t b = 0; b < q.B; ++b)
    for (uint64_t p = 0; p < s.n; ++p) out[b * ld + p] = base[b] + off[b * s.np + p];
  return PZ_OK;
}

// Re-base every part's offsets (or, if an instance's spread has grown to the window, return
// the part to the u64 column).  Rare: once per kBal32Period steps.
static int bal32_rebase(pz_epoch_state* st);


uint64_t shard_words(uint64_t N, int world) { return std::max<uint64_t>(1, (N + 64ull * world - 1) / (64ull * world)); }

int step_world1(pz_epoch_state* st) {
  for (Shard& s : st->sh) {
    (void)hipSetDevice(s.dev);
    for (uint32_t p = 0; p < st->nparts; ++p) {
      EpochArgs& a = s.part[p].a;
      if (st->fused && epoch_one_enabled(s.part[p].f)) {  // one instance: the single-launch step
        hipError_t e = launch_epoch_one(a, s.part[p].f, s.s);
        if (e != hipSuccess) return hip_fail(e, "epoch step (single launch)");
        continue;
      }
      if (st->fused && s.part[p].window) {  // the window pass: one launch
        Part& q = s.part[p];
        q.w.bal32 = q.f.bal32;  // (a re-base may have returned the part to the u64 column)
        q.w.bal32_base = q.f.bal32_base;
        hipError_t e = launch_epoch_window(a, q.w, s.s);
        if (e != hipSuccess) return hip_fail(e, "epoch step (window pass)");
        continue;
      }
      hipError_t e = launch_epoch_count(a, true, true, a.natt != 0, s.s);
      if (e == hipSuccess) e = launch_epoch_mid(a, a.natt && st->nrec, true, s.s);
      if (e == hipSuccess) e = launch_epoch_reward(a, s.s);
      if (e != hipSuccess) return hip_fail(e, "epoch step");
    }
  }
  return PZ_OK;
}

void flip(pz_epoch_state* st) {
  for (Shard& s : st->sh)
    for (uint32_t p = 0; p < st->nparts; ++p) {
      Part& q = s.part[p];
      q.results = q.red[q.cur];
      q.cur ^= 1;
      if (q.f.win_in_wave) {  // the winners ping-pong too (the step just enqueued wrote a.winner)
        q.win_results = q.a.winner;
        std::swap(q.a.winner, q.f.winner_next);
      }
      if (q.window) {
        q.win_results = q.a.winner;
        std::swap(q.a.winner, q.w.winner_next);
        std::swap(q.w.pacc, q.w.pacc_next);  // (the step just enqueued zeroed pacc_next)
      }
      const uint64_t Bp = q.B, natt = st->natt;
      q.a.scal = q.red[q.cur];
      q.a.vote = q.red[q.cur] + Bp * kScal;
      q.a.total = q.red[q.cur] + Bp * kScal + Bp * natt;
      q.a.scal_next = q.red[q.cur ^ 1];
      const uint64_t pre = Bp * kScal + 2 * Bp * natt;  // after {scal, vote, total}: not all-reduced
      q.f.pre = q.red[q.cur] + pre;
      q.f.pre_next = q.red[q.cur ^ 1] + pre;
      q.f.vote_next = q.red[q.cur ^ 1] + Bp * kScal;
      q.f.total_next = q.red[q.cur ^ 1] + Bp * kScal + Bp * natt;
      if (q.window && st->world > 1) {  // non-owned attestations' tallies must read zero
        q.w.vote_next = q.f.vote_next;
        q.w.total_next = q.f.total_next;
      }
    }
}

int wait(Shard& s, hipEvent_t ev) {
  (void)hipSetDevice(s.dev);
  hipError_t e = hipStreamWaitEvent(s.s, ev, 0);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "hipStreamWaitEvent");
}

// One-pass step at N > 1.  The ranks' ranges are committee-aligned, so every committee's
// tallies are complete on one rank: per part, pre + fused + the winners each rank owns, then
// ONE grouped collective -- a u64 sum of the per-instance scalars (partial next-cycle totals,
// flags) and a u32 minimum of the proposed winners -- while the next part computes.  The
// per-attestation vote/total stay on their owner ranks (pz_epoch_state_tallies completes
// them on demand): 8 B x (8 + nrec/2) per instance cross xGMI instead of 16 B per attestation.
int step_sharded_fused(pz_epoch_state* st) {
  pz_comm* c = st->comm;
  const int L = (int)st->sh.size();
  std::vector<hipStream_t> streams(L);
  std::vector<uint64_t*> sbufs(L);
  std::vector<uint32_t*> mbufs(L);
  std::vector<hipEvent_t> evs(L);
  for (int i = 0; i < L; ++i) streams[i] = st->sh[i].s;
  int rc;
  for (uint32_t p = 0; p < st->nparts; ++p) {
    for (int i = 0; i < L; ++i) {
      Shard& s = st->sh[i];
      Part& q = s.part[p];
      (void)hipSetDevice(s.dev);
      q.w.bal32 = q.f.bal32;
      q.w.bal32_base = q.f.bal32_base;
      hipError_t e = launch_epoch_window(q.a, q.w, s.s);
      if (e != hipSuccess) return hip_fail(e, "epoch one-pass (window pass)");
      sbufs[i] = q.red[q.cur];
      mbufs[i] = q.a.winner;
      evs[i] = q.ev_red;
    }
    const uint64_t Bp = st->sh[0].part[p].B;
    if ((rc = c->allreduce_sum_min(sbufs.data(), Bp * kScal, mbufs.data(), st->nrec ? Bp * st->nrec : 0,
                                   streams.data(), evs.data())))
      return rc;
  }
  for (uint32_t p = 0; p < st->nparts; ++p)
    for (int i = 0; i < L; ++i)
      if ((rc = wait(st->sh[i], st->sh[i].part[p].ev_red))) return rc;
  return PZ_OK;
}

int step_sharded(pz_epoch_state* st) {
  if (st->fused) return step_sharded_fused(st);
  pz_comm* c = st->comm;
  const int L = (int)st->sh.size();
  std::vector<hipStream_t> streams(L);
  std::vector<uint64_t*> bufs(L);
  std::vector<const void*> sends(L);
  std::vector<void*> recvs(L);
  std::vector<hipEvent_t> evs(L);
  for (int i = 0; i < L; ++i) streams[i] = st->sh[i].s;
  int rc;
  // pass 1 of every part, each followed by the all-reduce of its partial sums
  for (uint32_t p = 0; p < st->nparts; ++p) {
    for (int i = 0; i < L; ++i) {
      Shard& s = st->sh[i];
      (void)hipSetDevice(s.dev);
      hipError_t e = launch_epoch_count(s.part[p].a, true, true, s.part[p].a.natt != 0, s.s);
      if (e != hipSuccess) return hip_fail(e, "pz_epoch_count_kernel");
      bufs[i] = s.part[p].red[s.part[p].cur];
      evs[i] = s.part[p].ev_red;
    }
    const uint64_t Bp = st->sh[0].part[p].B;
    if ((rc = c->allreduce_u64(bufs.data(), Bp * kScal + 2 * Bp * st->natt, streams.data(), evs.data()))) return rc;
  }
  // pass 2 of every part (part 0's finish overlaps part 1's all-reduce)
  for (uint32_t p = 0; p < st->nparts; ++p) {
    for (int i = 0; i < L; ++i)
      if ((rc = wait(st->sh[i], st->sh[i].part[p].ev_red))) return rc;
    if (st->general) {  // rank != index: every rank rebuilds the global compacted active list
      for (int i = 0; i < L; ++i) {
        Shard& s = st->sh[i];
        Part& q = s.part[p];
        (void)hipSetDevice(s.dev);
        if (s.wl) {
          hipError_t e = hipMemcpy2DAsync(q.mask_send, st->sw * 8, q.a.act_mask, s.wl * 8, s.wl * 8, q.B,
                                          hipMemcpyDeviceToDevice, s.s);
          if (e != hipSuccess) return hip_fail(e, "active-mask pack");
        }
        sends[i] = q.mask_send;
        recvs[i] = q.gmask;
        evs[i] = q.ev_gather;
      }
      if ((rc = c->allgather(sends.data(), recvs.data(), (size_t)st->sh[0].part[p].B * st->sw * 8, streams.data(),
                             evs.data())))
        return rc;
      for (int i = 0; i < L; ++i) {
        Shard& s = st->sh[i];
        Part& q = s.part[p];
        if ((rc = wait(s, q.ev_gather))) return rc;
        hipError_t e = launch_epoch_gather_compact(q.a, q.gmask, st->sw, q.gblk, s.s);
        if (e != hipSuccess) return hip_fail(e, "pz_epoch_gcompact_kernel");
      }
    }
    for (int i = 0; i < L; ++i) {
      Shard& s = st->sh[i];
      Part& q = s.part[p];
      (void)hipSetDevice(s.dev);
      hipError_t e = launch_epoch_mid(q.a, q.a.natt && st->nrec, false, s.s);
      if (e == hipSuccess) e = launch_epoch_reward(q.a, s.s);
      // the next-cycle totals (column kNextBal of scal) made contiguous for the all-reduce
      if (e == hipSuccess)
        e = hipMemcpy2DAsync(q.nb, 8, q.a.scal + kNextBal, kScal * 8, 8, q.B, hipMemcpyDeviceToDevice, s.s);
      if (e != hipSuccess) return hip_fail(e, "epoch finish");
      bufs[i] = q.nb;
      evs[i] = q.ev_nb;
    }
    if ((rc = c->allreduce_u64(bufs.data(), st->sh[0].part[p].B, streams.data(), evs.data()))) return rc;
  }
  for (uint32_t p = 0; p < st->nparts; ++p)
    for (int i = 0; i < L; ++i) {
      Shard& s = st->sh[i];
      Part& q = s.part[p];
      if ((rc = wait(s, q.ev_nb))) return rc;
      hipError_t e = hipMemcpy2DAsync(q.a.scal + kNextBal, kScal * 8, q.nb, 8, 8, q.B, hipMemcpyDeviceToDevice, s.s);
      if (e != hipSuccess) return hip_fail(e, "next-cycle total unpack");
    }
  return PZ_OK;
}

int check_host(const pz_epoch_host* h) {
  if (!h) return fail(PZ_EINVAL, "host description is null");
  if (!h->ninst || !h->nval) return fail(PZ_EINVAL, "empty epoch (ninst %u, nval %llu)", h->ninst,
                                          (unsigned long long)h->nval);
  if (!h->balance || !h->start || !h->end || !h->dynasty || !h->total_deposit)
    return fail(PZ_EINVAL, "missing validator arrays");
  if (h->ninst > 65535 || (uint64_t)h->ninst * h->natt >= (1ull << 32) || h->nval >= (1ull << 32))
    return fail(PZ_EINVAL, "more than 65535 instances, 2^32 attestations or 2^32 validators");
  if (h->natt) {
    if (!h->bits || !h->boffs || !h->att_comm || !h->att_shard || !h->committee || !h->coffs)
      return fail(PZ_EINVAL, "missing attestation / committee arrays");
    if (h->boffs[0] != 0) return fail(PZ_EINVAL, "boffs[0] must be 0");
    int rc = check_csr(h->boffs, (uint64_t)h->ninst * h->natt, "bitfield");
    if (rc || (rc = check_csr(h->coffs, h->ncomm, "committee"))) return rc;
    if (h->coffs[0] != 0) return fail(PZ_EINVAL, "coffs[0] must be 0");
    for (uint64_t i = 0; i < (uint64_t)h->ninst * h->natt; ++i)
      if (h->att_comm[i] >= h->ncomm) return fail(PZ_EINVAL, "attestation %llu names committee %u of %llu",
                                                  (unsigned long long)i, h->att_comm[i], (unsigned long long)h->ncomm);
  }
  if (h->nrec && !h->rec_dynasty) return fail(PZ_EINVAL, "missing crosslink record dynasties");
  return PZ_OK;
}

// Rank r's first storage position in the committee-order one-pass step: the committee start
// nearest to r*N/world (so every committee, and its tallies, lives on one rank).
uint64_t committee_boundary(const pz_epoch_host* h, uint64_t r, int world, uint64_t N) {
  if (r == 0) return 0;
  if (r >= (uint64_t)world) return N;
  const uint64_t t = N * r / (uint64_t)world;
  const uint64_t* e = h->coffs + h->ncomm + 1;
  const uint64_t* it = std::lower_bound(h->coffs, e, t);
  uint64_t b = it == e ? N : *it;
  if (it != h->coffs && t - *(it - 1) < b - t) b = *(it - 1);
  // monotone in r: never before the previous rank's boundary
  return std::max<uint64_t>(b, r > 1 ? committee_boundary(h, r - 1, world, N) : 0);
}

// The step a pz_epoch_state takes for h (host only; pz_epoch_plan exports it).
struct Plan {
  bool all_active = true;  // every validator active in every instance
  bool co = false;         // committee-order layout (see pz_epoch_batch.co_index)
  bool fused = false;      // one-pass step on that layout
};
Plan plan_layout(const pz_epoch_host* h) {
  Plan p;
  const uint64_t N = h->nval;
  for (uint64_t b = 0; b < h->ninst && p.all_active; ++b) {
    const uint64_t d = h->dynasty[b];
    for (uint64_t v = 0; v < N; ++v) {
      const uint64_t k = b * N + v;
      if (!(h->start[k] <= d && d < h->end[k])) {
        p.all_active = false;
        break;
      }
    }
  }
  // Committee order when every validator is active and the committees partition [0, N):
  // the crosslink tallies then stream contiguous balances instead of gathering them.
  if (p.all_active && h->natt && h->layout != PZ_LAYOUT_INDEX && h->coffs[h->ncomm] == N) {
    std::vector<uint8_t> seen(N, 0);
    bool part = true;
    for (uint64_t k = 0; k < N && part; ++k) {
      const uint32_t v = h->committee[k];
      part = v < N && !seen[v];
      if (part) seen[v] = 1;
    }
    p.co = part;
  }
  // One pass needs no shard panic (it depends on the tallies, which the one pass forms while
  // it rewards).
  if (p.co && h->layout == PZ_LAYOUT_AUTO) {
    p.fused = true;
    for (uint64_t i = 0; i < (uint64_t)h->ninst * h->natt && p.fused; ++i) p.fused = h->att_shard[i] < h->nrec;
  }
  return p;
}

// Global rank r's storage positions [lo, hi): 64-aligned validator ranges, or committee-
// aligned ones for the sharded one-pass step (no committee straddles two ranks).
void shard_range(const pz_epoch_host* h, const Plan& p, int r, int world, uint64_t* lo, uint64_t* hi) {
  const uint64_t N = h->nval, span = 64 * shard_words(N, world);
  *lo = std::min<uint64_t>(N, (uint64_t)r * span);
  *hi = std::min<uint64_t>(N, (uint64_t)(r + 1) * span);
  if (p.fused && world > 1) {
    *lo = committee_boundary(h, (uint64_t)r, world, N);
    *hi = committee_boundary(h, (uint64_t)r + 1, world, N);
  }
}

// The committee CSR restricted to members in [lo, hi) (plus, on global rank 0, members >=
// N, whose processCrosslinks panic that rank raises), each with its position in its full
// committee.
void local_committees(const pz_epoch_host* h, uint64_t lo, uint64_t hi, bool keep_oob, std::vector<uint32_t>& mem,
                      std::vector<uint64_t>& offs, std::vector<uint32_t>& pos) {
  offs.assign(h->ncomm + 1, 0);
  for (uint64_t c = 0; c < h->ncomm; ++c) {
    for (uint64_t k = h->coffs[c]; k < h->coffs[c + 1]; ++k) {
      const uint32_t v = h->committee[k];
      if ((v >= lo && v < hi) || (keep_oob && v >= h->nval)) {
        mem.push_back(v);
        pos.push_back((uint32_t)(k - h->coffs[c]));
      }
    }
    offs[c + 1] = mem.size();
  }
}

}  // namespace

// The window pass's plan for one part of one rank (epoch.h WinArgs): the rank's committees
// (those whose first position lies in [lo, hi); the last rank also takes the empty ones at N)
// split into R ranges of about equal positions, R = CUs / B (one block per CU), each range's
// committee pieces with, per instance, the piece's committee and attestation facts (so the
// kernel reads them beside the stream: no committee table, no vote bitmap), and the LDS
// carve-up.  The last bitfield goes into LDS when the block still fits the CU's 160 KiB.
static int plan_window(pz_epoch_state* st, const pz_epoch_host* h, Shard& s, Part& q, const std::vector<uint32_t>& catt_offs,
                const std::vector<uint32_t>& catt) {
  const uint64_t Bp = q.B, i0 = q.i0, natt = st->natt, nc1 = st->ncomm + 1, N = st->N;
  const uint64_t* coffs = h->coffs;
  const uint64_t cg0 = std::lower_bound(coffs, coffs + st->ncomm, s.lo) - coffs;
  const uint64_t cg1 = s.hi >= N ? st->ncomm : (uint64_t)(std::lower_bound(coffs, coffs + st->ncomm, s.hi) - coffs);
  const uint32_t nlc = (uint32_t)(cg1 - cg0);
  std::vector<uint32_t> lcs(nlc + 1);
  for (uint32_t k = 0; k <= nlc; ++k) lcs[k] = (uint32_t)((k < nlc ? coffs[cg0 + k] : s.hi) - s.lo);
  // per instance: the attestation columns
  std::vector<uint32_t> csz((size_t)Bp * natt);
  for (uint64_t b = 0; b < Bp; ++b) {
    const uint64_t gb = (i0 + b) * natt;
    for (uint64_t g = 0; g < natt; ++g) {
      const uint32_t c = h->att_comm[gb + g];
      csz[b * natt + g] = (uint32_t)(coffs[c + 1] - coffs[c]);
    }
    if (h->boffs[gb + natt] - (h->boffs[gb] & ~15ull) >= (1ull << 28))
      return fail(PZ_EINVAL, "window pass: an instance's bitfields exceed 256 MiB");
  }
  // the last bitfield's LDS copy: from (lb & ~15) to the instance's end, 16-B chunks
  uint64_t lbf = 0;
  for (uint64_t b = 0; b < Bp; ++b) {
    const uint64_t gb = (i0 + b) * natt, lb = h->boffs[gb + natt - 1], pend = h->boffs[gb + natt];
    lbf = std::max<uint64_t>(lbf, (pend - (lb & ~15ull) + 15) & ~15ull);
  }
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s.dev);
  uint32_t R = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(std::max<uint32_t>(nlc, 1), ((uint64_t)cus + Bp - 1) / Bp));
  std::vector<uint4> rdesc;
  std::vector<uint4> pieces;  // {first position, positions, committee (local), range}
  WinArgs& w = q.w;
  std::memset(&w, 0, sizeof w);
  constexpr size_t kLdsMax = 160 * 1024 - 1024;  // (the kernel's static reduction slots)
  auto catt_at = [&](uint64_t b, uint64_t c) { return catt_offs[(i0 + b) * nc1 + c]; };
  for (;;) {
    rdesc.assign(R, make_uint4(0, 0, 0, 0));
    pieces.clear();
    uint32_t c = 0, maxc = 0, maxk = 0;
    for (uint32_t r = 0; r < R; ++r) {
      const uint64_t t = (uint64_t)lcs[nlc] * (r + 1) / R;
      uint32_t c1 = c;
      if (r + 1 == R) {
        c1 = nlc;
      } else {
        while (c1 < nlc && lcs[c1 + 1] <= t) ++c1;
        if (c1 == c && c1 < nlc) ++c1;  // at least one committee per range while they last
      }
      const uint32_t pb = (uint32_t)pieces.size();
      // pieces: a committee's first from its first position to the next 256 boundary after its
      // rounded-down start, then 256-position runs from 4-aligned starts
      for (uint32_t cc = c; cc < c1; ++cc) {
        const uint64_t cs = lcs[cc], ce = lcs[cc + 1];
        for (uint64_t ps = cs; ps < ce;) {
          const uint64_t pe = std::min<uint64_t>(ce, (ps & ~3ull) + 256);
          pieces.push_back(make_uint4((uint32_t)ps, (uint32_t)(pe - ps), cc, r));
          ps = pe;
        }
      }
      rdesc[r] = make_uint4(c, c1, pb, (uint32_t)pieces.size() - pb);
      maxc = std::max(maxc, c1 - c);
      for (uint64_t b = 0; b < Bp; ++b) maxk = std::max(maxk, catt_at(b, cg0 + c1) - catt_at(b, cg0 + c));
      c = c1;
    }
    w.R = R;
    w.lds_maxc = std::max<uint32_t>(maxc, 1);
    w.lds_maxk = std::max<uint32_t>(maxk, 1);
    if ((w.lds_maxc + w.lds_maxk) & 1) ++w.lds_maxk;  // (keeps the last bitfield's copy 16-B aligned)
    w.lds_lbf = (uint32_t)lbf;
    w.dma_k = 0;
    if (window_lds_bytes(w) <= kLdsMax) {
      // the straight-line copy: the smallest instantiated count that holds every instance's copy,
      // its LDS padded to whole wave instructions, when that still fits (and no copy is empty)
      bool nonempty = true;
      for (uint64_t b = 0; b < Bp; ++b) {
        const uint64_t gb = (i0 + b) * natt;
        nonempty = nonempty && h->boffs[gb + natt] > h->boffs[gb + natt - 1];
      }
      for (uint32_t k : kWinDmaK) {
        if (!nonempty || (uint64_t)k * 16 * kWinThreads < lbf) continue;
        WinArgs t = w;
        t.lds_lbf = k * 16 * kWinThreads;
        if (window_lds_bytes(t) <= kLdsMax) w.lds_lbf = t.lds_lbf, w.dma_k = k;
        break;
      }
      break;
    }
    w.lds_lbf = 0;  // the reward bits looked up in L2 instead
    if (window_lds_bytes(w) <= kLdsMax) break;
    if (R >= nlc) return fail(PZ_EINVAL, "window pass: no range split fits the LDS");
    R = std::min<uint32_t>(nlc, 2 * R);
  }
  pieces.push_back(make_uint4(0, 0, 0, 0));  // (an empty last range's first descriptor load stays in bounds)
  const uint32_t ptot = (uint32_t)pieces.size();
  // per instance and piece (epoch.h WinArgs.pinfo) and per instance and range (WinArgs.rk)
  std::vector<uint4> pinfo(2 * (size_t)Bp * ptot, make_uint4(0, 0, 0, 0));
  std::vector<uint2> rk((size_t)Bp * R);
  for (uint64_t b = 0; b < Bp; ++b) {
    const uint64_t gb = (i0 + b) * natt, pbase = h->boffs[gb] & ~15ull;
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t k0 = catt_at(b, cg0 + rdesc[r].x);
      rk[b * R + r] = make_uint2(k0, catt_at(b, cg0 + rdesc[r].y) - k0);
    }
    for (uint32_t k = 0; k + 1 < ptot; ++k) {
      const uint4 pc = pieces[k];
      const uint32_t cc = pc.z, cr0 = rdesc[pc.w].x;
      const uint64_t c = cg0 + cc, cs = lcs[cc];
      const uint32_t na = catt_at(b, c + 1) - catt_at(b, c), kb = catt_at(b, c);
      const uint32_t kind = na == 0 ? 0 : na == 1 ? 1 : 2;
      uint32_t vbit = 0, vlim = 0;
      if (kind == 1) {  // the single attestation's bitfield: bit (position - cs), MSB first
        const uint32_t g = catt[(i0 + b) * natt + kb];
        const uint64_t bo = h->boffs[gb + g], blen = h->boffs[gb + g + 1] - bo;
        const uint64_t nb = std::min<uint64_t>(coffs[c + 1] - coffs[c], 8 * blen);
        vbit = (uint32_t)(8 * (bo - pbase) + (pc.x - cs));
        vlim = (uint32_t)std::min<uint64_t>(pc.y, nb > pc.x - cs ? nb - (pc.x - cs) : 0);
      } else if (kind == 2) {  // the per-attestation path: the committee's start and attestations' end
        vbit = (uint32_t)cs;
        vlim = catt_at(b, c + 1);
      }
      pinfo[2 * (b * ptot + k)] = make_uint4(pc.x, pc.y, cc - cr0, kind);
      pinfo[2 * (b * ptot + k) + 1] = make_uint4(kb, vbit, vlim, 0);
    }
  }
  // by catt index (one load per attestation, no catt -> column chains in the kernel): kind-2
  // pieces' bitfields {first byte - pbase, bits} (< 2^28 bytes per instance: checked above), and
  // the epilogue's {attestation, committee - its range's cr0, shard, record dynasty} (the record
  // dynasties are the state's, fixed at its creation like att_win's before; sh < nrec: plan_layout)
  std::vector<uint2> ckb((size_t)Bp * natt);
  std::vector<uint4> cq((size_t)Bp * natt, make_uint4(0, 0, 0, 0));
  bool dyn64 = false;  // (a dynasty past the saturated 32-bit compare: the high words too)
  for (uint64_t b = 0; b < Bp; ++b) dyn64 = dyn64 || h->dynasty[i0 + b] >= 0xFFFFFFFFull;
  std::vector<uint32_t> cqh(dyn64 ? (size_t)Bp * natt : 0, 0u);
  for (uint64_t b = 0; b < Bp; ++b) {
    const uint64_t gb = (i0 + b) * natt, pbase = h->boffs[gb] & ~15ull;
    for (uint64_t k = 0; k < natt; ++k) {
      const uint32_t g = catt[gb + k];
      const uint64_t bo = h->boffs[gb + g], blen = h->boffs[gb + g + 1] - bo;
      ckb[b * natt + k] = make_uint2((uint32_t)(bo - pbase), (uint32_t)(8 * blen));
    }
    for (uint32_t r = 0; r < R; ++r) {
      const uint2 kr = rk[b * R + r];
      for (uint32_t k = kr.x; k < kr.x + kr.y; ++k) {
        const uint32_t g = catt[gb + k], sh = h->att_shard[gb + g];
        const uint32_t cl = (uint32_t)(h->att_comm[gb + g] - cg0 - rdesc[r].x);
        const uint64_t rd = h->rec_dynasty[(i0 + b) * st->nrec + sh];
        cq[b * natt + k] = make_uint4(g, cl, sh, dyn64 ? (uint32_t)rd : (uint32_t)std::min<uint64_t>(rd, 0xFFFFFFFFull));
        if (dyn64) cqh[b * natt + k] = (uint32_t)(rd >> 32);
      }
    }
  }
  uint4 *d_rdesc = nullptr, *d_cq = nullptr, *d_pinfo = nullptr;
  uint2 *d_rk = nullptr, *d_ckb = nullptr;
  uint32_t *d_csz = nullptr, *d_wn = nullptr, *d_cqh = nullptr;
  uint64_t* d_pacc = nullptr;
  int rc;
  if ((rc = upload(s, &d_rdesc, rdesc.data(), rdesc.size())) || (rc = upload(s, &d_pinfo, pinfo.data(), pinfo.size())) ||
      (rc = upload(s, &d_rk, rk.data(), rk.size())) || (rc = upload(s, &d_csz, csz.data(), csz.size())) ||
      (rc = upload(s, &d_cq, cq.data(), cq.size())) || (rc = upload(s, &d_cqh, cqh.data(), cqh.size())) || (rc = upload(s, &d_ckb, ckb.data(), ckb.size())) ||
      (rc = dalloc(s, &d_wn, (size_t)Bp * std::max<uint32_t>(st->nrec, 1))) || (rc = dalloc(s, &d_pacc, 2 * (size_t)Bp)))
    return rc;
  // the meeting word's fields (epoch.h WinArgs.pacc): bits below 2^39, at most 511 blocks
  if (R > 1 && R <= 511) {
    w.pacc = d_pacc;
    w.pacc_next = d_pacc + Bp;
  }
  w.rdesc = d_rdesc;
  for (uint32_t r = 0; r < R && r < kWinKargR; ++r) w.rdk[r] = rdesc[r];
  w.pinfo = d_pinfo;
  w.ptot = ptot;
  w.rk = d_rk;
  w.cg0 = (uint32_t)cg0;
  w.catt = q.f.catt;
  w.att_csize = d_csz;
  w.cq = d_cq;
  w.cqh = dyn64 ? d_cqh : nullptr;
  w.ckb = d_ckb;
  w.se16 = q.f.se16;
  w.se = q.f.se;
  w.vstride = s.np;
  w.winner_next = d_wn;
  w.rank0 = s.grank == 0 ? 1 : 0;
  q.window = true;
  return PZ_OK;
}

pz_epoch_state::~pz_epoch_state() {
  for (Shard& s : sh) {
    (void)hipSetDevice(s.dev);
    if (s.s) (void)hipStreamSynchronize(s.s);
    if (s.own && s.own != s.s) (void)hipStreamSynchronize(s.own);
    for (void* p : s.allocs) (void)hipFree(p);
    for (Part& q : s.part) {
      if (q.ev_red) (void)hipEventDestroy(q.ev_red);
      if (q.ev_gather) (void)hipEventDestroy(q.ev_gather);
      if (q.ev_nb) (void)hipEventDestroy(q.ev_nb);
    }
    if (s.own) (void)hipStreamDestroy(s.own);
  }
}

extern "C" {

int pz_epoch_state_new(pz_comm* comm, int device, const pz_epoch_host* h, pz_epoch_state** out) {
  return pz_epoch_state_new_opts(comm, device, h, nullptr, out);
}

int pz_epoch_state_new_opts(pz_comm* comm, int device, const pz_epoch_host* h, const pz_epoch_options* opts,
                            pz_epoch_state** out) {
  if (!out) return fail(PZ_EINVAL, "out is null");
  *out = nullptr;
  int rc = check_host(h);
  if (rc) return rc;
  pz_epoch_state* st = new pz_epoch_state();
  if (opts) st->opts = *opts;
  st->comm = comm;
  st->world = comm ? comm->world : 1;
  st->B = h->ninst;
  st->N = h->nval;
  st->natt = h->natt;
  st->nrec = h->nrec;
  st->ncomm = h->ncomm;
  st->sw = shard_words(st->N, st->world);
  const Plan pl = plan_layout(h);
  st->all_active = pl.all_active;
  st->general = !st->all_active && st->world > 1;
  st->co = pl.co;
  st->fused = pl.fused;
  if (st->co) st->co_inv.assign(h->committee, h->committee + st->N);
  // attestations by committee, per instance (the one pass adds a committee's slice into each)
  std::vector<uint32_t> catt_offs, catt;
  std::vector<FusedCommittee> cinfo;
  if (st->fused) {
    const uint64_t nc1 = st->ncomm + 1;
    catt_offs.assign((size_t)st->B * nc1, 0);
    catt.resize((size_t)st->B * st->natt);
    for (uint64_t b = 0; b < st->B; ++b) {
      uint32_t* o = catt_offs.data() + b * nc1;
      const uint32_t* ac = h->att_comm + b * st->natt;
      for (uint64_t g = 0; g < st->natt; ++g) ++o[ac[g] + 1];
      for (uint64_t k = 0; k < st->ncomm; ++k) o[k + 1] += o[k];
      std::vector<uint32_t> fill(o, o + st->ncomm);
      for (uint64_t g = 0; g < st->natt; ++g) catt[b * st->natt + fill[ac[g]]++] = (uint32_t)g;
    }
    cinfo.resize((size_t)st->B * st->ncomm);
    for (uint64_t b = 0; b < st->B; ++b)
      for (uint64_t c = 0; c < st->ncomm; ++c) {
        const uint32_t* o = catt_offs.data() + b * nc1;
        FusedCommittee& ci = cinfo[b * st->ncomm + c];
        ci.boff = 0;
        ci.nbits = 0;
        ci.ga = o[c + 1] - o[c] == 0 ? 0xFFFFFFFEu : 0xFFFFFFFFu;
        // (several attestations: boff carries their catt range {k0, k1}, nbits stays 0 -- the
        // kernels read a committee's bitfield through boff only when it has exactly one)
        if (o[c + 1] - o[c] > 1) ci.boff = (uint64_t)o[c] | ((uint64_t)o[c + 1] << 32);
        if (o[c + 1] - o[c] == 1) {
          const uint64_t g = catt[b * st->natt + o[c]], ga = b * st->natt + g;
          ci.ga = (uint32_t)g;
          ci.boff = h->boffs[ga];
          ci.nbits = (uint32_t)(8 * (h->boffs[ga + 1] - h->boffs[ga]));
        }
      }
  }
  st->nparts = (st->world > 1 && st->B >= 2) ? 2 : 1;
  const int nlocal = comm ? comm->nlocal : 1;
  st->sh.resize(nlocal);
  const uint64_t nb_total = h->natt ? h->boffs[(uint64_t)st->B * st->natt] : 0;
  uint64_t max_inst_bytes = 0;
  for (uint64_t b = 0; b < st->B && h->natt; ++b)
    max_inst_bytes = std::max(max_inst_bytes, h->boffs[(b + 1) * st->natt] - h->boffs[b * st->natt]);
  for (int i = 0; i < nlocal && !rc; ++i) {
    Shard& s = st->sh[i];
    s.dev = comm ? comm->dev[i] : device;
    s.grank = comm ? comm->rank0 + i : 0;
    shard_range(h, pl, s.grank, st->world, &s.lo, &s.hi);
    s.n = s.hi - s.lo;
    s.np = st->fused ? (s.n + 3) & ~3ull : s.n;  // (rows of the one-pass stream: 16-B quads of u32)
    s.wl = (s.n + 63) / 64;
    DeviceCtx* dc;
    if ((rc = device_ctx(s.dev, &dc))) break;
    (void)hipSetDevice(s.dev);
    hipError_t e = hipStreamCreateWithFlags(&s.own, hipStreamNonBlocking);
    if (e != hipSuccess) {
      rc = hip_fail(e, "hipStreamCreate");
      break;
    }
    s.s = s.own;
    uint64_t *bal, *start, *end, *dyn, *tdep, *boffs = nullptr, *coffs = nullptr, *recd = nullptr;
    uint8_t* bits = nullptr;
    uint32_t *committee = nullptr, *cpos = nullptr, *att_comm = nullptr, *att_shard = nullptr;
    uint32_t *winner, *blk_cnt, *act_list;
    uint64_t* act_mask;
    const uint64_t vbpi = vblocks_per_inst(s.n);
    uint32_t* co_index = nullptr;
    uint2* se = nullptr;
    uint32_t* se16 = nullptr;
    if (st->co) {
      const uint32_t* inv = st->co_inv.data();
      if ((rc = upload_perm(s, &bal, h->balance, st->B, st->N, inv)) ||
          (rc = upload_perm(s, &start, h->start, st->B, st->N, inv)) ||
          (rc = upload_perm(s, &end, h->end, st->B, st->N, inv)))
        break;
      // np entries: the pad position of an odd range holds a valid index too (the one-pass
      // kernel reads co_index by 16-B pairs and looks every element's bit up unconditionally)
      std::vector<uint32_t> ci(inv + s.lo, inv + s.hi);
      ci.resize(std::max<uint64_t>(s.np, s.n), s.n ? inv[s.lo] : 0);
      if ((rc = upload(s, &co_index, ci.data(), ci.size()))) break;
      // the one-pass stream's {start, end}: 4 B when every CurrentDynasty is below 0xFFFF, 8 B
      // when below 2^32 - 1 (saturated bounds classify exactly below the saturation value),
      // else the 64-bit columns
      bool small_d = st->fused, tiny_d = st->fused;
      for (uint64_t b = 0; b < st->B && small_d; ++b) small_d = h->dynasty[b] < 0xFFFFFFFFull;
      for (uint64_t b = 0; b < st->B && tiny_d; ++b) tiny_d = h->dynasty[b] < 0xFFFFull;
      if (tiny_d) {
        if ((rc = upload_se16(s, &se16, h->start, h->end, st->B, st->N, inv))) break;
      } else if (small_d && (rc = upload_se(s, &se, h->start, h->end, st->B, st->N, inv))) {
        break;
      }
    } else if ((rc = upload_range(s, &bal, h->balance, st->B, st->N)) ||
               (rc = upload_range(s, &start, h->start, st->B, st->N)) ||
               (rc = upload_range(s, &end, h->end, st->B, st->N))) {
      break;
    }
    if ((rc = upload(s, &dyn, h->dynasty, st->B)) ||
        (rc = upload(s, &tdep, h->total_deposit, st->B)))
      break;
    if (st->natt) {
      std::vector<uint32_t> mem, pos;
      std::vector<uint64_t> offs;
      if (st->co) {  // committee c = storage positions [coffs[c], coffs[c+1]); no member list
        mem.assign(1, 0);
        offs.assign(h->coffs, h->coffs + h->ncomm + 1);
      } else if (st->world > 1) {
        local_committees(h, s.lo, s.hi, s.grank == 0, mem, offs, pos);
      } else {
        mem.assign(h->committee, h->committee + h->coffs[h->ncomm]);
        offs.assign(h->coffs, h->coffs + h->ncomm + 1);
      }
      const uint64_t na = (uint64_t)st->B * st->natt;
      // (16 B before and after the bitfields: the window pass's vote-bit loads reach up to 4 B
      // before an instance's first bitfield, the 16-B loads up to 15 B past the last)
      if ((rc = dalloc(s, &bits, nb_total + 32)) || (rc = upload_into(bits + 16, h->bits, nb_total)) ||
          (rc = upload(s, &boffs, h->boffs, na + 1)) || (rc = upload(s, &committee, mem.data(), mem.size())) ||
          (rc = upload(s, &coffs, offs.data(), offs.size())) || (rc = upload(s, &att_comm, h->att_comm, na)) ||
          (rc = upload(s, &att_shard, h->att_shard, na)))
        break;
      if (st->world > 1 && !st->co && (rc = upload(s, &cpos, pos.data(), pos.size()))) break;
    }
    if (st->nrec && (rc = upload(s, &recd, h->rec_dynasty, (size_t)st->B * st->nrec))) break;
    uint32_t *d_catt_offs = nullptr, *d_catt = nullptr;
    uint4 *d_items = nullptr, *d_items_ci = nullptr;
    FusedCommittee* d_cinfo = nullptr;
    uint64_t nitems = 0;
    std::vector<uint4> items;
    if (st->fused) {
      // committee pieces inside [lo, hi): <= 256 positions of a window that starts at the
      // committee's first local position rounded down to a multiple of 4 (local index = position
      // - lo; the quad kernels give each lane 4 positions from there, the pair kernels 2 from the
      // piece's even position)
      for (uint64_t c = 0; c < st->ncomm; ++c) {
        const uint64_t cb = h->coffs[c], ce = h->coffs[c + 1];
        const uint64_t r0 = std::max(cb, s.lo), r1 = std::min(ce, s.hi), base = s.lo + ((r0 - s.lo) & ~3ull);
        for (uint64_t x = r0; x < r1;) {
          const uint64_t y = std::min(r1, base + ((x - base) / 256 + 1) * 256);
          items.push_back(make_uint4((uint32_t)x, (uint32_t)(y - x), (uint32_t)c, (uint32_t)cb));
          x = y;
        }
      }
      nitems = items.size();
      // each piece's committee info per instance, read beside the piece (no items -> cinfo hop)
      std::vector<uint4> ic((size_t)st->B * nitems);
      for (uint64_t b = 0; b < st->B; ++b)
        for (uint64_t k = 0; k < nitems; ++k) {
          const FusedCommittee& ci = cinfo[b * st->ncomm + items[k].z];
          ic[b * nitems + k] = make_uint4((uint32_t)ci.boff, (uint32_t)(ci.boff >> 32), ci.nbits, ci.ga);
        }
      if ((rc = upload(s, &d_items, items.data(), items.size())) || (rc = upload(s, &d_cinfo, cinfo.data(), cinfo.size())) ||
          (rc = upload(s, &d_items_ci, ic.data(), ic.size())) ||
          (rc = upload(s, &d_catt_offs, catt_offs.data(), catt_offs.size())) ||
          (rc = upload(s, &d_catt, catt.data(), catt.size())))
        break;
    }
    if ((rc = dalloc(s, &winner, (size_t)st->B * std::max<uint32_t>(st->nrec, 1))) ||
        (rc = dalloc(s, &act_mask, (size_t)st->B * std::max<uint64_t>(s.wl, 1))) ||
        (rc = dalloc(s, &blk_cnt, (size_t)st->B * (vbpi + 1))) ||
        (rc = dalloc(s, &act_list, st->all_active ? 1 : (size_t)st->B * st->N)))
      break;
    for (uint32_t p = 0; p < st->nparts && !rc; ++p) {
      Part& q = s.part[p];
      q.i0 = st->B * p / st->nparts;
      q.B = st->B * (p + 1) / st->nparts - q.i0;
      const uint64_t Bp = q.B, i0 = q.i0;
      for (int k = 0; k < 2 && !rc; ++k) rc = dalloc(s, &q.red[k], Bp * kScal + 2 * Bp * st->natt + Bp * kPre);
      if (rc) break;
      if (st->general && ((rc = dalloc(s, &q.mask_send, Bp * st->sw)) ||
                          (rc = dalloc(s, &q.gmask, (size_t)st->world * Bp * st->sw)) ||
                          (rc = dalloc(s, &q.gblk, Bp * vblocks_per_inst(st->N)))))
        break;
      if ((rc = dalloc(s, &q.nb, Bp))) break;
      e = hipEventCreateWithFlags(&q.ev_red, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&q.ev_gather, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&q.ev_nb, hipEventDisableTiming);
      if (e != hipSuccess) {
        rc = hip_fail(e, "hipEventCreate");
        break;
      }
      EpochArgs& a = q.a;
      std::memset(&a, 0, sizeof a);
      a.ninst = q.B;
      a.nval = s.n;
      a.val_offset = s.lo;
      a.nval_global = st->N;
      a.kind = PZ_KIND_ACTIVE;
      a.balance = bal + i0 * s.np;
      a.start = start + i0 * s.np;
      a.end = end + i0 * s.np;
      a.dynasty = dyn + i0;
      a.total_deposit = tdep + i0;
      a.natt = st->natt;
      if (st->natt) {
        a.bits = bits + 16;
        a.boffs = boffs + i0 * st->natt;
        a.max_inst_bytes = max_inst_bytes;
        a.committee = committee;
        a.coffs = coffs;
        a.cpos = cpos;
        a.co_index = co_index;
        a.att_comm = att_comm + i0 * st->natt;
        a.att_shard = att_shard + i0 * st->natt;
      }
      a.pop_rank = (uint32_t)s.grank;
      a.pop_world = (uint32_t)st->world;
      a.nrec = st->nrec;
      a.rec_dynasty = recd ? recd + i0 * st->nrec : nullptr;
      a.winner = winner + i0 * std::max<uint32_t>(st->nrec, 1);
      a.act_mask = act_mask + i0 * std::max<uint64_t>(s.wl, 1);
      a.blk_cnt = blk_cnt + i0 * (vbpi + 1);
      a.act_list = st->all_active ? act_list : act_list + i0 * st->N;
      std::memset(&q.f, 0, sizeof q.f);
      if (st->fused) {
        q.f.items = d_items;
        q.f.nitems = nitems;
        q.f.cinfo = d_cinfo + i0 * st->ncomm;
        q.f.items_ci = d_items_ci + i0 * nitems;
        q.f.catt_offs = d_catt_offs + i0 * (st->ncomm + 1);
        q.f.catt = d_catt + i0 * st->natt;
        q.f.ncomm = st->ncomm;
        q.f.rank0 = s.grank == 0 ? 1 : 0;
        q.f.own_only = st->world > 1 ? 1 : 0;
        q.f.vstride = s.np;
        q.f.se = se ? se + i0 * s.np : nullptr;
        q.f.se16 = se16 ? se16 + i0 * s.np : nullptr;
        if (!fused_ok(a)) rc = fail(PZ_EINVAL, "one-pass epoch: validator arrays not on the 16-B path");
        // one instance on one rank: the single-launch step (latency path), within its limits
        // and when every attested committee is one piece (the waves form the winners)
        bool one = !rc && !st->opts.window_only && Bp == 1 && st->world == 1 && st->natt && st->nrec > 0 && st->natt <= kOneMaxAtt &&
                   st->nrec <= kOneMaxRec && max_inst_bytes <= kOneMaxBitBytes;
        std::vector<uint2> aw;
        if (one) {
          std::vector<uint32_t> pieces(st->ncomm, 0);
          for (const uint4& it : items) ++pieces[it.z];
          aw.resize(st->natt);
          for (uint64_t g = 0; g < st->natt && one; ++g) {
            const uint64_t ga = i0 * st->natt + g;
            const uint32_t sh = h->att_shard[ga];
            one = pieces[h->att_comm[ga]] == 1 && sh < st->nrec;
            const uint64_t rd = one ? h->rec_dynasty[i0 * st->nrec + sh] : 0;
            if (rd >> 32) one = false;  // (a 32-bit record dynasty)
            aw[g] = make_uint2(sh, (uint32_t)rd);
          }
        }
        if (one) {
          q.f.one = 1;
          q.f.win_in_wave = 1;
          std::vector<uint32_t> cs(st->natt);
          for (uint64_t g = 0; g < st->natt; ++g) {
            const uint32_t c = h->att_comm[i0 * st->natt + g];
            cs[g] = (uint32_t)(h->coffs[c + 1] - h->coffs[c]);
          }
          // the several-attestation committees' entries in catt order (FusedArgs.one_ck/one_cw)
          const uint64_t gb = i0 * st->natt, pbase = h->boffs[gb] & ~15ull;
          std::vector<uint4> ck(st->natt, make_uint4(0, 0, 0, 0));
          std::vector<uint2> cw(st->natt, make_uint2(0, 0));
          for (uint64_t k = 0; k < st->natt; ++k) {
            const uint32_t g = catt[gb + k];
            const uint64_t bo = h->boffs[gb + g];
            ck[k] = make_uint4((uint32_t)(bo - pbase), (uint32_t)(8 * (h->boffs[gb + g + 1] - bo)), g, 0);
            cw[k] = aw[g];
          }
          uint32_t *d_cs = nullptr, *w2 = nullptr;
          uint2 *d_aw = nullptr, *d_cw = nullptr;
          uint4* d_ck = nullptr;
          rc = dalloc(s, &q.f.ticket, 1);
          if (!rc) rc = upload(s, &d_cs, cs.data(), cs.size());
          if (!rc) rc = upload(s, &d_aw, aw.data(), aw.size());
          if (!rc) rc = upload(s, &d_ck, ck.data(), ck.size());
          if (!rc) rc = upload(s, &d_cw, cw.data(), cw.size());
          if (!rc) rc = dalloc(s, &w2, st->nrec);
          q.f.att_csize = d_cs;
          q.f.att_win = d_aw;
          q.f.one_ck = d_ck;
          q.f.one_cw = d_cw;
          q.f.winner_next = w2;
        } else if (!rc) {
          rc = plan_window(st, h, s, q, catt_offs, catt);
        }
        // the balances as u32 offsets (FusedArgs.bal32) for the window pass
        if (!rc && q.window && s.n) {
          const uint32_t* inv = st->co_inv.data();
          auto vals = [&](uint64_t b, uint64_t p) { return h->balance[(i0 + b) * st->N + inv[s.lo + p]]; };
          std::vector<uint64_t> base;
          uint64_t spread = 0;
          if (bal32_bases(Bp, s.n, vals, base, &spread)) {
            rc = bal32_upload(s, q, vals, base, true);
            st->b32 = true;
            q.w.narrow = spread < kNarrowSpread ? 1 : 0;  // (then the state re-bases every kNarrowPeriod steps)
          }
        }
        // the winners ping-pong (a step resets the next one's buffer): both start empty
        if (!rc && st->nrec && (q.f.one || q.window)) {
          uint32_t* nxt = q.f.one ? q.f.winner_next : q.w.winner_next;
          hipError_t e2 = hipMemsetAsync(nxt, 0xFF, (size_t)Bp * st->nrec * 4, s.s);
          if (e2 == hipSuccess) e2 = hipMemsetAsync(a.winner, 0xFF, (size_t)Bp * st->nrec * 4, s.s);
          if (e2 != hipSuccess) rc = hip_fail(e2, "hipMemsetAsync (winners)");
        }
      }
      q.cur = 1;  // flip() below binds red[0] as the first step's buffer
    }
  }
  if (rc) {
    delete st;
    return rc;
  }
  for (Shard& s : st->sh) {
    (void)hipSetDevice(s.dev);
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
      delete st;
      return hip_fail(e, "epoch state upload");
    }
  }
  st->b32_left = bal32_period(st->opts.rebase_period, any_narrow(st));
  flip(st);
  *out = st;
  return PZ_OK;
}

int pz_epoch_state_step(pz_epoch_state* st) {
  if (!st) return fail(PZ_EINVAL, "state is null");
  int rc;
  if (st->b32 && st->b32_left == 0) {
    if ((rc = bal32_rebase(st))) return rc;
    st->b32_left = bal32_period(st->opts.rebase_period, any_narrow(st));
  }
  rc = st->world > 1 ? step_sharded(st) : step_world1(st);
  if (rc) return rc;
  flip(st);
  ++st->steps;
  if (st->b32) --st->b32_left;
  return PZ_OK;
}

int pz_epoch_state_sync(pz_epoch_state* st) {
  if (!st) return fail(PZ_EINVAL, "state is null");
  for (Shard& s : st->sh) {
    (void)hipSetDevice(s.dev);
    hipError_t e = hipStreamSynchronize(s.s);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize (epoch state)");
  }
  return PZ_OK;
}

int pz_epoch_state_shard(const pz_epoch_state* st, int local, uint64_t* lo, uint64_t* hi, int* device,
                         void** stream) {
  if (!st) return fail(PZ_EINVAL, "state is null");
  if (local < 0 || local >= (int)st->sh.size()) return fail(PZ_EINVAL, "local rank %d of %zu", local, st->sh.size());
  const Shard& s = st->sh[local];
  if (lo) *lo = s.lo;
  if (hi) *hi = s.hi;
  if (device) *device = s.dev;
  if (stream) *stream = s.s;
  return PZ_OK;
}

int pz_epoch_state_bind_stream(pz_epoch_state* st, int local, void* stream) {
  if (!st) return fail(PZ_EINVAL, "state is null");
  if (local < 0 || local >= (int)st->sh.size()) return fail(PZ_EINVAL, "local rank %d of %zu", local, st->sh.size());
  Shard& s = st->sh[local];
  (void)hipSetDevice(s.dev);
  hipError_t e = hipStreamSynchronize(s.s);
  if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize (bind stream)");
  s.s = stream ? (hipStream_t)stream : s.own;
  return PZ_OK;
}

int pz_epoch_state_results(pz_epoch_state* st, int local, uint64_t* balance, uint64_t* scal, uint64_t* vote,
                           uint64_t* total, uint32_t* winner) {
  int rc = pz_epoch_state_shard(st, local, nullptr, nullptr, nullptr, nullptr);
  if (rc || (rc = pz_epoch_state_sync(st))) return rc;
  if (!st->steps) return fail(PZ_EINVAL, "no step has run");
  Shard& s = st->sh[local];
  (void)hipSetDevice(s.dev);
  hipError_t e = hipSuccess;
  for (uint32_t p = 0; p < st->nparts && e == hipSuccess; ++p) {
    const Part& q = s.part[p];
    const uint64_t Bp = q.B, i0 = q.i0, na = st->natt;
    if (balance && s.n && (rc = part_balances(s, q, balance + i0 * s.n, s.n))) return rc;
    if (e == hipSuccess && scal) e = hipMemcpy(scal + i0 * kScal, q.results, Bp * kScal * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess && vote && na)
      e = hipMemcpy(vote + i0 * na, q.results + Bp * kScal, Bp * na * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess && total && na)
      e = hipMemcpy(total + i0 * na, q.results + Bp * kScal + Bp * na, Bp * na * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess && winner && st->nrec)
      e = hipMemcpy(winner + i0 * st->nrec, q.win_results ? q.win_results : q.a.winner, Bp * st->nrec * 4,
                    hipMemcpyDeviceToHost);
  }
  return e == hipSuccess ? PZ_OK : hip_fail(e, "epoch state results D2H");
}

namespace {
bool any_narrow(const pz_epoch_state* st) {
  for (const Shard& s : st->sh)
    for (uint32_t p = 0; p < st->nparts; ++p)
      if (s.part[p].window && s.part[p].w.narrow) return true;
  return false;
}

int bal32_rebase(pz_epoch_state* st) {
  int rc = pz_epoch_state_sync(st);
  if (rc) return rc;
  bool any = false;
  for (Shard& s : st->sh) {
    (void)hipSetDevice(s.dev);
    for (uint32_t p = 0; p < st->nparts; ++p) {
      Part& q = s.part[p];
      if (!q.f.bal32) continue;
      std::vector<uint64_t> v((size_t)q.B * s.n), base;
      if ((rc = part_balances(s, q, v.data(), s.n))) return rc;
      auto vals = [&](uint64_t b, uint64_t x) { return v[b * s.n + x]; };
      uint64_t spread = 0;
      if (bal32_bases(q.B, s.n, vals, base, &spread)) {
        if ((rc = bal32_upload(s, q, vals, base, false))) return rc;
        q.w.narrow = spread < kNarrowSpread ? 1 : 0;
        any = true;
        continue;
      }
      q.w.narrow = 0;
      // the spread outgrew the window: this part returns to the u64 column
      hipError_t e = hipMemcpy2D(q.a.balance, s.np * 8, v.data(), s.n * 8, s.n * 8, q.B, hipMemcpyHostToDevice);
      if (e != hipSuccess) return hip_fail(e, "hipMemcpy2D H2D (epoch state re-base)");
      q.f.bal32 = nullptr;
      q.f.bal32_base = nullptr;
    }
  }
  st->b32 = any;
  return PZ_OK;
}
}  // namespace

int pz_epoch_state_columns(const pz_epoch_state* st, uint32_t* balance_bytes, uint32_t* dynasty_bytes) {
  if (!st || !balance_bytes || !dynasty_bytes) return fail(PZ_EINVAL, "null pointer");
  uint32_t bb = 0, db = 0;
  for (const Shard& s : st->sh)
    for (uint32_t p = 0; p < st->nparts; ++p) {
      const Part& q = s.part[p];
      bb = std::max<uint32_t>(bb, q.f.bal32 ? 4 : 8);
      db = std::max<uint32_t>(db, q.f.se16 ? 4 : q.f.se ? 8 : 16);
    }
  *balance_bytes = bb;
  *dynasty_bytes = db;
  return PZ_OK;
}

int pz_epoch_state_validators(const pz_epoch_state* st, int local, uint32_t* index) {
  if (!st) return fail(PZ_EINVAL, "null pointer");
  if (local < 0 || local >= (int)st->sh.size()) return fail(PZ_EINVAL, "local rank %d of %zu", local, st->sh.size());
  const Shard& s = st->sh[local];
  if (!index && s.n) return fail(PZ_EINVAL, "null pointer");  // an empty range may pass NULL
  for (uint64_t q = 0; q < s.n; ++q) index[q] = st->co ? st->co_inv[s.lo + q] : (uint32_t)(s.lo + q);
  return PZ_OK;
}

int pz_epoch_state_tallies(pz_epoch_state* st) {
  if (!st) return fail(PZ_EINVAL, "state is null");
  if (!st->steps) return fail(PZ_EINVAL, "no step has run");
  if (!(st->fused && st->world > 1) || !st->natt) return PZ_OK;  // already complete on every rank
  // summed once per step: a second all-reduce of complete tallies would multiply them by world
  if (st->tallied == st->steps) return PZ_OK;
  const int L = (int)st->sh.size();
  std::vector<hipStream_t> streams(L);
  std::vector<uint64_t*> bufs(L);
  std::vector<hipEvent_t> evs(L);
  int rc;
  for (uint32_t p = 0; p < st->nparts; ++p) {
    for (int i = 0; i < L; ++i) {
      Part& q = st->sh[i].part[p];
      streams[i] = st->sh[i].s;
      bufs[i] = q.results + (uint64_t)q.B * kScal;  // {vote, total} of the last step
      evs[i] = q.ev_nb;
    }
    if ((rc = st->comm->allreduce_u64(bufs.data(), 2ull * st->sh[0].part[p].B * st->natt, streams.data(), evs.data())))
      return rc;
    for (int i = 0; i < L; ++i)
      if ((rc = wait(st->sh[i], st->sh[i].part[p].ev_nb))) return rc;
  }
  if ((rc = pz_epoch_state_sync(st))) return rc;
  st->tallied = st->steps;
  return PZ_OK;
}

int pz_epoch_state_layout(const pz_epoch_state* st, int* committee_order) {
  if (!st || !committee_order) return fail(PZ_EINVAL, "null pointer");
  *committee_order = st->fused ? 2 : st->co ? 1 : 0;
  return PZ_OK;
}

void pz_epoch_state_free(pz_epoch_state* st) { delete st; }

int pz_epoch_plan(const pz_epoch_host* h, int world, int rank, uint64_t* lo, uint64_t* hi, int* committee_order) {
  if (!lo || !hi || !committee_order) return fail(PZ_EINVAL, "null pointer");
  if (world < 1 || rank < 0 || rank >= world) return fail(PZ_EINVAL, "rank %d outside world %d", rank, world);
  int rc = check_host(h);
  if (rc) return rc;
  const Plan p = plan_layout(h);
  shard_range(h, p, rank, world, lo, hi);
  *committee_order = p.fused ? 2 : p.co ? 1 : 0;
  return PZ_OK;
}

}  // extern "C"
