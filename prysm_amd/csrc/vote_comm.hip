// pz_comm_vote_tally: the block vote-cache tally (blockchain/core.go:300-345,
// calculateBlockVoteCache) sharded by validator range over the ranks of a pz_comm
// (include/prysm_hip.h).
//
// Each local rank uploads the replicated inputs (committees, attestations, work items) and
// its 64-aligned validator range [lo, hi) of the balances and of every slot's voter bitmap,
// tallies only the committee members it owns (votes.hip tally_item with the range), and the
// per-slot partial totals -- plus a panic flag -- are summed by one all-reduce.  A voter's
// dedup bit lives on exactly one rank, so the union stays exact and the u64 sums commute:
// every rank ends with the totals the one-GPU tally gives.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "comm.h"
#include "runtime.h"
#include "votes.h"

using namespace pz;

namespace {

struct RankWork {
  int dev = 0;
  hipStream_t s = nullptr;
  hipEvent_t done = nullptr;
  uint64_t lo = 0, hi = 0, wlo = 0, wn = 0;  // validator range, bitmap word range
  std::vector<void*> allocs;
  uint64_t* red = nullptr;  // [nslots + 1]: totals, then the panic flag
  pz_vote_batch v;
  ~RankWork() {
    (void)hipSetDevice(dev);
    if (s) (void)hipStreamSynchronize(s);
    for (void* p : allocs) (void)hipFree(p);
    if (done) (void)hipEventDestroy(done);
    if (s) (void)hipStreamDestroy(s);
  }
  // Device copy of host[0, count) followed by `pad` zero bytes (the whole buffer zeroed when
  // host is null); never reads past host + count.
  template <typename T>
  T* up(const T* host, size_t count, int* rc, size_t pad = 0) {
    if (*rc) return nullptr;
    void* p = nullptr;
    const size_t bytes = count * sizeof(T), alloc = std::max<size_t>(bytes + pad, 16);
    hipError_t e = hipMalloc(&p, alloc);
    if (e != hipSuccess) {
      *rc = hip_fail(e, "hipMalloc (vote tally)");
      return nullptr;
    }
    allocs.push_back(p);
    if (host && bytes) {
      e = hipMemcpyAsync(p, host, bytes, hipMemcpyHostToDevice, s);
      if (e == hipSuccess && alloc > bytes) e = hipMemsetAsync(static_cast<uint8_t*>(p) + bytes, 0, alloc - bytes, s);
    } else {
      e = hipMemsetAsync(p, 0, alloc, s);
    }
    if (e != hipSuccess) *rc = hip_fail(e, "H2D (vote tally)");
    return static_cast<T*>(p);
  }
};

}  // namespace

extern "C" int pz_comm_vote_tally(const pz_comm* comm, const uint32_t* committee, const uint64_t* coffs,
                                  uint64_t ncomm, const uint32_t* att_comm, const uint8_t* bits,
                                  const uint64_t* boffs, uint64_t natt, const uint32_t* item_att,
                                  const uint32_t* item_slot, uint64_t nitems, const uint64_t* balance, uint64_t nval,
                                  uint32_t* bitmaps, uint64_t nslots, uint64_t words_per_slot, uint64_t* totals) {
  if (!comm) return fail(PZ_EINVAL, "comm is null");
  if (!nitems) return PZ_OK;
  int rc;
  if ((rc = check_csr(coffs, ncomm, "committee"))) return rc;
  if ((rc = check_csr(boffs, natt, "bitfield"))) return rc;
  if (!item_att || !item_slot || !att_comm || !bitmaps || !totals || !balance || !committee)
    return fail(PZ_EINVAL, "null pointer");
  if (words_per_slot * 32 < nval) return fail(PZ_EINVAL, "words_per_slot too small");
  for (uint64_t i = 0; i < nitems; ++i)
    if (item_att[i] >= natt || item_slot[i] >= nslots)
      return fail(PZ_EINVAL, "work item %llu out of range", (unsigned long long)i);
  for (uint64_t a = 0; a < natt; ++a)
    if (att_comm[a] >= ncomm) return fail(PZ_EINVAL, "attestation %llu names a missing committee", (unsigned long long)a);
  pz_comm* c = const_cast<pz_comm*>(comm);
  const int L = c->nlocal, world = c->world;
  const uint64_t span = 64 * std::max<uint64_t>(1, (nval + 64ull * world - 1) / (64ull * world));
  std::vector<uint64_t> rb = rebase(boffs, natt), rcf = rebase(coffs, ncomm);
  std::vector<RankWork> rk(L);
  std::vector<uint64_t*> bufs(L);
  std::vector<hipStream_t> streams(L);
  std::vector<hipEvent_t> evs(L);
  // every rank's bitmap words, packed [nslots][wn]: one host buffer per rank, alive until the
  // final sync, so no rank's upload waits for another's
  std::vector<std::vector<uint32_t>> slices(L);
  rc = PZ_OK;
  for (int i = 0; i < L && !rc; ++i) {
    RankWork& w = rk[i];
    w.dev = c->dev[i];
    const uint64_t grank = (uint64_t)(c->rank0 + i);
    w.lo = std::min<uint64_t>(nval, grank * span);
    w.hi = std::min<uint64_t>(nval, (grank + 1) * span);
    w.wlo = w.lo / 32;
    w.wn = (w.hi - w.lo + 31) / 32;
    (void)hipSetDevice(w.dev);
    hipError_t e = hipStreamCreateWithFlags(&w.s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&w.done, hipEventDisableTiming);
    if (e != hipSuccess) {
      rc = hip_fail(e, "stream/event (vote tally)");
      break;
    }
    std::memset(&w.v, 0, sizeof w.v);
    pz_vote_batch& v = w.v;
    v.committee = w.up(committee + coffs[0], rcf[ncomm], &rc);
    v.coffs = w.up(rcf.data(), ncomm + 1, &rc);
    v.att_comm = w.up(att_comm, natt, &rc);
    v.bits = w.up(bits ? bits + boffs[0] : bits, rb[natt], &rc, 16);  // 16-B zero pad for the wide loads
    v.boffs = w.up(rb.data(), natt + 1, &rc);
    v.item_att = w.up(item_att, nitems, &rc);
    v.item_slot = w.up(item_slot, nitems, &rc);
    v.nitems = nitems;
    v.balance = w.up(balance + w.lo, w.hi - w.lo, &rc);
    v.nval = w.hi - w.lo;
    v.val_offset = w.lo;
    v.nval_global = nval;
    std::vector<uint32_t>& slice = slices[i];
    slice.assign(std::max<uint64_t>(nslots * w.wn, 1), 0);
    for (uint64_t s = 0; s < nslots; ++s)
      std::memcpy(slice.data() + s * w.wn, bitmaps + s * words_per_slot + w.wlo, w.wn * 4);
    v.bitmaps = w.up(slice.data(), nslots * w.wn, &rc);
    v.words_per_slot = w.wn;
    // partial totals: rank 0 starts from the caller's totals, the others from zero
    w.red = w.up<uint64_t>(nullptr, nslots + 1, &rc);
    if (!rc && grank == 0) {
      e = hipMemcpyAsync(w.red, totals, nslots * 8, hipMemcpyHostToDevice, w.s);
      if (e != hipSuccess) rc = hip_fail(e, "H2D totals");
    }
    if (rc) break;
    v.totals = w.red;
    v.err = w.red + nslots;
    if (w.hi > w.lo || grank == 0) {  // an empty range still raises the panics on rank 0
      if (w.hi == w.lo) v.nval = 0;
      e = launch_vote_tally(v, w.s);
      if (e != hipSuccess) rc = hip_fail(e, "pz_vote_tally_kernel (sharded)");
    }
    // no sync here: the local ranks tally concurrently, and the all-reduce orders itself
    // after every rank's stream
    bufs[i] = w.red;
    streams[i] = w.s;
    evs[i] = w.done;
  }
  if (!rc && world > 1) rc = c->allreduce_u64(bufs.data(), nslots + 1, streams.data(), evs.data());
  std::vector<uint64_t> red(nslots + 1);
  for (int i = 0; i < L && !rc; ++i) {
    RankWork& w = rk[i];
    (void)hipSetDevice(w.dev);
    std::vector<uint32_t>& slice = slices[i];
    hipError_t e = world > 1 ? hipStreamWaitEvent(w.s, w.done, 0) : hipSuccess;
    if (e == hipSuccess && i == 0) e = hipMemcpyAsync(red.data(), w.red, (nslots + 1) * 8, hipMemcpyDeviceToHost, w.s);
    if (e == hipSuccess && w.wn)
      e = hipMemcpyAsync(slice.data(), w.v.bitmaps, nslots * w.wn * 4, hipMemcpyDeviceToHost, w.s);
    if (e == hipSuccess) e = hipStreamSynchronize(w.s);
    if (e != hipSuccess) {
      rc = hip_fail(e, "D2H (vote tally)");
      break;
    }
    for (uint64_t s = 0; s < nslots; ++s)
      std::memcpy(bitmaps + s * words_per_slot + w.wlo, slice.data() + s * w.wn, w.wn * 4);
  }
  if (rc) return rc;
  std::memcpy(totals, red.data(), nslots * 8);
  if (red[nslots]) return fail(PZ_EINDEX, "calculateBlockVoteCache would panic (short bitfield or voter >= len(validators))");
  return PZ_OK;
}
