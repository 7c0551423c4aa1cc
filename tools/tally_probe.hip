// Where the voter-major vote tally's time goes (tools/ only): a configs[4]-shaped flush (natt
// attestations of k-member committees over nval validators, every voter new for the 64 parents
// of a two-word id run, the bitfields inline) tallied by the product body (votes_dev.h), timed
// with events, then again with per-wave phase stamps (wall clock, 100 MHz).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tally_probe.hip -o build/tally_probe
//   build/tally_probe [natt=320] [k=128] [nval=65536] [waves_per_block=4] [host_queue=1]
//                     [shuffled=1] [idle_us=0]
// shuffled 0: committee members in validator order (a voter-position vote cache: an
// attestation's voter words are contiguous); idle_us > 0: the GPU idles that long before each
// flush, and each flush's id words are fresh (cold) rows, as in a replay's transitions.
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "../prysm_amd/csrc/votes_dev.h"

using namespace pz;

extern "C" __global__ void __launch_bounds__(1024) probe_plain(VoteWordArgs a) {
  vote_words_body(a, gridDim.x, blockIdx.x);
}
extern "C" __global__ void __launch_bounds__(1024) probe_traced(VoteWordArgs a, uint64_t* tr) {
  vote_words_body(a, gridDim.x, blockIdx.x, tr);
}

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t natt = argc > 1 ? atoi(argv[1]) : 320;
  const uint32_t k = argc > 2 ? atoi(argv[2]) : 128;
  const uint32_t nval = argc > 3 ? atoi(argv[3]) : 65536;
  const uint32_t wpb = argc > 4 ? atoi(argv[4]) : 4;
  const bool host_q = argc > 5 ? atoi(argv[5]) != 0 : true;
  const bool shuffled = argc > 6 ? atoi(argv[6]) != 0 : true;
  const int idle_us = argc > 7 ? atoi(argv[7]) : 0;
  if (k > 256 || nval % k || wpb < 1 || wpb > 16) {
    fprintf(stderr, "k <= 256 dividing nval; 1-16 waves per block\n");
    return 2;
  }
  std::mt19937_64 rng(7);
  std::vector<uint32_t> members(nval);
  std::iota(members.begin(), members.end(), 0u);
  if (shuffled) std::shuffle(members.begin(), members.end(), rng);
  const uint32_t ncomm = nval / k;
  std::vector<VoteRec> rec(natt);
  for (uint32_t i = 0; i < natt; ++i) {
    VoteRec& r = rec[i];
    std::memset(&r, 0, sizeof r);
    r.cb = (uint32_t)((i % ncomm) * k);  // distinct committees: every voter new
    r.k = k;
    r.s0 = 13 + i / 5;  // a run over two id words, one new parent per block (+ the flush's base)
    r.form = 0;
    r.step = ~1ull;
    r.absent = 0;
    for (uint32_t b = 0; b < k; ++b) reinterpret_cast<uint8_t*>(r.bits)[b >> 3] |= (uint8_t)(0x80 >> (b & 7));
  }
  const uint32_t nwords = 128;  // flush f uses words 2 (f % 60) and 2 (f % 60) + 1
  uint32_t *d_comm, *d_ticket;
  uint64_t *d_bal, *d_bm, *d_tot, *d_err;
  uint8_t* d_present;
  VoteRec* q = nullptr;
  CK(hipMalloc(&d_comm, nval * 4));
  CK(hipMalloc(&d_bal, nval * 8));
  CK(hipMalloc(&d_bm, (size_t)nwords * nval * 8));
  CK(hipMalloc(&d_tot, nwords * 64 * 8));
  CK(hipMalloc(&d_present, nwords * 64));
  CK(hipMalloc(&d_err, 8));
  CK(hipMalloc(&d_ticket, 4));
  CK(hipMemcpy(d_comm, members.data(), nval * 4, hipMemcpyHostToDevice));
  std::vector<uint64_t> bal(nval, 32000000000ull);
  CK(hipMemcpy(d_bal, bal.data(), nval * 8, hipMemcpyHostToDevice));
  CK(hipMemset(d_ticket, 0, 4));
  CK(hipMemset(d_err, 0, 8));
  if (host_q) {
    CK(hipHostMalloc((void**)&q, natt * sizeof(VoteRec), hipHostMallocDefault));
    std::memcpy(q, rec.data(), natt * sizeof(VoteRec));
  } else {
    CK(hipMalloc(&q, natt * sizeof(VoteRec)));
    CK(hipMemcpy(q, rec.data(), natt * sizeof(VoteRec), hipMemcpyHostToDevice));
  }
  uint64_t* gout;
  CK(hipHostMalloc((void**)&gout, (kJustifySlots + 2) * 8, hipHostMallocDefault));
  VoteWordArgs a;
  std::memset(&a, 0, sizeof a);
  a.committee = d_comm;
  a.rec = q;
  a.natt = natt;
  a.chunks = 1;
  a.balance = d_bal;
  a.nval = a.nval_global = nval;
  a.bm = d_bm;
  a.totals = d_tot;
  a.present = d_present;
  a.err = d_err;
  a.gather_out = gout;
  a.ticket = d_ticket;
  const uint32_t nblk = (natt + wpb - 1) / wpb;
  uint64_t* d_tr;
  CK(hipMalloc(&d_tr, (size_t)nblk * wpb * 8 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hipMemset(d_bm, 0, (size_t)nwords * nval * 8));
  CK(hipMemset(d_tot, 0, nwords * 64 * 8));
  std::vector<VoteRec> qf(natt);
  int flush = 0;
  // one flush: fresh words (idle mode) or the same words cleared first (back to back)
  auto prepare = [&]() {
    const uint32_t base = idle_us > 0 ? 128 * (flush % 60) : 0;
    if (idle_us <= 0) {
      CK(hipMemsetAsync(d_bm, 0, (size_t)2 * nval * 8, s));
      CK(hipMemsetAsync(d_tot, 0, 2 * 64 * 8, s));
    }
    for (uint32_t i = 0; i < natt; ++i) {
      qf[i] = rec[i];
      qf[i].s0 += base;
    }
    if (host_q) std::memcpy(q, qf.data(), natt * sizeof(VoteRec));
    else CK(hipMemcpyAsync(q, qf.data(), natt * sizeof(VoteRec), hipMemcpyHostToDevice, s));
    for (int j = 0; j < kJustifySlots; ++j) a.gq.slot[j] = base + 13 + j;
    a.gather_seq = ++flush;
    CK(hipStreamSynchronize(s));
    if (idle_us > 0) usleep(idle_us);
  };
  std::vector<float> ms;
  for (int it = 0; it < 40; ++it) {
    prepare();
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(probe_plain, dim3(nblk), dim3(64 * wpb), 0, s, a);
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (it >= 5) ms.push_back(t * 1000.f);
  }
  std::sort(ms.begin(), ms.end());
  printf("natt %u k %u nval %u waves/block %u queue %s members %s idle %d us: plain kernel event time median %.2f us (min %.2f)\n",
         natt, k, nval, wpb, host_q ? "pinned host" : "device", shuffled ? "shuffled" : "in order", idle_us,
         ms[ms.size() / 2], ms[0]);
  printf("totals[0..3] %llu %llu %llu %llu seq %llu\n", (unsigned long long)gout[0], (unsigned long long)gout[1],
         (unsigned long long)gout[2], (unsigned long long)gout[3], (unsigned long long)gout[kJustifySlots + 1]);
  // traced run
  std::vector<uint64_t> tr((size_t)nblk * wpb * 8);
  std::vector<std::vector<double>> ph(8);
  for (int it = 0; it < 10; ++it) {
    CK(hipMemsetAsync(d_tr, 0, tr.size() * 8, s));
    prepare();
    hipLaunchKernelGGL(probe_traced, dim3(nblk), dim3(64 * wpb), 0, s, a, d_tr);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(tr.data(), d_tr, tr.size() * 8, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull;
    for (size_t w = 0; w < natt; ++w) t0 = std::min(t0, tr[w * 8]);
    for (size_t w = 0; w < natt; ++w)
      for (int p = 0; p < 8; ++p)
        if (tr[w * 8 + p]) ph[p].push_back((tr[w * 8 + p] - t0) * 0.01);  // 100 MHz -> us
  }
  const char* names[8] = {"wave start", "record loaded", "members loaded", "balances loaded", "word atomics returned",
                          "wave done", "block flushed", "gather stored (last block)"};
  for (int p = 0; p < 8; ++p) {
    auto& v = ph[p];
    if (v.empty()) continue;
    std::sort(v.begin(), v.end());
    printf("  %-28s since the first wave: p10 %6.2f  median %6.2f  p90 %6.2f  max %6.2f us (n %zu)\n", names[p],
           v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back(), v.size());
  }
  return 0;
}
