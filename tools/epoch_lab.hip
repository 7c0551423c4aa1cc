// Stand-alone lab for the epoch streaming pass (round 5): times candidate kernel structures on
// the bench's cold 1M x 16 and 65,536 x 256 shapes without the library, so that one GPU call
// measures several forms.  Not product code: the product kernel is prysm_amd/csrc/epoch.hip.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/epoch_lab.hip -o build/epoch_lab
//   build/epoch_lab [N B R NT]
//
// The form under test ("window" pass): one launch per step, no pre pass.  Block (instance,
// committee-aligned position range) does
//   prologue: stage the instance's last bitfield in LDS while counting every bitfield's bits
//             (GetAttestersTotalDeposit) and checking their lengths; place the range's committee
//             bitfields in position order in an LDS bitmap (the vote bits);
//   loop:     fixed 256-position windows (64 lanes x 4), loads D windows ahead; reward bits from
//             the LDS copy of the last bitfield through co_index; crosslink tallies as per-
//             committee segment sums into LDS;
//   epilogue: the range's committees' tallies out with plain stores, winners by atomicMin.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

constexpr uint32_t kNoAtt = 0xFFFFFFFEu, kManyAtt = 0xFFFFFFFFu;

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16_nt(const void* p) {
  const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(x.x, x.y, x.z, x.w);
}

__device__ __forceinline__ uint64_t wsum(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#define ST(CTRL, RM)                                                                              \
  {                                                                                             \
    const uint32_t l2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, RM, 0xf, false); \
    const uint32_t h2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, RM, 0xf, false); \
    const uint64_t t = (((uint64_t)hi << 32) | lo) + (((uint64_t)h2 << 32) | l2);               \
    lo = (uint32_t)t;                                                                           \
    hi = (uint32_t)(t >> 32);                                                                   \
  }
  ST(0xB1, 0xf) ST(0x4E, 0xf) ST(0x141, 0xf) ST(0x140, 0xf) ST(0x142, 0xa) ST(0x143, 0xc)
#undef ST
  const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
  const uint32_t rh = (uint32_t)__builtin_amdgcn_readlane((int)hi, 63);
  return ((uint64_t)rh << 32) | rl;
}

struct Args {
  uint32_t B, R, natt, ncomm, nrec;
  uint64_t N, vstride;
  uint32_t* bal32;
  const uint64_t* base;
  const uint32_t* se16;
  const uint32_t* co_index;
  const uint8_t* bits;
  const uint64_t* boffs;     // [B*natt+1]
  const uint32_t* csize;     // [B][natt]
  const uint32_t* cstart;    // [ncomm+1]
  const uint4* rdesc;        // [R] {cr0, cr1, wbase, nwin}
  const uint32_t* wdesc;     // [windows] first committee overlapping the window
  const uint4* cinfo;        // [B][ncomm] {boff lo, boff hi, ga, -}
  const uint2* att_win;      // [B][natt]
  const uint64_t* dyn;
  const uint64_t* tdep;
  uint64_t* vote;
  uint64_t* total;
  uint32_t* winner;
  uint64_t* scal;            // [B][8]
  uint32_t maxc;             // most committees in a range
  uint32_t lbytes;           // LDS bytes for the last bitfield copy
  uint32_t vwords;           // LDS words of the vote-bit map
};

// FL bits: 1 reward bits from L2 instead of LDS; 2 no tallies; 4 no prologue bit count (pop=all);
// 8 no store
template <int NT, int D, int FL>
__global__ void __launch_bounds__(NT) win_kernel(Args a) {
  extern __shared__ __align__(16) uint8_t lds[];
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t inst = blockIdx.x / a.R, r = blockIdx.x - inst * a.R;
  const uint4 rd = a.rdesc[r];
  const uint32_t cr0 = rd.x, cr1 = rd.y, wb = rd.z, nwin = rd.w;
  const uint64_t P0 = a.cstart[cr0], P1 = a.cstart[cr1], P0a = P0 & ~3ull;
  uint8_t* lbf = lds;
  uint32_t* vb = reinterpret_cast<uint32_t*>(lds + a.lbytes);
  uint32_t* cst = vb + a.vwords;                                    // [maxc+1] starts rel. P0a
  uint64_t* tot = reinterpret_cast<uint64_t*>(cst + ((a.maxc + 2) & ~1u));
  uint64_t* vot = tot + a.maxc;
  uint8_t* kd = reinterpret_cast<uint8_t*>(vot + a.maxc);
  __shared__ uint64_t red[NW][3];
  const uint64_t vs = a.vstride;
  uint32_t* Bal = a.bal32 + (uint64_t)inst * vs;
  const uint32_t* SE = a.se16 + (uint64_t)inst * vs;
  // the first D windows' loads, before anything else
  uint4 qb[D], qs[D], qc[D];
  uint32_t qd[D];
  auto load_win = [&](int j, uint32_t k) {
    const uint64_t p = P0a + 256ull * k + 4ull * lane;
    const bool any = k < nwin && p + 3 >= P0 && p < P1;
    const uint64_t pp = any ? p : P0a;
    qb[j] = *reinterpret_cast<const uint4*>(Bal + pp);
    qs[j] = ld16_nt(SE + pp);
    qc[j] = *reinterpret_cast<const uint4*>(a.co_index + pp);
    qd[j] = a.wdesc[wb + (k < nwin ? k : 0)];
  };
#pragma unroll
  for (int j = 0; j < D; ++j) load_win(j, wave + j * NW);
  // zero the LDS vote bits and tallies
  for (uint32_t i = tid; i < a.vwords; i += NT) vb[i] = 0;
  for (uint32_t i = tid; i < a.maxc; i += NT) tot[i] = 0, vot[i] = 0;
  const uint64_t gb = (uint64_t)inst * a.natt;
  const uint64_t pbeg = a.boffs[gb], pend = a.boffs[gb + a.natt], lb = a.boffs[gb + a.natt - 1];
  const uint64_t pbase = pbeg & ~15ull, lbase = lb & ~15ull;
  __syncthreads();
  // committee starts and kinds; the vote bits of single-attestation committees
  uint4 ci = make_uint4(0, 0, kNoAtt, 0);
  uint32_t myc = cr0 + tid;
  if (myc <= cr1) cst[myc - cr0] = (uint32_t)(a.cstart[myc] - P0a);
  if (myc < cr1) ci = a.cinfo[(uint64_t)inst * a.ncomm + myc];
  // flat pass: bit count of every bitfield, the last one copied into LDS
  uint64_t pop = 0, err = 0;
  if (!(FL & 4)) {
    const uint64_t nch = (pend - pbase + 15) / 16;
    constexpr int U = 8;
    for (uint64_t c0 = tid; c0 < nch; c0 += (uint64_t)U * NT) {
      uint4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t c = c0 + (uint64_t)u * NT;
        x[u] = c < nch ? *reinterpret_cast<const uint4*>(a.bits + pbase + 16 * c) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t c = c0 + (uint64_t)u * NT;
        if (c >= nch) continue;
        const uint64_t ad = pbase + 16 * c;
        const uint32_t w[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
        if (ad >= pbeg && ad + 16 <= pend) {
          pop += __popc(w[0]) + __popc(w[1]) + __popc(w[2]) + __popc(w[3]);
        } else {
#pragma unroll
          for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const uint64_t at = ad + 4 * d + b;
              if (at >= pbeg && at < pend) pop += __popc((w[d] >> (8 * b)) & 0xFFu);
            }
        }
        if (ad >= lbase) *reinterpret_cast<uint4*>(lbf + (ad - lbase)) = x[u];
      }
    }
    for (uint32_t g = tid; g < a.natt; g += NT)
      if ((uint64_t)a.csize[gb + g] > 8 * (a.boffs[gb + g + 1] - a.boffs[gb + g])) err = 1;
  } else {
    pop = tid == 0 ? a.N * 2 : 0;
  }
  if (myc < cr1) kd[myc - cr0] = ci.z == kNoAtt ? 0 : ci.z == kManyAtt ? 2 : 1;
  __syncthreads();  // cst complete
  // vote bits: (committee, 32-bit word) items over the block, all loads of a round in flight
  {
    const uint32_t items = (cr1 - cr0) * 8;  // (committees of <= 256 members here)
    constexpr int U = 4;
    for (uint32_t t0 = tid; t0 < items; t0 += U * NT) {
      uint4 cc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t t = t0 + u * NT;
        cc[u] = t < items ? a.cinfo[(uint64_t)inst * a.ncomm + cr0 + t / 8] : make_uint4(0, 0, kNoAtt, 0);
      }
      uint64_t raw[U];
      uint32_t sh8[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t t = t0 + u * NT, cl = t / 8, m = t % 8;
        const uint32_t cs = t < items ? cst[cl + 1] - cst[cl] : 0;
        const bool ok = t < items && cc[u].z < kNoAtt && 32 * m < cs;
        const uint64_t ad = (((uint64_t)cc[u].y << 32) | cc[u].x) + 4 * m, da = ad & ~3ull;
        sh8[u] = (uint32_t)(ad - da) * 8;
        raw[u] = 0;
        if (ok) __builtin_memcpy(&raw[u], __builtin_assume_aligned(a.bits + da, 4), 8);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t t = t0 + u * NT, cl = t / 8, m = t % 8;
        const uint32_t cs = t < items ? cst[cl + 1] - cst[cl] : 0;
        if (!(t < items && cc[u].z < kNoAtt && 32 * m < cs)) continue;
        uint32_t W = __builtin_bitreverse32(__builtin_bswap32((uint32_t)(raw[u] >> sh8[u])));
        const uint32_t left = cs - 32 * m;
        if (left < 32) W &= (1u << left) - 1u;
        const uint32_t o = cst[cl] + 32 * m, sh = o & 31;
        atomicOr(&vb[o >> 5], W << sh);
        if (sh) atomicOr(&vb[(o >> 5) + 1], W >> (32 - sh));
      }
    }
  }
  pop = wsum(pop);
  err = wsum(err);
  if (lane == 0) red[wave][0] = pop, red[wave][1] = err;
  __syncthreads();
  pop = 0, err = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) pop += red[w][0], err += red[w][1];
  const uint64_t L = pend - lb;
  const bool rwd_err = (a.N - 1) >= 8 * L;
  const bool thr = (pop * 32ull * 3ull) >= (a.tdep[inst] * 2ull);
  const bool skip = err != 0 || (thr && rwd_err);
  const bool applied = thr && !skip;
  const uint64_t d = a.dyn[inst];
  const uint64_t bbase = a.base[inst];
  const uint8_t* lbf8 = (FL & 1) ? a.bits + lb : lbf + (lb - lbase);
  uint64_t sum = 0, nm = 0;
  for (uint32_t k = wave; k < nwin; k += D * NW) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const uint32_t kk = k + j * NW;
      if (kk >= nwin) break;
      const uint64_t p = P0a + 256ull * kk + 4ull * lane;
      const uint32_t loc = (uint32_t)(p - P0a);
      bool v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = p + i >= P0 && p + i < P1;
      uint64_t b[4] = {bbase + qb[j].x, bbase + qb[j].y, bbase + qb[j].z, bbase + qb[j].w};
      const uint32_t s4[4] = {qs[j].x, qs[j].y, qs[j].z, qs[j].w};
      const uint32_t c4[4] = {qc[j].x, qc[j].y, qc[j].z, qc[j].w};
      uint32_t rb[4] = {0, 0, 0, 0};
      if (applied) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t ix = v[i] ? c4[i] : 0u;
          rb[i] = (lbf8[ix >> 3] >> (7 - (ix & 7))) & 1u;
        }
      }
      if (!(FL & 2)) {
        const uint32_t vw = (vb[loc >> 5] >> (loc & 31)) & 0xFu;
        const uint32_t wend = 256 * kk + 256;
        uint32_t c = qd[j];
        c = __builtin_amdgcn_readfirstlane(c);
        for (;;) {
          const uint32_t cl = c - cr0;
          const uint32_t s_lo = __builtin_amdgcn_readfirstlane(cst[cl]);
          const uint32_t s_hi = __builtin_amdgcn_readfirstlane(cst[cl + 1]);
          const uint32_t kind = __builtin_amdgcn_readfirstlane(kd[cl]);
          if (kind) {
            uint64_t t = 0, x = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const bool in = v[i] && loc + i >= s_lo && loc + i < s_hi;
              t += in ? b[i] : 0;
              x += (in && ((vw >> i) & 1)) ? b[i] : 0;
            }
            t = wsum(t);
            x = wsum(x);
            if (lane == 0) {
              atomicAdd((unsigned long long*)&tot[cl], (unsigned long long)t);
              atomicAdd((unsigned long long*)&vot[cl], (unsigned long long)x);
            }
          }
          ++c;
          if (s_hi >= wend || c >= cr1) break;
        }
      }
      bool act[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        act[i] = (uint64_t)(s4[i] & 0xFFFFu) <= d && d < (uint64_t)(s4[i] >> 16);
        nm += (v[i] && !act[i]) ? 1 : 0;
      }
      if (applied) {
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = rb[i] ? b[i] + 1 : b[i] - 1;
        if (!(FL & 8)) {
          if (v[0] && v[1] && v[2] && v[3]) {
            *reinterpret_cast<uint4*>(Bal + p) = make_uint4((uint32_t)(b[0] - bbase), (uint32_t)(b[1] - bbase),
                                                            (uint32_t)(b[2] - bbase), (uint32_t)(b[3] - bbase));
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (v[i]) Bal[p + i] = (uint32_t)(b[i] - bbase);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) sum += (v[i] && act[i]) ? b[i] : 0;
      load_win(j, kk + D * NW);
    }
  }
  sum = wsum(sum);
  nm = wsum(nm);
  if (lane == 0) red[wave][0] = sum, red[wave][1] = nm;
  __syncthreads();
  uint64_t* sc = a.scal + (uint64_t)inst * 8;
  if (tid == 0) {
    uint64_t s = 0, n = 0;
    for (int w = 0; w < NW; ++w) s += red[w][0], n += red[w][1];
    if (s && !skip) atomicAdd((unsigned long long*)&sc[5], (unsigned long long)s);
    if (n) atomicAdd((unsigned long long*)&sc[7], (unsigned long long)n);
    if (r == 0) {
      sc[0] = pop;
      sc[4] = applied;
      sc[2] = err ? 2 : 0;
      sc[3] = rwd_err;
    }
  }
  if (!(FL & 2)) {
    for (uint32_t c = cr0 + tid; c < cr1; c += NT) {
      const uint32_t cl = c - cr0;
      if (kd[cl] != 1) continue;
      const uint4 cc = c == myc ? ci : a.cinfo[(uint64_t)inst * a.ncomm + c];
      const uint32_t g = cc.z;
      const uint64_t V = vot[cl], T = tot[cl];
      a.vote[gb + g] = V;
      a.total[gb + g] = T;
      const uint2 w = a.att_win[gb + g];
      if (3ull * V >= 2ull * T && d > (uint64_t)w.y) atomicMin(&a.winner[(uint64_t)inst * a.nrec + w.x], g);
    }
  }
}

__global__ void yard_kernel(uint32_t* x, const uint32_t* y, uint64_t n4) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 a = reinterpret_cast<uint4*>(x)[i];
    const uint4 b = ld16_nt(reinterpret_cast<const uint4*>(y) + i);
    a.x += b.x, a.y += b.y, a.z += b.z, a.w += b.w;
    reinterpret_cast<uint4*>(x)[i] = a;
  }
}

// ---------------------------------------------------------------------------------------------
struct Set {
  Args a;
  std::vector<uint32_t> h_bal;  // initial offsets (for the check)
};

static uint32_t sizes_split(uint64_t L, uint32_t k, uint32_t j) { return (uint32_t)((j + 1) * L / k - j * L / k); }

int main(int argc, char** argv) {
  const uint64_t N = argc > 1 ? strtoull(argv[1], 0, 10) : (1ull << 20);
  const uint32_t B = argc > 2 ? atoi(argv[2]) : 16;
  const uint32_t R = argc > 3 ? atoi(argv[3]) : 16;
  const int which = argc > 4 ? atoi(argv[4]) : -1;
  const uint32_t nrec = 1024;
  // committees: 64 slots x cps (casper/sharding.go)
  const uint32_t cps = (uint32_t)(N / 16384 + 1);
  std::vector<uint32_t> cstart{0};
  for (uint32_t s = 0; s < 64; ++s)
    for (uint32_t j = 0; j < cps; ++j) cstart.push_back(cstart.back() + sizes_split(N / 64, cps, j));
  const uint32_t ncomm = (uint32_t)cstart.size() - 1, natt = ncomm + 1;
  // ranges: committee-aligned, ~N/R positions each
  std::vector<uint4> rdesc(R);
  std::vector<uint32_t> wdesc;
  uint32_t maxc = 0, maxspan = 0;
  {
    uint32_t c = 0;
    for (uint32_t r = 0; r < R; ++r) {
      const uint64_t t = N * (r + 1) / R;
      uint32_t c1 = c;
      while (c1 < ncomm && (r == R - 1 || cstart[c1 + 1] <= t)) ++c1;
      const uint64_t P0 = cstart[c], P1 = cstart[c1], P0a = P0 & ~3ull;
      const uint32_t nwin = (uint32_t)((P1 - P0a + 255) / 256);
      rdesc[r] = make_uint4(c, c1, (uint32_t)wdesc.size(), nwin);
      uint32_t cc = c;
      for (uint32_t k = 0; k < nwin; ++k) {
        const uint64_t ws = P0a + 256ull * k;
        while (cc + 1 < c1 && cstart[cc + 1] <= ws) ++cc;
        wdesc.push_back(cc);
      }
      maxc = std::max(maxc, c1 - c);
      maxspan = std::max<uint32_t>(maxspan, (uint32_t)(P1 - P0a));
      c = c1;
    }
  }
  const uint64_t vstride = (N + 3) & ~3ull;
  const uint64_t lastb = (N + 7) / 8;
  const uint32_t lbytes = (uint32_t)((lastb + 32 + 15) & ~15ull);
  const uint32_t vwords = (maxspan + 256) / 32 + 4;
  const size_t ldsb = lbytes + 4ull * vwords + 4ull * ((maxc + 2) & ~1u) + 16ull * maxc + maxc + 16;
  setvbuf(stdout, nullptr, _IONBF, 0);
  printf("N %llu B %u R %u ncomm %u maxc %u maxspan %u lds %zu\n", (unsigned long long)N, B, R, ncomm, maxc, maxspan,
         ldsb);
  // blens per instance
  std::vector<uint64_t> blen(natt);
  for (uint32_t c = 0; c < ncomm; ++c) blen[c] = (cstart[c + 1] - cstart[c] + 7) / 8;
  blen[ncomm] = lastb;
  const uint64_t per = std::accumulate(blen.begin(), blen.end(), 0ull);
  const int nsets = std::max<int>(4, (int)((800000000ull + N * B * 8 - 1) / (N * B * 8)));
  std::mt19937_64 rng(7);
  std::vector<uint32_t> perm(N);
  std::iota(perm.begin(), perm.end(), 0u);
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<Set> sets(nsets);
  std::vector<uint32_t> h_csize((size_t)B * natt);
  for (uint32_t b = 0; b < B; ++b)
    for (uint32_t g = 0; g < natt; ++g) h_csize[(size_t)b * natt + g] = g < ncomm ? cstart[g + 1] - cstart[g] : cstart[ncomm] - cstart[ncomm - 1];
  std::vector<uint64_t> h_boffs((size_t)B * natt + 1, 0);
  for (uint64_t i = 0; i < (uint64_t)B * natt; ++i) h_boffs[i + 1] = h_boffs[i] + blen[i % natt];
  std::vector<uint4> h_cinfo((size_t)B * ncomm);
  for (uint32_t b = 0; b < B; ++b)
    for (uint32_t c = 0; c < ncomm; ++c) {
      const uint64_t bo = h_boffs[(uint64_t)b * natt + c];
      h_cinfo[(size_t)b * ncomm + c] = make_uint4((uint32_t)bo, (uint32_t)(bo >> 32), c, 0);
    }
  std::vector<uint2> h_aw((size_t)B * natt);
  for (uint32_t b = 0; b < B; ++b)
    for (uint32_t g = 0; g < natt; ++g) h_aw[(size_t)b * natt + g] = make_uint2(g % nrec, 0);
  uint32_t *d_csize, *d_cstart, *d_wdesc;
  uint4 *d_rdesc, *d_cinfo;
  uint64_t* d_boffs;
  uint2* d_aw;
  CK(hipMalloc(&d_csize, h_csize.size() * 4));
  CK(hipMemcpy(d_csize, h_csize.data(), h_csize.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_cstart, cstart.size() * 4));
  CK(hipMemcpy(d_cstart, cstart.data(), cstart.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_wdesc, wdesc.size() * 4));
  CK(hipMemcpy(d_wdesc, wdesc.data(), wdesc.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_rdesc, rdesc.size() * 16));
  CK(hipMemcpy(d_rdesc, rdesc.data(), rdesc.size() * 16, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_cinfo, h_cinfo.size() * 16));
  CK(hipMemcpy(d_cinfo, h_cinfo.data(), h_cinfo.size() * 16, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_boffs, h_boffs.size() * 8));
  CK(hipMemcpy(d_boffs, h_boffs.data(), h_boffs.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_aw, h_aw.size() * 8));
  CK(hipMemcpy(d_aw, h_aw.data(), h_aw.size() * 8, hipMemcpyHostToDevice));
  std::vector<uint8_t> h_bits0;
  std::vector<uint64_t> h_base0;
  for (int k = 0; k < nsets; ++k) {
    Args& a = sets[k].a;
    std::memset(&a, 0, sizeof a);
    a.B = B, a.R = R, a.natt = natt, a.ncomm = ncomm, a.nrec = nrec, a.N = N, a.vstride = vstride;
    std::vector<uint32_t> bal((size_t)B * vstride), se((size_t)B * vstride, 0xFFFF0000u);
    std::vector<uint64_t> base(B), tdep(B, 0), dyn(B, 1);
    for (uint32_t b = 0; b < B; ++b) {
      base[b] = 16 - (1ull << 30);
      for (uint64_t p = 0; p < vstride; ++p) {
        const uint32_t x = 16 + (uint32_t)(rng() % 33);
        bal[(size_t)b * vstride + p] = p < N ? (uint32_t)(x + (1ull << 30) - 16) : 0;
        if (p < N) tdep[b] += x;
      }
    }
    std::vector<uint8_t> bits(per * B + 64);
    for (auto& x : bits) x = (uint8_t)(rng() | rng());
    // trailing bits clear
    for (uint64_t i = 0; i < (uint64_t)B * natt; ++i) {
      const uint32_t g = (uint32_t)(i % natt);
      const uint64_t kb = g < ncomm ? cstart[g + 1] - cstart[g] : N;
      if (kb % 8) bits[h_boffs[i + 1] - 1] &= (uint8_t)(0xFF << (8 - kb % 8));
    }
    sets[k].h_bal = bal;
    if (k == 0) h_bits0 = bits, h_base0 = base;
    uint32_t *d_bal, *d_se, *d_ci, *d_win;
    uint64_t *d_base, *d_tdep, *d_dyn, *d_vote, *d_total, *d_scal;
    uint8_t* d_bits;
    CK(hipMalloc(&d_bal, bal.size() * 4));
    CK(hipMemcpy(d_bal, bal.data(), bal.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_se, se.size() * 4));
    CK(hipMemcpy(d_se, se.data(), se.size() * 4, hipMemcpyHostToDevice));
    std::vector<uint32_t> ci(vstride, 0);
    for (uint64_t p = 0; p < N; ++p) ci[p] = perm[p];
    CK(hipMalloc(&d_ci, ci.size() * 4));
    CK(hipMemcpy(d_ci, ci.data(), ci.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_bits, bits.size()));
    CK(hipMemcpy(d_bits, bits.data(), bits.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_base, B * 8));
    CK(hipMemcpy(d_base, base.data(), B * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_tdep, B * 8));
    CK(hipMemcpy(d_tdep, tdep.data(), B * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_dyn, B * 8));
    CK(hipMemcpy(d_dyn, dyn.data(), B * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_vote, (size_t)B * natt * 8));
    CK(hipMalloc(&d_total, (size_t)B * natt * 8));
    CK(hipMalloc(&d_win, (size_t)B * nrec * 4));
    CK(hipMalloc(&d_scal, (size_t)B * 64));
    CK(hipMemset(d_scal, 0, (size_t)B * 64));
    a.bal32 = d_bal, a.base = d_base, a.se16 = d_se, a.co_index = d_ci, a.bits = d_bits, a.boffs = d_boffs;
    a.csize = d_csize, a.cstart = d_cstart, a.rdesc = d_rdesc, a.wdesc = d_wdesc, a.cinfo = d_cinfo, a.att_win = d_aw;
    a.dyn = d_dyn, a.tdep = d_tdep, a.vote = d_vote, a.total = d_total, a.winner = d_win, a.scal = d_scal;
    a.maxc = maxc, a.lbytes = lbytes, a.vwords = vwords;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int steps = nsets * ((48 + nsets - 1) / nsets);
  auto timeit = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w)
      for (int k = 0; k < nsets; ++k) launch(k);
    CK(hipDeviceSynchronize());
    float best = 1e9, tot = 0;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < steps; ++i) launch(i % nsets);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms / steps);
      tot += ms / steps;
    }
    const double bytes = (double)N * B * 12.25;
    printf("%-44s %8.2f us/step (best of 3; mean %.2f)  %.3f of 8 TB/s by 12.25 B\n", name, best * 1e3, tot / 3 * 1e3,
           bytes / (best * 1e-3) / 8e12);
    fflush(stdout);
  };
  // yardstick: x += y over the same element count (12 B per element), cold rotation
  {
    std::vector<uint32_t*> ys(nsets);
    for (int k = 0; k < nsets; ++k) CK(hipMalloc(&ys[k], (size_t)B * vstride * 4));
    timeit("yardstick x+=y (int32, 12 B/elem)", [&](int k) {
      hipLaunchKernelGGL(yard_kernel, dim3(2048), dim3(256), 0, 0, sets[k].a.bal32, ys[k], (uint64_t)B * vstride / 4);
    });
    for (auto y : ys) CK(hipFree(y));
  }
#define RUN(NT, D, FL, NAME)                                                                             \
  {                                                                                                      \
    CK(hipFuncSetAttribute((const void*)win_kernel<NT, D, FL>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                           (int)ldsb));                                                                  \
    timeit(NAME, [&](int k) {                                                                            \
      hipLaunchKernelGGL((win_kernel<NT, D, FL>), dim3(B * R), dim3(NT), ldsb, 0, sets[k].a);           \
    });                                                                                                  \
  }
  if (which < 0 || which == 0) RUN(1024, 2, 0, "window 1024t D2")
  if (which < 0 || which == 1) RUN(1024, 3, 0, "window 1024t D3")
  if (which < 0 || which == 2) RUN(512, 3, 0, "window 512t D3")
  if (which < 0 || which == 3) RUN(512, 4, 0, "window 512t D4")
  if (which < 0 || which == 4) RUN(1024, 2, 1, "window 1024t D2, reward bits from L2")
  if (which < 0 || which == 5) RUN(1024, 2, 2, "window 1024t D2, no tallies")
  if (which < 0 || which == 6) RUN(1024, 2, 4, "window 1024t D2, no prologue count")
  if (which < 0 || which == 7) RUN(1024, 2, 7, "window 1024t D2, none of the three")
  if (which < 0 || which == 8) RUN(1024, 2, 15, "window 1024t D2, nothing but loads")
  // ---- check set 0 after one fresh step against a CPU model ----
  {
    Args& a = sets[0].a;
    CK(hipMemcpy(a.bal32, sets[0].h_bal.data(), sets[0].h_bal.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(a.scal, 0, (size_t)B * 64));
    CK(hipMemset(a.winner, 0xFF, (size_t)B * nrec * 4));
    CK(hipMemset(a.vote, 0, (size_t)B * natt * 8));
    CK(hipMemset(a.total, 0, (size_t)B * natt * 8));
    CK(hipFuncSetAttribute((const void*)win_kernel<1024, 2, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsb));
    hipLaunchKernelGGL((win_kernel<1024, 2, 0>), dim3(B * R), dim3(1024), ldsb, 0, a);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> gb((size_t)B * vstride);
    std::vector<uint64_t> gv((size_t)B * natt), gt((size_t)B * natt), gs((size_t)B * 8);
    std::vector<uint32_t> gw((size_t)B * nrec);
    CK(hipMemcpy(gb.data(), a.bal32, gb.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gv.data(), a.vote, gv.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gt.data(), a.total, gt.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gs.data(), a.scal, gs.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gw.data(), a.winner, gw.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (uint32_t b = 0; b < B && bad < 5; b += (B > 4 ? B / 4 : 1)) {
      const uint64_t gbase = (uint64_t)b * natt;
      const uint8_t* bits = h_bits0.data();
      uint64_t pop = 0;
      for (uint64_t i = h_boffs[gbase]; i < h_boffs[gbase + natt]; ++i) pop += __builtin_popcount(bits[i]);
      uint64_t tdep = 0;
      const uint32_t* hb = sets[0].h_bal.data() + (size_t)b * vstride;
      for (uint64_t p = 0; p < N; ++p) tdep += hb[p] - (1ull << 30) + 16;
      const bool applied = pop * 96 >= tdep * 2;
      const uint8_t* lbf = bits + h_boffs[gbase + natt - 1];
      uint64_t nxt = 0;
      for (uint64_t p = 0; p < N; ++p) {
        const uint64_t bal = h_base0[b] + hb[p];
        const uint32_t v = perm[p];
        const bool rw = (lbf[v >> 3] >> (7 - (v & 7))) & 1;
        const uint64_t nb = applied ? (rw ? bal + 1 : bal - 1) : bal;
        nxt += nb;
        if ((uint32_t)(nb - h_base0[b]) != gb[(size_t)b * vstride + p] && bad++ < 5)
          printf("bal mismatch inst %u pos %llu\n", b, (unsigned long long)p);
      }
      if (gs[b * 8 + 5] != nxt && bad++ < 5) printf("next mismatch inst %u\n", b);
      if (gs[b * 8 + 0] != pop && bad++ < 5) printf("pop mismatch inst %u %llu %llu\n", b, (unsigned long long)gs[b * 8], (unsigned long long)pop);
      std::vector<uint32_t> win(nrec, 0xFFFFFFFFu);
      for (uint32_t c = 0; c < ncomm; ++c) {
        const uint8_t* bf = bits + h_boffs[gbase + c];
        uint64_t T = 0, V = 0;
        for (uint32_t j = 0; j < cstart[c + 1] - cstart[c]; ++j) {
          const uint64_t bal = h_base0[b] + hb[cstart[c] + j];
          T += bal;
          if ((bf[j >> 3] >> (7 - (j & 7))) & 1) V += bal;
        }
        if ((gt[gbase + c] != T || gv[gbase + c] != V) && bad++ < 5) printf("tally mismatch inst %u comm %u\n", b, c);
        if (3 * V >= 2 * T) win[c % nrec] = std::min(win[c % nrec], c);
      }
      for (uint32_t s = 0; s < nrec; ++s)
        if (win[s] != gw[(size_t)b * nrec + s] && bad++ < 5) printf("winner mismatch inst %u shard %u\n", b, s);
    }
    printf("check (window 1024t D2): %s\n", bad ? "MISMATCH" : "ok");
  }
  return 0;
}
