// Host BLAKE2b-512 for long single messages (see serial_hash.h for why these stay on the
// host).  RFC 7693 BLAKE2b, the algorithm of golang.org/x/crypto/blake2b @ a49355c that the
// reference calls at types/state.go:146,245 for the state roots.
//
// The AVX2 path keeps the 4x4 state as four row vectors and runs the four column G functions
// (then the four diagonal ones) as one vector G, re-aligning rows with permute4x64 between the
// halves of a round; rotr32/24/16 are in-lane shuffles and rotr63 is (x >> 63) | (x + x).
#include <sched.h>
#include <cstdlib>
#include "serial_hash.h"

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

namespace pz {

namespace {

constexpr uint64_t kIV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                             0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                             0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

// Message schedule; rounds 10 and 11 reuse rows 0 and 1.
constexpr uint8_t kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

inline uint64_t load64(const uint8_t* p) {
  uint64_t x;
  std::memcpy(&x, p, 8);  // x86-64 is little-endian, as BLAKE2b's word order
  return x;
}

// ---- portable compression (hosts without AVX2) ----------------------------------------------
inline uint64_t ror(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

void compress_scalar(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  uint64_t v[16];
  for (int i = 0; i < 8; ++i) v[i] = h[i], v[8 + i] = kIV[i];
  v[12] ^= t;
  if (last) v[14] = ~v[14];
  auto g = [&](int a, int b, int c, int d, uint64_t x, uint64_t y) {
    v[a] += v[b] + x;
    v[d] = ror(v[d] ^ v[a], 32);
    v[c] += v[d];
    v[b] = ror(v[b] ^ v[c], 24);
    v[a] += v[b] + y;
    v[d] = ror(v[d] ^ v[a], 16);
    v[c] += v[d];
    v[b] = ror(v[b] ^ v[c], 63);
  };
  for (int r = 0; r < 12; ++r) {
    const uint8_t* s = kSigma[r % 10];
    g(0, 4, 8, 12, m[s[0]], m[s[1]]);
    g(1, 5, 9, 13, m[s[2]], m[s[3]]);
    g(2, 6, 10, 14, m[s[4]], m[s[5]]);
    g(3, 7, 11, 15, m[s[6]], m[s[7]]);
    g(0, 5, 10, 15, m[s[8]], m[s[9]]);
    g(1, 6, 11, 12, m[s[10]], m[s[11]]);
    g(2, 7, 8, 13, m[s[12]], m[s[13]]);
    g(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[8 + i];
}

// ---- AVX2 row-vector compression ------------------------------------------------------------
__attribute__((target("avx2"))) inline __m256i vrot24(__m256i x) {
  const __m256i k = _mm256_setr_epi8(3, 4, 5, 6, 7, 0, 1, 2, 11, 12, 13, 14, 15, 8, 9, 10, 3, 4, 5, 6, 7, 0, 1, 2, 11,
                                     12, 13, 14, 15, 8, 9, 10);
  return _mm256_shuffle_epi8(x, k);
}
__attribute__((target("avx2"))) inline __m256i vrot16(__m256i x) {
  const __m256i k = _mm256_setr_epi8(2, 3, 4, 5, 6, 7, 0, 1, 10, 11, 12, 13, 14, 15, 8, 9, 2, 3, 4, 5, 6, 7, 0, 1, 10,
                                     11, 12, 13, 14, 15, 8, 9);
  return _mm256_shuffle_epi8(x, k);
}

// One vector G over four (a, b, c, d) columns with message words x, y.
#define PZ_VG(A, B, C, D, X, Y)                                         \
  do {                                                                  \
    A = _mm256_add_epi64(_mm256_add_epi64(A, B), X);                     \
    D = _mm256_shuffle_epi32(_mm256_xor_si256(D, A), 0xB1);              \
    C = _mm256_add_epi64(C, D);                                          \
    B = vrot24(_mm256_xor_si256(B, C));                                  \
    A = _mm256_add_epi64(_mm256_add_epi64(A, B), Y);                     \
    D = vrot16(_mm256_xor_si256(D, A));                                  \
    C = _mm256_add_epi64(C, D);                                          \
    B = _mm256_xor_si256(B, C);                                          \
    B = _mm256_or_si256(_mm256_srli_epi64(B, 63), _mm256_add_epi64(B, B)); \
  } while (0)

__attribute__((target("avx2"))) void compress_avx2(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(h));
  __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(h + 4));
  __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(kIV));
  __m256i d = _mm256_set_epi64x((long long)kIV[7], (long long)(last ? ~kIV[6] : kIV[6]),
                                (long long)kIV[5], (long long)(kIV[4] ^ t));
  const __m256i a0 = a, b0 = b;
  for (int r = 0; r < 12; ++r) {
    const uint8_t* s = kSigma[r % 10];
    const __m256i x0 = _mm256_set_epi64x((long long)m[s[6]], (long long)m[s[4]], (long long)m[s[2]], (long long)m[s[0]]);
    const __m256i y0 = _mm256_set_epi64x((long long)m[s[7]], (long long)m[s[5]], (long long)m[s[3]], (long long)m[s[1]]);
    PZ_VG(a, b, c, d, x0, y0);
    // diagonalise: columns become (v0,v5,v10,v15), (v1,v6,v11,v12), (v2,v7,v8,v13), (v3,v4,v9,v14)
    b = _mm256_permute4x64_epi64(b, 0x39);
    c = _mm256_permute4x64_epi64(c, 0x4E);
    d = _mm256_permute4x64_epi64(d, 0x93);
    const __m256i x1 = _mm256_set_epi64x((long long)m[s[14]], (long long)m[s[12]], (long long)m[s[10]], (long long)m[s[8]]);
    const __m256i y1 = _mm256_set_epi64x((long long)m[s[15]], (long long)m[s[13]], (long long)m[s[11]], (long long)m[s[9]]);
    PZ_VG(a, b, c, d, x1, y1);
    b = _mm256_permute4x64_epi64(b, 0x93);
    c = _mm256_permute4x64_epi64(c, 0x4E);
    d = _mm256_permute4x64_epi64(d, 0x39);
  }
  a = _mm256_xor_si256(a0, _mm256_xor_si256(a, c));
  b = _mm256_xor_si256(b0, _mm256_xor_si256(b, d));
  _mm256_storeu_si256(reinterpret_cast<__m256i*>(h), a);
  _mm256_storeu_si256(reinterpret_cast<__m256i*>(h + 4), b);
}
#undef PZ_VG

using CompressFn = void (*)(uint64_t*, const uint64_t*, uint64_t, bool);

CompressFn pick() { return __builtin_cpu_supports("avx2") ? compress_avx2 : compress_scalar; }

std::atomic<uint64_t> g_threshold{64 * 1024};
std::atomic<uint64_t> g_small{PZ_SMALL_BATCH_DEFAULT};

}  // namespace

void host_blake2b512(const uint8_t* msg, size_t len, uint8_t out[64]) {
  static const CompressFn compress = pick();
  uint64_t h[8];
  for (int i = 0; i < 8; ++i) h[i] = kIV[i];
  h[0] ^= 0x01010040ULL;  // parameter block: digest length 64, key length 0, fanout 1, depth 1
  uint64_t m[16];
  size_t off = 0;
  while (len - off > 128) {  // every block but the last
    for (int i = 0; i < 16; ++i) m[i] = load64(msg + off + 8 * i);
    off += 128;
    compress(h, m, (uint64_t)off, false);
  }
  uint8_t tail[128] = {0};  // the final (possibly partial or empty) block, zero-padded
  if (len > off) std::memcpy(tail, msg + off, len - off);
  for (int i = 0; i < 16; ++i) m[i] = load64(tail + 8 * i);
  compress(h, m, (uint64_t)len, true);
  std::memcpy(out, h, 64);
}

void host_blake2b512_many(const uint8_t* data, const uint64_t* offsets, const std::vector<uint64_t>& which,
                          uint8_t* out, uint32_t out_bytes, unsigned threads) {
  if (which.empty()) return;
  std::atomic<size_t> next{0};
  auto worker = [&]() {
    uint8_t d[64];
    for (size_t k; (k = next.fetch_add(1)) < which.size();) {
      const uint64_t i = which[k];
      host_blake2b512(data + offsets[i], offsets[i + 1] - offsets[i], d);
      std::memcpy(out + i * out_bytes, d, out_bytes);
    }
  };
  const unsigned nt = std::max(1u, std::min<unsigned>(threads, (unsigned)which.size()));
  std::vector<std::thread> pool;
  for (unsigned t = 1; t < nt; ++t) pool.emplace_back(worker);
  worker();  // the calling thread works too
  for (auto& t : pool) t.join();
}

uint64_t serial_threshold() { return g_threshold.load(); }
uint64_t small_batch_threshold() { return g_small.load(); }
uint64_t set_small_batch_threshold(uint64_t c) { return g_small.exchange(c); }
uint64_t set_serial_threshold(uint64_t bytes) { return g_threshold.exchange(bytes); }

}  // namespace pz

namespace pz {

// Host threads for the serial hashes (and the chain's parse): min(16, the affinity set) unless
// pz_set_host_threads chose a count (16: the CPU share of one GPU on the bench boxes).
static std::atomic<unsigned> g_host_threads{0};
unsigned host_threads() {
  const unsigned v = g_host_threads.load();
  if (v) return v;
  static const unsigned n = [] {
    unsigned c = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) c = std::max(1, CPU_COUNT(&set));
    return std::min(16u, c);
  }();
  return n;
}
unsigned set_host_threads(unsigned n) { return g_host_threads.exchange(n > 256 ? 256 : n); }

std::vector<uint64_t> long_messages(const uint64_t* offsets, uint64_t n) {
  std::vector<uint64_t> w;
  const uint64_t thr = serial_threshold();
  for (uint64_t i = 0; i < n; ++i)
    if (offsets[i + 1] - offsets[i] >= thr) w.push_back(i);
  return w;
}

void SerialHashJob::start(const uint8_t* data, const uint64_t* offsets, std::vector<uint64_t> which, uint8_t* out,
                          uint32_t out_bytes) {
  join();
  which_ = std::move(which);
  if (which_.empty()) return;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const unsigned nt = std::min(8u, hw);
  thread_ = new std::thread([this, data, offsets, out, out_bytes, nt]() {
    host_blake2b512_many(data, offsets, which_, out, out_bytes, nt);
  });
}

void SerialHashJob::join() {
  if (!thread_) return;
  auto* t = static_cast<std::thread*>(thread_);
  t->join();
  delete t;
  thread_ = nullptr;
}

}  // namespace pz

#ifdef PZ_AB_BUILD
// Internal (tests, the A/B library): the host hasher on one message.
extern "C" void pz_debug_host_blake2b512(const uint8_t* msg, uint64_t len, uint8_t out[64]) {
  pz::host_blake2b512(msg, (size_t)len, out);
}
#endif
