/* ORACLE (test infrastructure only) — portable C restatement of BLAKE2b-512 (RFC 7693),
 * the algorithm of golang.org/x/crypto/blake2b @ a49355c that the reference calls at
 * types/block.go:74, types/attestation.go:56,74, types/state.go:146,245.
 * Used as bench.py's cpu_baseline ("port") and cross-checked against hashlib in tests. */
#include <stdint.h>
#include <string.h>

static const uint64_t IV[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

static const uint8_t SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void compress(uint64_t h[8], const uint8_t blk[128], uint64_t t, int last) {
  uint64_t m[16], v[16];
  for (int i = 0; i < 16; ++i) memcpy(&m[i], blk + 8 * i, 8); /* little-endian host */
  for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = IV[i]; }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
#define GG(a, b, c, d, x, y)                                     \
  v[a] = v[a] + v[b] + (x); v[d] = rotr(v[d] ^ v[a], 32);        \
  v[c] = v[c] + v[d];       v[b] = rotr(v[b] ^ v[c], 24);        \
  v[a] = v[a] + v[b] + (y); v[d] = rotr(v[d] ^ v[a], 16);        \
  v[c] = v[c] + v[d];       v[b] = rotr(v[b] ^ v[c], 63);
  for (int r = 0; r < 12; ++r) {
    const uint8_t* s = SIGMA[r];
    GG(0, 4, 8, 12, m[s[0]], m[s[1]]);
    GG(1, 5, 9, 13, m[s[2]], m[s[3]]);
    GG(2, 6, 10, 14, m[s[4]], m[s[5]]);
    GG(3, 7, 11, 15, m[s[6]], m[s[7]]);
    GG(0, 5, 10, 15, m[s[8]], m[s[9]]);
    GG(1, 6, 11, 12, m[s[10]], m[s[11]]);
    GG(2, 7, 8, 13, m[s[12]], m[s[13]]);
    GG(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
#undef GG
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

void oracle_blake2b512(const uint8_t* msg, uint64_t len, uint8_t out[64]) {
  uint64_t h[8];
  memcpy(h, IV, sizeof h);
  h[0] ^= 0x01010040ULL;
  uint64_t off = 0;
  uint8_t blk[128];
  while (len - off > 128) {
    compress(h, msg + off, off + 128, 0);
    off += 128;
  }
  memset(blk, 0, sizeof blk);
  if (len - off) memcpy(blk, msg + off, len - off);
  compress(h, blk, len, 1);
  memcpy(out, h, 64);
}

/* n CSR messages -> n * out_bytes digest bytes */
void oracle_blake2b512_csr(const uint8_t* data, const uint64_t* offsets, uint64_t n, uint8_t* out,
                           uint32_t out_bytes) {
  uint8_t d[64];
  for (uint64_t i = 0; i < n; ++i) {
    oracle_blake2b512(data + offsets[i], offsets[i + 1] - offsets[i], d);
    memcpy(out + i * out_bytes, d, out_bytes);
  }
}

/* n fixed-length records of len bytes at stride */
void oracle_blake2b512_fixed(const uint8_t* data, uint64_t stride, uint64_t len, uint64_t n,
                             uint8_t* out, uint32_t out_bytes) {
  uint8_t d[64];
  for (uint64_t i = 0; i < n; ++i) {
    oracle_blake2b512(data + i * stride, len, d);
    memcpy(out + i * out_bytes, d, out_bytes);
  }
}
