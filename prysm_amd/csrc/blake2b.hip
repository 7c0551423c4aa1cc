// BLAKE2b-512 batch kernels for gfx950 (CDNA4, wave64).
//
// Restates RFC 7693 (the algorithm of golang.org/x/crypto/blake2b @ a49355c, which the
// reference calls at types/block.go:74, types/attestation.go:56,74, types/state.go:146,245,
// blockchain/core.go:290 and utils/shuffle.go:19) as one-lane-per-message integer code:
//   * the 16-word state v[] and the chaining value h[] live in VGPR pairs;
//   * 64-bit adds lower to v_lshl_add_u64 (one VALU op on gfx950);
//   * rotr 32 is a register-pair swap, rotr 24/16/63 are two v_alignbit_b32 each;
//   * 12 rounds are fully unrolled so sigma[] indexes registers statically.
// Fixed-length records are staged global->LDS with coalesced 16-byte loads (8 lanes cover
// one 128-byte block) and read back one row per lane; variable-length (CSR) messages are
// read per lane with dword loads + v_alignbit funnel shifts.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "blake2b_kernels.h"

namespace pz {

#define IV0 0x6a09e667f3bcc908ULL
#define IV1 0xbb67ae8584caa73bULL
#define IV2 0x3c6ef372fe94f82bULL
#define IV3 0xa54ff53a5f1d36f1ULL
#define IV4 0x510e527fade682d1ULL
#define IV5 0x9b05688c2b3e6c1fULL
#define IV6 0x1f83d9abfb41bd6bULL
#define IV7 0x5be0cd19137e2179ULL

__device__ __forceinline__ uint64_t pack(uint32_t lo, uint32_t hi) {
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t rotr32(uint64_t x) { return (x >> 32) | (x << 32); }
__device__ __forceinline__ uint64_t rotr24(uint64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return pack(__builtin_amdgcn_alignbit(hi, lo, 24), __builtin_amdgcn_alignbit(lo, hi, 24));
}
__device__ __forceinline__ uint64_t rotr16(uint64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return pack(__builtin_amdgcn_alignbit(hi, lo, 16), __builtin_amdgcn_alignbit(lo, hi, 16));
}
__device__ __forceinline__ uint64_t rotr63(uint64_t x) {  // == rotl 1
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return pack(__builtin_amdgcn_alignbit(lo, hi, 31), __builtin_amdgcn_alignbit(hi, lo, 31));
}

#define G(a, b, c, d, x, y)        \
  do {                             \
    a = a + b + (x);               \
    d = rotr32(d ^ a);             \
    c = c + d;                     \
    b = rotr24(b ^ c);             \
    a = a + b + (y);               \
    d = rotr16(d ^ a);             \
    c = c + d;                     \
    b = rotr63(b ^ c);             \
  } while (0)

// One round with the message permutation sigma[r] spelled out as literals (RFC 7693 §2.7).
#define ROUND(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  do {                                                                             \
    G(v0, v4, v8, v12, m[s0], m[s1]);                                              \
    G(v1, v5, v9, v13, m[s2], m[s3]);                                              \
    G(v2, v6, v10, v14, m[s4], m[s5]);                                             \
    G(v3, v7, v11, v15, m[s6], m[s7]);                                             \
    G(v0, v5, v10, v15, m[s8], m[s9]);                                             \
    G(v1, v6, v11, v12, m[s10], m[s11]);                                           \
    G(v2, v7, v8, v13, m[s12], m[s13]);                                            \
    G(v3, v4, v9, v14, m[s14], m[s15]);                                            \
  } while (0)

// RFC 7693 compression function F(h, m, t, f); t < 2^64 here (messages < 16 EiB).
__device__ __forceinline__ void compress(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                         bool last) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3];
  uint64_t v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3;
  uint64_t v12 = IV4 ^ t, v13 = IV5, v14 = last ? ~IV6 : IV6, v15 = IV7;
  ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3);
  ROUND(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4);
  ROUND(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8);
  ROUND(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13);
  ROUND(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9);
  ROUND(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11);
  ROUND(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10);
  ROUND(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5);
  ROUND(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0);
  ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3);
  h[0] ^= v0 ^ v8;
  h[1] ^= v1 ^ v9;
  h[2] ^= v2 ^ v10;
  h[3] ^= v3 ^ v11;
  h[4] ^= v4 ^ v12;
  h[5] ^= v5 ^ v13;
  h[6] ^= v6 ^ v14;
  h[7] ^= v7 ^ v15;
}

__device__ __forceinline__ void init_h(uint64_t h[8]) {
  // parameter block: digest length 64, key length 0, fanout 1, depth 1
  h[0] = IV0 ^ 0x01010040ULL;
  h[1] = IV1; h[2] = IV2; h[3] = IV3; h[4] = IV4; h[5] = IV5; h[6] = IV6; h[7] = IV7;
}

__device__ __forceinline__ void store_digest(uint8_t* out, const uint64_t h[8], uint32_t out_bytes) {
  // out is 32- or 64-byte aligned per message (out + i*out_bytes with a 16-B aligned base)
  uint4* o = reinterpret_cast<uint4*>(out);
  o[0] = make_uint4((uint32_t)h[0], (uint32_t)(h[0] >> 32), (uint32_t)h[1], (uint32_t)(h[1] >> 32));
  o[1] = make_uint4((uint32_t)h[2], (uint32_t)(h[2] >> 32), (uint32_t)h[3], (uint32_t)(h[3] >> 32));
  if (out_bytes == 64) {
    o[2] = make_uint4((uint32_t)h[4], (uint32_t)(h[4] >> 32), (uint32_t)h[5], (uint32_t)(h[5] >> 32));
    o[3] = make_uint4((uint32_t)h[6], (uint32_t)(h[6] >> 32), (uint32_t)h[7], (uint32_t)(h[7] >> 32));
  }
}

// Zero bytes [keep, 16) of a 16-byte chunk (keep in 0..16).
__device__ __forceinline__ uint4 mask_chunk(uint4 c, uint32_t keep) {
  uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int lo = 4 * k;
    uint32_t valid = keep <= (uint32_t)lo ? 0u : (keep >= (uint32_t)lo + 4 ? 4u : keep - lo);
    uint32_t msk = valid >= 4 ? 0xffffffffu : ((1u << (8 * valid)) - 1u);
    w[k] &= msk;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ------------------------------------------------------------------------------------------
// Fixed-length records, LDS-staged.  One wave = 64 consecutive messages; each wave owns a
// private LDS slab [64 rows][144 B] (128-B block + 16-B pad: conflict-free ds_read_b128).
// ------------------------------------------------------------------------------------------
constexpr int kWavesPerBlock = 4;
constexpr int kRowBytes = 144;
constexpr int kSlabBytes = 64 * kRowBytes;

// Requires stride < 2^26 (64 messages x stride fit 32-bit offsets; the launcher checks).
extern "C" __global__ void __launch_bounds__(256)
pz_b2b_fixed_kernel(const uint8_t* __restrict__ msgs, uint64_t stride, uint64_t len, uint64_t n,
                    uint8_t* __restrict__ out, uint32_t out_bytes) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerBlock * kSlabBytes];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform -> SGPR math
  uint8_t* slab = lds + wave * kSlabBytes;
  const uint64_t m0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wave) * 64;
  if (m0 >= n) return;  // whole wave idle (wave-uniform)
  const uint64_t msg = m0 + lane;
  const uint64_t nblocks = len == 0 ? 1 : (len + 127) / 128;
  // Chunk `it` of this lane: message row r = it*8 + lane/8, 16-byte part lane%8.  A wave
  // instruction therefore reads 8 whole 128-B lines; offsets are 32-bit against the
  // wave-uniform base (SGPR pair), so the address math stays out of the 64-bit VALU.
  const uint8_t* wbase = msgs + m0 * stride;
  const uint32_t lrow = (uint32_t)lane >> 3, lpart = (uint32_t)lane & 7;
  const uint32_t s32 = (uint32_t)stride;
  const bool full_wave = m0 + 64 <= n;
  const uint32_t rows_left = full_wave ? 64u : (uint32_t)(n - m0);

  uint64_t h[8];
  init_h(h);
  for (uint64_t t = 0; t < nblocks; ++t) {
    // ---- stage: 512 16-byte chunks (64 msgs x 8 parts), 8 per lane, all loads in flight
    const uint32_t boff = (uint32_t)t * 128u + lpart * 16u;
    uint4 v[8];
    if (full_wave && (t + 1 < nblocks || (len & 127) == 0)) {  // wave-uniform fast path
#pragma unroll
      for (int it = 0; it < 8; ++it)
        v[it] = *reinterpret_cast<const uint4*>(wbase + ((it * 8u + lrow) * s32 + boff));
    } else {  // tail wave / partial last block: clamp addresses, zero what lies outside
      const uint32_t safe_off = boff < (uint32_t)len ? boff : 0u;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const uint32_t r = it * 8u + lrow;
        const bool ok = r < rows_left && boff < (uint32_t)len;
        const uint32_t rr = r < rows_left ? r : 0u;
        uint4 q = *reinterpret_cast<const uint4*>(wbase + (rr * s32 + safe_off));
        if (boff + 16 > (uint32_t)len) q = mask_chunk(q, boff < (uint32_t)len ? (uint32_t)len - boff : 0u);
        v[it] = ok ? q : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int it = 0; it < 8; ++it)
      *reinterpret_cast<uint4*>(slab + (it * 8 + lrow) * kRowBytes + lpart * 16) = v[it];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- read this lane's row
    uint64_t m[16];
    const uint4* row = reinterpret_cast<const uint4*>(slab + lane * kRowBytes);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint4 q = row[k];
      m[2 * k] = pack(q.x, q.y);
      m[2 * k + 1] = pack(q.z, q.w);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool last = (t + 1 == nblocks);
    const uint64_t ctr = last ? len : (t + 1) * 128;
    compress(h, m, ctr, last);
  }
  if (msg < n) store_digest(out + msg * out_bytes, h, out_bytes);
}

// ------------------------------------------------------------------------------------------
// Persistent variant: the grid is sized to the resident waves and every wave walks groups of
// 64 messages g, g+W, g+2W, ...  As soon as a block's 16 message words are in registers the
// wave's LDS slab is free, so the NEXT block (of this group, or the first block of the wave's
// next group) is fetched into it by LDS-DMA (global_load_lds_dwordx4: no VGPRs, no
// ds_write) while the current block is compressed.  DMA writes each wave-instruction's 1 KiB
// linearly, so rows are unpadded 128 B and the bank-conflict fix moves to the SOURCE: 16-B
// chunk k of message row r is stored at position k ^ ((r >> 1) & 7), which makes every
// ds_read_b128 lane group hit 16 distinct 16-B bank quads.
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

constexpr int kDmaSlabBytes = 64 * 128;  // 8 KiB per wave

struct FixedGeom {
  const uint8_t* msgs;
  uint64_t stride, len, n, ngroups, nblocks;
  uint32_t lrow, lpart, s32;
};

__device__ __forceinline__ uint32_t chunk_pos(uint32_t r, uint32_t k) { return k ^ ((r >> 1) & 7u); }

__device__ __forceinline__ bool block_is_full(const FixedGeom& G, uint64_t g, uint64_t t) {
  return g * 64 + 64 <= G.n && (t + 1 < G.nblocks || (G.len & 127) == 0);
}

// Full block: 8 DMA instructions.  Instruction `it`, lane L fills row r = it*8 + L/8 at
// position p = L%8, i.e. global chunk k = p ^ ((r>>1)&7) (the swizzle is an involution).
__device__ __forceinline__ void dma_block(uint8_t* slab, const FixedGeom& G, uint64_t g, uint64_t t) {
  const uint8_t* wbase = G.msgs + g * 64 * G.stride;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const uint32_t r = it * 8u + G.lrow;
    const uint32_t k = chunk_pos(r, G.lpart);
    const uint8_t* src = wbase + (r * G.s32 + (uint32_t)t * 128u + k * 16u);
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(slab + it * 1024), 16, 0, 0);
  }
}

// Tail wave / partial last block: register path with clamped addresses and zero masking,
// written into the same swizzled layout.
__device__ __forceinline__ void reg_block(uint8_t* slab, const FixedGeom& G, uint64_t g, uint64_t t) {
  const uint64_t m0 = g * 64;
  const uint8_t* wbase = G.msgs + m0 * G.stride;
  const uint32_t rows_left = m0 + 64 <= G.n ? 64u : (uint32_t)(G.n - m0);
  const uint32_t len = (uint32_t)G.len;
  const uint32_t boff = (uint32_t)t * 128u + G.lpart * 16u;
  const uint32_t safe_off = boff < len ? boff : 0u;
  uint4 v[8];
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const uint32_t r = it * 8u + G.lrow;
    const bool ok = r < rows_left && boff < len;
    const uint32_t rr = r < rows_left ? r : 0u;
    uint4 q = *reinterpret_cast<const uint4*>(wbase + (rr * G.s32 + safe_off));
    if (boff + 16 > len) q = mask_chunk(q, boff < len ? len - boff : 0u);
    v[it] = ok ? q : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const uint32_t r = it * 8u + G.lrow;
    *reinterpret_cast<uint4*>(slab + r * 128u + chunk_pos(r, G.lpart) * 16u) = v[it];
  }
}

__device__ __forceinline__ void read_block_words(const uint8_t* slab, int lane, uint64_t m[16]) {
  const uint32_t r = (uint32_t)lane;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 q = *reinterpret_cast<const uint4*>(slab + r * 128u + chunk_pos(r, (uint32_t)k) * 16u);
    m[2 * k] = pack(q.x, q.y);
    m[2 * k + 1] = pack(q.z, q.w);
  }
}

extern "C" __global__ void __launch_bounds__(256)
pz_b2b_fixed_persistent_kernel(const uint8_t* __restrict__ msgs, uint64_t stride, uint64_t len, uint64_t n,
                               uint8_t* __restrict__ out, uint32_t out_bytes) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerBlock * kDmaSlabBytes];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform -> SGPR math
  uint8_t* slab = lds + wave * kDmaSlabBytes;
  FixedGeom G;
  G.msgs = msgs; G.stride = stride; G.len = len; G.n = n;
  G.ngroups = (n + 63) / 64;
  G.nblocks = len == 0 ? 1 : (len + 127) / 128;
  G.lrow = (uint32_t)lane >> 3; G.lpart = (uint32_t)lane & 7; G.s32 = (uint32_t)stride;
  const uint64_t W = (uint64_t)gridDim.x * kWavesPerBlock;
  uint64_t g = (uint64_t)blockIdx.x * kWavesPerBlock + wave;
  if (g >= G.ngroups) return;  // wave-uniform
  // Host contract (launch_b2b_fixed): n % 64 == 0 and stride >= nblocks*128, so every DMA
  // reads whole 128-B blocks inside the record's own stride slot; bytes past `len` in the
  // last block are zeroed in registers.
  const uint32_t tail = (uint32_t)(G.len - (G.nblocks - 1) * 128);  // 0..128 valid bytes of the last block
  uint64_t t = 0;
  uint64_t h[8];
  dma_block(slab, G, g, 0);
  while (true) {  // flattened walk over this wave's (group, block) pairs
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint64_t m[16];
    read_block_words(slab, lane, m);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // words in VGPRs: the slab is free
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t nt = t + 1 < G.nblocks ? t + 1 : 0;
    const uint64_t ng = t + 1 < G.nblocks ? g : g + W;
    if (ng < G.ngroups) dma_block(slab, G, ng, nt);  // lands while this block is compressed
    if (t == 0) init_h(h);
    const bool last = (t + 1 == G.nblocks);
    if (last && tail < 128) {  // wave-uniform: zero bytes >= len of a partial last block
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t lo = 8u * k;
        const uint32_t valid = tail <= lo ? 0u : (tail >= lo + 8 ? 8u : tail - lo);
        m[k] &= valid >= 8 ? ~0ull : ((1ull << (8 * valid)) - 1ull);
      }
    }
    compress(h, m, last ? G.len : (t + 1) * 128, last);
    if (last) {
      const uint64_t msg = g * 64 + lane;
      if (msg < n) store_digest(out + msg * out_bytes, h, out_bytes);
    }
    t = nt;
    g = ng;
    if (g >= G.ngroups) break;
  }
}

// ------------------------------------------------------------------------------------------
// CSR (variable-length) messages: one lane per message, per-lane dword loads.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t load_dword_tail(const uint8_t* p, uint32_t nbytes) {
  // nbytes in 1..3: byte loads so nothing past the message is touched
  uint32_t w = p[0];
  if (nbytes > 1) w |= (uint32_t)p[1] << 8;
  if (nbytes > 2) w |= (uint32_t)p[2] << 16;
  return w;
}

// Load the 128-byte block at p (rem bytes of the message remain from p; bytes >= rem are 0).
// Requires the CSR contract: 4 readable bytes past the message end.
__device__ __forceinline__ void load_block_csr(const uint8_t* p, uint64_t rem, uint64_t m[16]) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
  const uint32_t* base = reinterpret_cast<const uint32_t*>(addr & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(addr & 3) * 8;
  const uint32_t keep = rem >= 128 ? 128u : (uint32_t)rem;
  // aligned dwords covering [p, p+keep): at most 33
  uint32_t w[33];
  const uint32_t ndw = (uint32_t)(((addr & 3) + keep + 3) >> 2);
#pragma unroll
  for (int k = 0; k < 33; ++k) w[k] = (uint32_t)k < ndw ? base[k] : 0u;
  uint32_t d[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    uint32_t x = sh ? __builtin_amdgcn_alignbit(w[k + 1], w[k], sh) : w[k];
    const uint32_t lo = 4u * k;
    uint32_t valid = keep <= lo ? 0u : (keep >= lo + 4 ? 4u : keep - lo);
    d[k] = x & (valid >= 4 ? 0xffffffffu : ((1u << (8 * valid)) - 1u));
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = pack(d[2 * k], d[2 * k + 1]);
}

// Message i is msgs[begs[i], ends[i]): CSR passes (offsets, offsets + 1); the span form
// (launch_b2b_spans) hashes messages that overlap or leave gaps, e.g. attestation records
// inside their blocks' bytes.
extern "C" __global__ void __launch_bounds__(256)
pz_b2b_csr_kernel(const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ begs,
                  const uint64_t* __restrict__ ends, uint64_t n, uint8_t* __restrict__ out, uint32_t out_bytes) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t beg = begs[i], end = ends[i];
  const uint64_t len = end - beg;
  const uint64_t nblocks = len == 0 ? 1 : (len + 127) / 128;
  uint64_t h[8];
  init_h(h);
  for (uint64_t t = 0; t < nblocks; ++t) {
    uint64_t m[16];
    const uint64_t rem = len - t * 128;
    if (len == 0) {
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] = 0;
    } else {
      load_block_csr(msgs + beg + t * 128, rem, m);
    }
    const bool last = (t + 1 == nblocks);
    compress(h, m, last ? len : (t + 1) * 128, last);
  }
  store_digest(out + i * out_bytes, h, out_bytes);
}

// ------------------------------------------------------------------------------------------
// processAttestation messages (blockchain/core.go:277-290), assembled on the fly from device
// data instead of being materialised on the host: message i is
//   hdr[0..10) | for r < 64: hlog[id(i, r)] (32 B) ' ' | ShardBlockHash
// (10 + 64 x 33 + len(ShardBlockHash) bytes; the 64 signed parent hashes are ids into the
// engine's hash log, which holds the block digests the GPU already computed: the first nw
// from the engine's recent-hash trail, the rest the attestation's own oblique ids).  One lane per
// message; each 128-byte block is assembled into the lane's LDS row (33-dword stride, no
// bank conflicts) from the few parent records it overlaps, their ids and 32-byte hashes all
// loaded first (a byte-at-a-time gather, one dependent load per byte, made the kernel 0.41 ms
// per 50,000 messages), then read back as the 16 message words.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kAttMsgParents = 64, kAttMsgRec = 33, kAttMsgHdr = 10;

// Byte k of a 32-byte hash held as two uint4.
__device__ __forceinline__ uint32_t hash_word(const uint4& a, const uint4& b, int k) {
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return w[k];
}
// The bytes of word w at row byte positions pos..pos+3 that fall inside the 128-byte block.
__device__ __forceinline__ void put_word(uint8_t* rb, int pos, uint32_t w) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if ((unsigned)(pos + e) < 128u) rb[pos + e] = (uint8_t)(w >> (8 * e));
}

extern "C" __global__ void __launch_bounds__(256)
pz_b2b_attmsg_kernel(const uint8_t* __restrict__ hlog, const uint32_t* __restrict__ trail,
                     const AttMsg* __restrict__ rec, const uint8_t* __restrict__ var, uint64_t n,
                     uint8_t* __restrict__ out) {
  __shared__ uint32_t rows[256 * 33];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;  // no block-wide barrier below: lanes only touch their own row
  uint32_t* row = rows + threadIdx.x * 33;
  uint8_t* rb = reinterpret_cast<uint8_t*>(row);
  const AttMsg* am = rec + i;
  const uint32_t* hw = reinterpret_cast<const uint32_t*>(am);  // the header: bytes 0..9
  const uint32_t nw = am->nw;
  const uint32_t* win = trail + am->wstart;
  const uint8_t* v = var + am->vo;
  const uint32_t* obl = reinterpret_cast<const uint32_t*>(v);
  const uint32_t* sbw = obl + (kAttMsgParents - nw);  // ShardBlockHash (4-byte aligned)
  const uint32_t sl = am->sl;
  constexpr int kSbh = kAttMsgHdr + kAttMsgParents * kAttMsgRec;  // where the ShardBlockHash starts
  const uint64_t len = kSbh + sl;
  const uint64_t nblocks = (len + 127) / 128;
  uint64_t h[8];
  init_h(h);
  for (uint64_t t = 0; t < nblocks; ++t) {
    const int base = (int)(t * 128);
#pragma unroll
    for (int k = 0; k < 32; ++k) row[k] = 0;
    if (t == 0) {
      put_word(rb, 0, hw[0]);
      put_word(rb, 4, hw[1]);
      put_word(rb, 8, hw[2] & 0xFFFFu);
    }
    // the (at most 5) 33-byte parent records overlapping [base, base + 128): every id, then
    // every hash, loaded before any byte is placed (two round trips per block, not one per byte)
    const int ra = base < (int)kAttMsgHdr + 33 ? 0 : (base - (int)kAttMsgHdr - 33) / 33 + 1;
    const int rz = min((int)kAttMsgParents - 1, (base + 128 - (int)kAttMsgHdr - 1) / 33);
    uint32_t id[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int r = ra + q;
      id[q] = r <= rz ? ((uint32_t)r < nw ? win[r] : obl[r - nw]) : 0u;
    }
    uint4 ha[5], hb[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      if (ra + q <= rz) {
        const uint4* hp = reinterpret_cast<const uint4*>(hlog + (uint64_t)id[q] * 32);
        ha[q] = hp[0];
        hb[q] = hp[1];
      } else {
        ha[q] = hb[q] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int r = ra + q;
      if (r > rz) continue;
      const int p0 = (int)kAttMsgHdr + 33 * r - base;
#pragma unroll
      for (int k = 0; k < 8; ++k) put_word(rb, p0 + 4 * k, hash_word(ha[q], hb[q], k));
      if ((unsigned)(p0 + 32) < 128u) rb[p0 + 32] = 0x20;
    }
    if (base + 128 > kSbh && (uint64_t)base < len) {
      const int qa = base > kSbh ? (base - kSbh) / 4 : 0;
      const int qz = min((int)((sl + 3) / 4), (base + 128 - kSbh + 3) / 4);
      for (int q = qa; q < qz; ++q) {
        uint32_t w = sbw[q];
        const uint32_t left = sl - 4 * q;  // bytes of the ShardBlockHash from word q on
        if (left < 4) w &= (1u << (8 * left)) - 1u;
        put_word(rb, kSbh + 4 * q - base, w);
      }
    }
    uint64_t mw[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) mw[k] = pack(row[2 * k], row[2 * k + 1]);
    const bool last = (t + 1 == nblocks);
    compress(h, mw, last ? len : (t + 1) * 128, last);
  }
  store_digest(out + i * 64, h, 64);
}

// ---- host-side launchers (declared in blake2b_kernels.h) ---------------------------------
#ifdef PZ_AB_BUILD
static int g_fixed_variant = 1;  // (A/B library) 1: persistent LDS-DMA kernel (+ plain tail), 0: plain grid
#else
constexpr int g_fixed_variant = 1;
#endif

static int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cached[dev] = cus;
  }
  return cached[dev];
}

static hipError_t launch_plain(const uint8_t* msgs, uint64_t stride, uint64_t len, uint64_t n, uint8_t* out,
                               uint32_t out_bytes, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint64_t waves = (n + 63) / 64;
  const uint64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(pz_b2b_fixed_kernel, dim3((uint32_t)blocks), dim3(64 * kWavesPerBlock), 0,
                     stream, msgs, stride, len, n, out, out_bytes);
  return hipGetLastError();
}

hipError_t launch_b2b_fixed(const uint8_t* msgs, uint64_t stride, uint64_t len, uint64_t n,
                            uint8_t* out, uint32_t out_bytes, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint64_t nblocks = len == 0 ? 1 : (len + 127) / 128;
  const uint64_t nfull = n & ~63ull;
  if (g_fixed_variant != 1 || stride < nblocks * 128 || nfull == 0)
    return launch_plain(msgs, stride, len, n, out, out_bytes, stream);
  // persistent grid: 4 resident 256-thread workgroups per CU (122 VGPRs -> 4 waves/SIMD)
  const uint64_t groups = nfull / 64;
  uint64_t blocks = (uint64_t)cu_count() * 4;
  const uint64_t need = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > need) blocks = need;
  hipLaunchKernelGGL(pz_b2b_fixed_persistent_kernel, dim3((uint32_t)blocks), dim3(64 * kWavesPerBlock), 0,
                     stream, msgs, stride, len, nfull, out, out_bytes);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nfull == n) return e;
  return launch_plain(msgs + nfull * stride, stride, len, n - nfull, out + nfull * out_bytes, out_bytes, stream);
}

#ifdef PZ_AB_BUILD
int set_fixed_variant(int v) {
  const int old = g_fixed_variant;
  g_fixed_variant = v;
  return old;
}
#endif

hipError_t launch_b2b_csr(const uint8_t* msgs, const uint64_t* offsets, uint64_t n, uint8_t* out,
                          uint32_t out_bytes, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(pz_b2b_csr_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, msgs,
                     offsets, offsets + 1, n, out, out_bytes);
  return hipGetLastError();
}

hipError_t launch_b2b_spans(const uint8_t* msgs, const uint64_t* begs, const uint64_t* ends, uint64_t n, uint8_t* out,
                            uint32_t out_bytes, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(pz_b2b_csr_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, msgs, begs, ends, n,
                     out, out_bytes);
  return hipGetLastError();
}

hipError_t launch_b2b_attmsg(const uint8_t* hlog, const uint32_t* trail, const AttMsg* rec, const uint8_t* var, uint64_t n,
                             uint8_t* out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(pz_b2b_attmsg_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, hlog, trail, rec,
                     var, n, out);
  return hipGetLastError();
}

}  // namespace pz
