// proto3 encoding of AttestationRecord columns on the device.
//
// Replaces golang/protobuf `proto.Marshal(AttestationRecord)` at types/attestation.go:51
// (Marshal) and :56 (Hash), and the records inside BeaconBlock (field 8, block.go:69) and
// ActiveState (field 1, state.go:141).  The record is messages.pb.go:889-896: slot 1,
// shard_id 2, justified_slot 3 (varints, omitted when 0), justified_block_hash 4,
// shard_block_hash 5, attester_bitfield 6 (bytes, omitted when empty), oblique_parent_hashes 7
// (repeated bytes: every element emitted, an empty one as `3a 00`), aggregate_sig 8 (packed
// varints, omitted when empty).
//
// Two launches (after a memset of the tile status words and ticket):
//   size   512 threads x 8 records per tile: every record's encoded size (one lane per record:
//          head loads coalesced, a record's element / value loads independent), the tile's
//          scan, its base by a decoupled look-back over the tiles before it, offsets out;
//   write  one 16-lane DPP row per record, four per wave: the record is assembled in an LDS
//          stage at (offset mod 16) -- literals by the row's lanes, segments copied with aligned
//          dword loads and written into the stage as whole dwords -- and stored in 16-B blocks.
// Round 4 ran size, a rocPRIM inclusive scan (two launches) and the write kernel; the write
// kernel placed segment bytes into the stage one ds_write_b8 at a time.  A one-launch form with
// a look-back per wave ran 0.85 ms per 1M records against 0.41 (profiles/r05/
// wire_att_probe_r5d.txt): ~6,000 waves are in flight, so a wave's look-back walks back over
// many windows before it meets a published prefix; dropped.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <vector>
#ifdef PZ_AB_BUILD
#include <rocprim/device/device_scan.hpp>
#endif

#include "runtime.h"

namespace pz {
namespace {

constexpr int kThreads = 256, kWaves = kThreads / 64;

struct AttArgs {
  const uint64_t* col[3];  // slot, shard_id, justified_slot
  const uint8_t* bdat[3];  // justified_block_hash, shard_block_hash, attester_bitfield
  const uint64_t* boff[3];
  const uint8_t* odat;  // oblique parent hashes: element CSR
  const uint64_t* ooff;
  const uint64_t* ofirst;  // record i owns elements ofirst[i] .. ofirst[i+1]
  const uint64_t* sig;
  const uint64_t* sfirst;  // record i owns values sfirst[i] .. sfirst[i+1]
  uint64_t n;
  uint32_t field, tag_len;
  uint64_t* sizes;
  uint64_t* offs;  // n+1
  uint8_t* out;
  uint64_t* status;  // [tiles] look-back status words, zero at launch
  uint32_t* ticket;  // tile ticket (after the status words), zero at launch
};

__device__ __forceinline__ uint32_t vlen(uint64_t x) { return (uint32_t)((70 - __clzll(x | 1)) / 7); }
// 32-bit values: one v_ffbh instead of two; (38 - clz) / 7 as a multiply by 37 and a shift
// (exact for 38 - clz in [7, 38])
__device__ __forceinline__ uint32_t vlen32(uint32_t x) { return ((38u - (uint32_t)__clz(x | 1)) * 37u) >> 8; }

__device__ __forceinline__ uint8_t* put_varint(uint8_t* p, uint64_t x) {
  while (x >= 0x80) {
    *p++ = (uint8_t)(x | 0x80);
    x >>= 7;
  }
  *p++ = (uint8_t)x;
  return p;
}

// put_varint into the LDS stage with at most four stores (8-, 4-, 2- and 1-byte pieces,
// unaligned): x's 7-bit groups spread into three dwords by bit-field extracts, the
// continuation bits from n = vlen(x).  ~35 VALU instructions for a 10-byte value against ~60
// for the byte loop; values under 128 keep the single byte store.
__device__ __forceinline__ void put_varint_pieces(uint8_t* p, uint64_t x) {
  if (x < 0x80) {
    *p = (uint8_t)x;
    return;
  }
  const uint32_t n = vlen(x), lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t m = __builtin_amdgcn_alignbit(hi, lo, 28);  // bits 28..59
  uint32_t w0 = (lo & 0x7f) | (__builtin_amdgcn_ubfe(lo, 7, 7) << 8) | (__builtin_amdgcn_ubfe(lo, 14, 7) << 16) |
                (__builtin_amdgcn_ubfe(lo, 21, 7) << 24);
  uint32_t w1 = (m & 0x7f) | (__builtin_amdgcn_ubfe(m, 7, 7) << 8) | (__builtin_amdgcn_ubfe(m, 14, 7) << 16) |
                (__builtin_amdgcn_ubfe(m, 21, 7) << 24);
  uint32_t w2 = __builtin_amdgcn_ubfe(hi, 24, 7) | ((hi >> 31) << 8);
  const uint32_t k = n - 1;  // bytes 0 .. k-1 carry the continuation bit (k in 1..9)
  const uint64_t c = k >= 8 ? ~0ull : (1ull << (8 * k)) - 1;
  w0 |= 0x80808080u & (uint32_t)c;
  w1 |= 0x80808080u & (uint32_t)(c >> 32);
  w2 |= k >= 9 ? 0x80u : 0u;
  if (n >= 8) {
    const uint2 v = make_uint2(w0, w1);
    __builtin_memcpy(p, &v, 8);
    if (n == 10) {
      const uint16_t h = (uint16_t)w2;
      __builtin_memcpy(p + 8, &h, 2);
    } else if (n == 9) {
      p[8] = (uint8_t)w2;
    }
  } else {
    uint32_t t = w0, o = 0;
    if (n & 4) {
      __builtin_memcpy(p, &w0, 4);
      t = w1;
      o = 4;
    }
    if (n & 2) {
      const uint16_t h = (uint16_t)t;
      __builtin_memcpy(p + o, &h, 2);
      t >>= 16;
      o += 2;
    }
    if (n & 1) p[o] = (uint8_t)t;
  }
}

__device__ __forceinline__ uint64_t wsum(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// Inclusive scan over the wave.
__device__ __forceinline__ uint64_t wscan(uint64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

struct Head {  // the record's scalar part, the same on every lane
  uint64_t v[3], bl[3], b0[3];
  uint64_t o0, o1, s0, s1;
};

[[maybe_unused]] __device__ __forceinline__ void load_head(const AttArgs& a, uint64_t i, Head& h) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    h.v[k] = a.col[k] ? a.col[k][i] : 0;
    h.b0[k] = a.boff[k] ? a.boff[k][i] : 0;
    h.bl[k] = a.boff[k] ? a.boff[k][i + 1] - h.b0[k] : 0;
  }
  h.o0 = a.ofirst ? a.ofirst[i] : 0;
  h.o1 = a.ofirst ? a.ofirst[i + 1] : 0;
  h.s0 = a.sfirst ? a.sfirst[i] : 0;
  h.s1 = a.sfirst ? a.sfirst[i + 1] : 0;
}

// load_head with every load issued: a NULL column reads a zero pair instead of branching
// round its load (the branches' joins waited for each load in turn: four round trips per head).
__device__ const uint64_t kZeroPair[2] = {0, 0};

__device__ __forceinline__ void load_head_flat(const AttArgs& a, uint64_t i, Head& h) {
  typedef const __attribute__((address_space(1))) uint64_t gu64;
  gu64* z = reinterpret_cast<gu64*>((uintptr_t)kZeroPair);
  auto col = [&](const uint64_t* p) { return p ? reinterpret_cast<gu64*>((uintptr_t)(p + i)) : z; };
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    h.v[k] = *col(a.col[k]);
    gu64* b = col(a.boff[k]);
    h.b0[k] = b[0];
    h.bl[k] = b[1] - b[0];
  }
  gu64* o = col(a.ofirst);
  gu64* g = col(a.sfirst);
  h.o0 = o[0];
  h.o1 = o[1];
  h.s0 = g[0];
  h.s1 = g[1];
}

// Fields 1-6 (scalars and bytes), the oblique elements and the packed signature body.
__device__ __forceinline__ void record_parts(const AttArgs& a, const Head& h, uint64_t* fixed, uint64_t* obl,
                                             uint64_t* sigb) {
  uint64_t f = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    f += h.v[k] ? 1 + vlen(h.v[k]) : 0;
    f += h.bl[k] ? 1 + vlen(h.bl[k]) + h.bl[k] : 0;
  }
  const int lane = threadIdx.x & 63;
  uint64_t o = 0, s = 0;
  for (uint64_t e = h.o0 + lane; e < h.o1; e += 64) {
    const uint64_t l = a.ooff[e + 1] - a.ooff[e];
    o += 1 + vlen(l) + l;
  }
  for (uint64_t e = h.s0 + lane; e < h.s1; e += 64) s += vlen(a.sig[e]);
  *fixed = f;
  *obl = wsum(o);
  *sigb = wsum(s);
}

__device__ __forceinline__ uint64_t body_size(uint64_t fixed, uint64_t obl, uint64_t sigb) {
  return fixed + obl + (sigb ? 1 + vlen(sigb) + sigb : 0);
}

// Lane-parallel byte copy.
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, uint64_t len) {
  for (uint64_t j = threadIdx.x & 63; j < len; j += 64) dst[j] = src[j];
}

// Write record `h` at p (HBM or the wave's LDS stage).  Lane 0 writes the headers; the lanes
// copy each bytes field / oblique element together and write one signature varint each.
__device__ __forceinline__ void write_record(const AttArgs& a, const Head& h, uint64_t body, uint64_t sigb,
                                             uint8_t* p) {
  const int lane = threadIdx.x & 63;
  if (a.field) {  // the frame, then fields in ascending order
    if (lane == 0) {
      uint8_t* q = put_varint(p, ((uint64_t)a.field << 3) | 2);
      put_varint(q, body);
    }
    p += a.tag_len + vlen(body);
  }
  for (int k = 0; k < 3; ++k)  // fields 1-3
    if (h.v[k]) {
      if (lane == 0) {
        p[0] = (uint8_t)((k + 1) << 3);
        put_varint(p + 1, h.v[k]);
      }
      p += 1 + vlen(h.v[k]);
    }
  for (int k = 0; k < 3; ++k)  // fields 4-6
    if (h.bl[k]) {
      const uint32_t hl = 1 + vlen(h.bl[k]);
      if (lane == 0) {
        p[0] = (uint8_t)(((k + 4) << 3) | 2);
        put_varint(p + 1, h.bl[k]);
      }
      copy_bytes(p + hl, a.bdat[k] + h.b0[k], h.bl[k]);
      p += hl + h.bl[k];
    }
  for (uint64_t e = h.o0; e < h.o1; ++e) {  // field 7, element by element
    const uint64_t b0 = a.ooff[e], l = a.ooff[e + 1] - b0;
    const uint32_t hl = 1 + vlen(l);
    if (lane == 0) {
      p[0] = (7 << 3) | 2;
      put_varint(p + 1, l);
    }
    copy_bytes(p + hl, a.odat + b0, l);
    p += hl + l;
  }
  if (sigb) {  // field 8: packed varints, one value per lane
    if (lane == 0) {
      p[0] = (8 << 3) | 2;
      put_varint(p + 1, sigb);
    }
    p += 1 + vlen(sigb);
    for (uint64_t e0 = h.s0; e0 < h.s1; e0 += 64) {
      const uint64_t e = e0 + lane;
      const uint64_t x = e < h.s1 ? a.sig[e] : 0;
      const uint64_t sz = e < h.s1 ? vlen(x) : 0;
      const uint64_t inc = wscan(sz);
      if (e < h.s1) put_varint(p + inc - sz, x);
      p += __shfl(inc, 63, 64);
    }
  }
}

// Each DPP row (16 lanes) owns a record, four per wave.  A record of at most kStage bytes
// whose segments (bytes fields 4-6 and oblique elements, at most 13 elements) are each at
// most kSegMax bytes, with at most 16 signature values, is assembled in the row's LDS stage
// and stored from there:
//  1. layout: sub-lane 0 writes the literal bytes (tags, lengths, scalar varints), sub-lane e
//     an element's header and sub-lane v a signature varint;
//  2. segments: sub-lane s copies segment s (s < 3: bytes field s, else element s - 3) with
//     dword loads aligned on its source, realigned in registers and written into the stage
//     byte by byte -- every lane's loads are in flight together;
//  3. store: the stage holds record byte j at sh + j with sh = o mod 16, so its 16-byte
//     blocks are the output's: whole blocks go out as dwordx4 stores, the two partial edge
//     blocks (shared with the neighbouring records) byte by byte.
// Other records are written by the whole wave, segment by segment (write_record).
//
// A record takes three dependent memory round trips (head -> element offsets -> segment
// bytes), so the kernel is latency-bound; what raises throughput is records in flight and
// few instructions per record (1M config-2 records: 1.66 ms with a wave per record and a
// per-byte gather, 0.82 ms with a record per half-wave, 0.45 ms with one per row):
//  - four records per wave (rocprofv3: 57% of a wave's cycles were memory waits with one);
//  - the record's head spread over the row (one load instruction, DPP row_newbcast reads);
//  - element / signature sizes scanned with DPP row shifts, not LDS permutes;
//  - loads in the global address space: generic (flat) loads share lgkmcnt with the LDS
//    reads, and a byte gather through a per-byte segment map made each load wait for two
//    dependent LDS reads -- the earlier kernel fetched a record's bytes almost one round
//    trip at a time.
// (A persistent, software-pipelined variant that prefetched the next record's head needed
// 130+ VGPRs -- 3 waves per SIMD -- and was slower.)
constexpr uint32_t kStage = 768, kStageAlloc = kStage + 32, kSegMax = 64, kSegWords = kSegMax / 4 + 1;

// A record per DPP row: 16 lanes, four records per wave.
constexpr int kRow = 16, kRecs = 64 / kRow, kMaxOblique = kRow - 3;

// Sub-lane k of the row loads head word k:
//   0-2   slot, shard_id, justified_slot
//   3-8   bytes fields 4-6: start, end (boff[k][i], boff[k][i+1])
//   9-10  oblique element range     11-12  signature value range     (AB form: 13-14 offs[i], offs[i+1])
constexpr int kHeadWords = 13;

template <bool NTL = false>
__device__ __forceinline__ uint64_t head_word(const AttArgs& a, int k, uint64_t i) {
  const uint64_t* p = nullptr;
  uint32_t d = 0;
  if (k < 3) {
    p = a.col[k];
  } else if (k < 9) {
    p = a.boff[(k - 3) >> 1];
    d = (k - 3) & 1;
  } else if (k < kHeadWords + 2) {
    p = k < 11 ? a.ofirst : k < 13 ? a.sfirst : a.offs;
    d = (k - 9) & 1;
  }
  return p ? (NTL ? __builtin_nontemporal_load(p + i + d) : p[i + d]) : 0;
}

__device__ __forceinline__ uint64_t rl64(uint64_t x, int k) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, k), hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), k);
  return ((uint64_t)hi << 32) | lo;
}

// Lane K of this lane's row (DPP row_newbcast).
template <int K>
__device__ __forceinline__ uint32_t bc32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + K, 0xf, 0xf, true);
}
template <int K>
__device__ __forceinline__ uint64_t bc64(uint64_t x) {
  return ((uint64_t)bc32<K>((uint32_t)(x >> 32)) << 32) | bc32<K>((uint32_t)x);
}

// Lane l - 1 of the row (0 for l = 0; DPP row_shr:1).
__device__ __forceinline__ uint32_t shr1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xf, 0xf, true);
}

// Lane l - 3 of the row (0 for l < 3; DPP row_shr:3).
__device__ __forceinline__ uint32_t shr3(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x113, 0xf, 0xf, true);
}

// Inclusive scan over each row with DPP shifts of 1, 2, 4, 8.
__device__ __forceinline__ uint32_t rscan32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x112, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x118, 0xf, 0xf, true);
  return x;
}

// Segment modes (the write kernel's template argument M): 0 round 4's form, the segment placed
// in the stage byte by byte; 1 the aligned form of early round 5, stage dwords realigned with
// v_alignbyte, the two edge words written byte-wise; 2 (the product) unaligned pieces, below.
// 0 and 1 are kept in the A/B library only.
//
// Aligned form: the source dwords wv (aligned on the source, first byte at r), len bytes, to
// stage bytes [d0, d0 + len).
template <int M>
__device__ __forceinline__ void stage_segment_aligned(uint8_t* row, uint32_t d0, uint32_t (&wv)[kSegWords + 1],
                                                      uint32_t r, uint32_t len) {
  if (M == 0) {
#pragma unroll
    for (int k = 0; k < (int)kSegWords; ++k) {
      const uint32_t d = __builtin_amdgcn_alignbyte(wv[k + 1], wv[k], r);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((uint32_t)(4 * k + b) < len) row[d0 + 4 * k + b] = (uint8_t)(d >> (8 * b));
    }
    return;
  }
  if (!len) return;
  // stage word k of the segment holds source bytes r + 4k - dm .. +3 (dm = d0 mod 4): one
  // v_alignbyte of the loaded words, one word lower when r < dm.  Words [kf, kl) are the
  // segment's alone and go out as dwords; the first and the last word, when shared with a
  // neighbour, are written byte by byte after the loop
  const uint32_t dend = d0 + len, dm = d0 & 3;
  const bool back = r < dm;
  const uint32_t delta = (r - dm) & 3, nwo = (dm + len + 3) >> 2;
  const uint32_t kf = (dm == 0 && len >= 4) ? 0u : 1u, kl = (dend & 3) ? nwo - 1 : nwo;
  const uint32_t nfull = kl > kf ? kl - kf : 0u;  // (a segment inside one word has none)
  uint32_t* sw = reinterpret_cast<uint32_t*>(row) + (d0 >> 2);
  const uint32_t bw = d0 & ~3u;
  uint32_t xf = 0, xl = 0;
#pragma unroll
  for (int k = 0; k < (int)kSegWords; ++k) {
    const uint32_t lo = back ? (k ? wv[k - 1] : 0u) : wv[k], hi = back ? wv[k] : wv[k + 1];
    const uint32_t x = __builtin_amdgcn_alignbyte(hi, lo, delta);
    if (k == 0) xf = x;
    xl = (uint32_t)k + 1 == nwo ? x : xl;
    if ((uint32_t)k - kf < nfull) sw[k] = x;  // (k in [kf, kl); unsigned: k < kf wraps high)
  }
  if (kf) {
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (bw + b >= d0 && bw + b < dend) row[bw + b] = (uint8_t)(xf >> (8 * b));
  }
  if ((dend & 3) && nwo > 1) {
    const uint32_t lw = bw + 4 * (nwo - 1);
#pragma unroll
    for (int b = 0; b < 3; ++b)
      if (lw + b < dend) row[lw + b] = (uint8_t)(xl >> (8 * b));
  }
}

// Unaligned form: a segment of len >= 16 bytes is four 16-byte pieces at min(16c, len - 16):
// every load and every stage write lies inside the segment -- the last piece overlaps the one
// before it with the same bytes -- so the neighbours' bytes are never touched and no select
// picks a word: ~25 VALU instructions per segment against ~130 for the aligned form.  (gfx950
// runs unaligned global and LDS accesses; HSA sets the unaligned mode.)  A segment under 16
// bytes (none in the bench's records) is loaded at stage time as aligned words and written
// byte by byte.
struct SegPieces {  // pieces 0-2; the fourth (a segment over 48 bytes) is loaded at stage time
  uint4 q[3];
};

typedef const __attribute__((address_space(1))) uint8_t gbyte;

__device__ __forceinline__ uint4 ldu16(gbyte* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ void stu16(uint8_t* p, uint4 v) { __builtin_memcpy(p, &v, 16); }

__device__ __forceinline__ void load_segment_unaligned(const uint8_t* src, uint32_t len, SegPieces& sp) {
  gbyte* g = reinterpret_cast<gbyte*>((uintptr_t)src);
  const uint32_t np = len >= 16 ? (len + 15) >> 4 : 0;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    if ((uint32_t)c < np) sp.q[c] = ldu16(g + min(16u * c, len - 16));
}

__device__ __forceinline__ void stage_segment_unaligned(uint8_t* d, const uint8_t* src, uint32_t len,
                                                        const SegPieces& sp) {
  const uint32_t np = len >= 16 ? (len + 15) >> 4 : 0;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    if ((uint32_t)c < np) stu16(d + min(16u * c, len - 16), sp.q[c]);
  if (np == 4) stu16(d + len - 16, ldu16(reinterpret_cast<gbyte*>((uintptr_t)src) + len - 16));
  if (len && len < 16) {
    typedef const __attribute__((address_space(1))) uint32_t gword;
    gword* ws = reinterpret_cast<gword*>((uintptr_t)src & ~(uintptr_t)3);
    const uint32_t r = (uint32_t)(uintptr_t)src & 3, nw = (r + len + 3) >> 2;
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) w[k] = (uint32_t)k < nw ? ws[k] : 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = __builtin_amdgcn_alignbyte(w[k + 1], w[k], r);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((uint32_t)(4 * k + b) < len) d[4 * k + b] = (uint8_t)(x >> (8 * b));
    }
  }
}

// NTF (A/B): bit 0 the whole 16-B output blocks stored nontemporally, bit 1 the head words
// loaded nontemporally
template <int M, int NTF = 0>
__device__ __forceinline__ void wire_att_write_rows(const AttArgs& a, uint8_t (*stage)[kStageAlloc], uint64_t i0) {
  const int lane = threadIdx.x & 63;
  const int sl = lane & (kRow - 1), ri = lane / kRow;
  if (i0 >= a.n) return;
  const uint64_t i = i0 + ri;
  const bool valid = i < a.n;
  const uint64_t hv = valid && sl < kHeadWords + 2 ? head_word<(NTF & 2) != 0>(a, sl, i) : 0;
  // Each lane's word below it (row_shr:1) and the difference: lanes 4, 6, 8 hold bl[0..2],
  // lane 10 the oblique count, 12 the value count, 14 the size.  Only what every lane needs is
  // broadcast; a lane's own operands come by one shift or one ds_bpermute.  Counts and lengths
  // travel as 32 bits: the fast path needs size <= kStage, which bounds them all, and a high
  // word that is not zero (malformed ranges) sends the record to the whole-wave path.
  const uint64_t hb = ((uint64_t)shr1((uint32_t)(hv >> 32)) << 32) | shr1((uint32_t)hv);
  const uint64_t hd = hv - hb;
  const uint64_t o0 = bc64<9>(hv), s0 = bc64<11>(hv), o = bc64<13>(hv), size = bc64<14>(hd);
  const uint32_t nob = bc32<10>((uint32_t)hd), nsig = bc32<12>((uint32_t)hd);
  const uint64_t wide = __ballot(sl >= 4 && sl <= 12 && !(sl & 1) && (hd >> 32) != 0);  // (lanes 4-12, even)
  bool fast = valid && size <= kStage && nob <= (uint32_t)kMaxOblique && nsig <= (uint32_t)kRow &&
              !((wide >> (kRow * ri)) & 0xffffull);
  // lanes 0-2: bytes field sl's start (word 3 + 2 sl) and length (difference 4 + 2 sl); lanes
  // 4-6: field sl - 3's length for its header (difference 2 sl - 4)
  const int rb = lane & ~(kRow - 1);
  const int bsrc = rb + (sl < 3 ? 3 + 2 * sl : 0), lsrc = rb + (sl < 3 ? 4 + 2 * sl : sl >= 4 && sl <= 6 ? 2 * sl - 4 : 0);
  const uint64_t b0s = ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(4 * bsrc, (int)(uint32_t)(hv >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_ds_bpermute(4 * bsrc, (int)(uint32_t)hv);
  const uint32_t bls = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * lsrc, (int)(uint32_t)hd);
  uint64_t eb0 = 0, sv = 0;
  uint32_t el = 0;
  if (fast && (uint32_t)sl < nob) {
    eb0 = a.ooff[o0 + sl];
    el = (uint32_t)(a.ooff[o0 + sl + 1] - eb0);
  }
  if (fast && (uint32_t)sl < nsig) sv = a.sig[s0 + sl];
  const uint32_t el_seg = shr3(el);
  const uint64_t eb_seg = ((uint64_t)shr3((uint32_t)(eb0 >> 32)) << 32) | shr3((uint32_t)eb0);
  uint64_t seg_len = 0;
  const uint8_t* seg_src = nullptr;
  if (sl < 3) {
    seg_len = bls;
    seg_src = (sl == 0 ? a.bdat[0] : sl == 1 ? a.bdat[1] : a.bdat[2]) + b0s;
  }
  if (sl >= 3 && (uint32_t)(sl - 3) < nob) {
    seg_len = el_seg;
    seg_src = a.odat + eb_seg;
  }
  const uint64_t long_seg = __ballot(fast && seg_len > kSegMax);
  if ((long_seg >> (kRow * ri)) & 0xffffull) fast = false;
  const uint32_t esz = fast && (uint32_t)sl < nob ? 1 + vlen32(el) + el : 0;
  const uint32_t ssz = fast && (uint32_t)sl < nsig ? vlen(sv) : 0;
  const uint32_t einc = rscan32(esz), sinc = rscan32(ssz);
  const uint32_t obl = bc32<15>(einc), sigb = bc32<15>(sinc);
  typedef const __attribute__((address_space(1))) uint32_t gword;
  const uint32_t len = fast ? (uint32_t)seg_len : 0;
  const uint32_t r = (uint32_t)(uintptr_t)seg_src & 3;
  uint32_t wv[kSegWords + 1];
  SegPieces sp;
  if (M < 2) {
    gword* ws = reinterpret_cast<gword*>((uintptr_t)seg_src & ~(uintptr_t)3);
    const uint32_t nw = len ? (r + len + 3) / 4 : 0;
#pragma unroll
    for (int k = 0; k <= (int)kSegWords; ++k) wv[k] = (uint32_t)k < nw ? ws[k] : 0;
  } else {
    load_segment_unaligned(seg_src, len, sp);
  }
  const uint32_t sh = (uint32_t)o & 15;
  uint8_t* st = stage[ri] + sh;
  uint32_t seg_dst = 0;
  if (fast) {
    uint64_t val = 0;
    uint32_t span = 0;
    if (sl >= 1 && sl <= 3) {
      val = hb;  // (fields 1-3: the word of lane sl - 1)
      span = val ? 1 + vlen(val) : 0;
    } else if (sl >= 4 && sl <= 6) {
      val = bls;
      span = val ? 1 + vlen32(bls) + bls : 0;
    } else if (sl == 7) {
      span = obl;
    } else if (sl == 8) {
      val = sigb;
      span = sigb ? 1 + vlen32(sigb) + sigb : 0;
    }
    const uint32_t inc = rscan32(span);
    const uint32_t body = bc32<8>(inc);
    const uint32_t frame = a.field ? a.tag_len + vlen32(body) : 0;
    const uint32_t pos = frame + inc - span;
    if (sl == 0 && a.field) {
      uint8_t* q = put_varint(st, ((uint64_t)a.field << 3) | 2);
      put_varint(q, body);
    }
    if (sl >= 1 && sl <= 8 && sl != 7 && val) {
      st[pos] = (uint8_t)((sl << 3) | (sl >= 4 ? 2 : 0));
      put_varint(st + pos + 1, val);
    }
    const uint32_t fd = (uint32_t)__builtin_amdgcn_mov_dpp((int)(pos + 1 + vlen(val)), 0x104, 0xf, 0xf, true);
    if (sl < 3) seg_dst = fd;
    const uint32_t ep = bc32<7>(pos) + einc - esz;
    if ((uint32_t)sl < nob) {
      st[ep] = (7 << 3) | 2;
      put_varint(st + ep + 1, el);
    }
    const uint32_t ed = shr3(ep + 1 + vlen32(el));
    if (sl >= 3 && (uint32_t)(sl - 3) < nob) seg_dst = ed;
    const uint32_t sp = bc32<8>(pos) + 1 + vlen32(sigb);
    if ((uint32_t)sl < nsig) {
      if (M == 2) {
        put_varint_pieces(st + sp + sinc - ssz, sv);
      } else {
        put_varint(st + sp + sinc - ssz, sv);
      }
    }
  }
  if (M < 2) {
    stage_segment_aligned<M>(stage[ri], sh + seg_dst, wv, r, len);
  } else {
    stage_segment_unaligned(stage[ri] + sh + seg_dst, seg_src, len, sp);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const uint32_t sz = fast ? (uint32_t)size : 0;
  const uint32_t nblk = (sh + sz + 15) / 16;
  const uint8_t* sb = stage[ri];
  uint8_t* ob = a.out + (o - sh);
  for (uint32_t q = sl; q < nblk; q += kRow) {
    const uint32_t lo = 16 * q, hi = lo + 16;
    if (lo >= sh && hi <= sh + sz) {
      if (NTF & 1) {
        typedef unsigned int v4u_ __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(*reinterpret_cast<const v4u_*>(sb + lo), reinterpret_cast<v4u_*>(ob + lo));
      } else {
        *reinterpret_cast<uint4*>(ob + lo) = *reinterpret_cast<const uint4*>(sb + lo);
      }
    } else if (M < 2) {
      for (uint32_t x = max(lo, sh); x < min(hi, sh + sz); ++x) ob[x] = sb[x];
    } else {  // an edge block shared with a neighbour: 1-, 2-, 4- and 8-byte pieces of [x, e)
      uint32_t x = max(lo, sh);
      const uint32_t l = min(hi, sh + sz) - x;
      if (l & 1) ob[x] = sb[x];
      x += l & 1;
      if (l & 2) {
        uint16_t v;
        __builtin_memcpy(&v, sb + x, 2);
        __builtin_memcpy(ob + x, &v, 2);
      }
      x += l & 2;
      if (l & 4) {
        uint32_t v;
        __builtin_memcpy(&v, sb + x, 4);
        __builtin_memcpy(ob + x, &v, 4);
      }
      x += l & 4;
      if (l & 8) {
        uint2 v;
        __builtin_memcpy(&v, sb + x, 8);
        __builtin_memcpy(ob + x, &v, 8);
      }
    }
  }
  for (int u = 0; u < kRecs; ++u) {
    const uint64_t iu = i0 + u;
    if (iu >= a.n) break;
    if (__builtin_amdgcn_readlane((uint32_t)fast, kRow * u)) continue;
    Head q;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      q.v[k] = rl64(hv, kRow * u + k);
      q.b0[k] = rl64(hv, kRow * u + 3 + 2 * k);
      q.bl[k] = rl64(hv, kRow * u + 4 + 2 * k) - q.b0[k];
    }
    q.o0 = rl64(hv, kRow * u + 9);
    q.o1 = rl64(hv, kRow * u + 10);
    q.s0 = rl64(hv, kRow * u + 11);
    q.s1 = rl64(hv, kRow * u + 12);
    uint64_t fixed, obl8, sigb8;
    record_parts(a, q, &fixed, &obl8, &sigb8);
    write_record(a, q, body_size(fixed, obl8, sigb8), sigb8, a.out + rl64(hv, kRow * u + 13));
  }
}

// ---- the encode: sizes + scan in one launch, then the writes ----------------------------------
constexpr uint64_t kFlagA = 1ull << 62, kFlagP = 2ull << 62, kVal = kFlagA - 1;

__device__ __forceinline__ uint64_t ld_status(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_status_fresh(uint64_t* p) {  // at the coherence point
  return __hip_atomic_fetch_add(p, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sizing tile: 512 threads x 8 records (thread t takes records t + 512q of the tile: every head
// load coalesced; 2 waves per SIMD leave 256 VGPRs for 8 records' loads in flight), 256 tiles
// per 1M records.  Tiles are numbered by a
// ticket taken at start, so every predecessor of a waiting tile is running or done (the
// dispatch order of workgroups is not guaranteed); a tile's look-back reads 1,024
// predecessors' status words a round.
constexpr int kSizeThreads = 512, kSizePer = 8;  // (the product's geometry; the A/B library's others below)
constexpr uint32_t kSizeTile = kSizeThreads * kSizePer;

__device__ __forceinline__ uint64_t record_size(const AttArgs& a, uint64_t i) {
  Head h;
  load_head(a, i, h);
  uint64_t body = 0, sigb = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    body += h.v[k] ? 1 + vlen(h.v[k]) : 0;
    body += h.bl[k] ? 1 + vlen(h.bl[k]) + h.bl[k] : 0;
  }
#pragma unroll 4
  for (uint64_t e = h.o0; e < h.o1; ++e) {
    const uint64_t l = a.ooff[e + 1] - a.ooff[e];
    body += 1 + vlen(l) + l;
  }
#pragma unroll 4
  for (uint64_t e = h.s0; e < h.s1; ++e) sigb += vlen(a.sig[e]);
  body += sigb ? 1 + vlen(sigb) + sigb : 0;
  return a.field ? a.tag_len + vlen(body) + body : body;
}

// A thread's P records sized with their loads in flight together.  Round 5's first sizing ran
// each record's element and value loops in turn (a loop's trip count is data, so nothing of
// record q + 1 was issued before record q's loops ended): ~5 dependent round trips per record,
// 40 per thread.  Here the heads of all P records load first; then, G records at a time, each
// record's first kSizeElems + 1 element offsets and kSizeSigs values load from clamped
// addresses (no predicate, so no branch keeps the next load waiting) and are masked in the sum.
// A record with more elements or values than that is sized again by the loops.
constexpr uint32_t kSizeElems = 12, kSizeSigs = 4;

template <int T, int P, int G>
__device__ __forceinline__ void size_records(const AttArgs& a, uint64_t t0, uint64_t (&sz)[P]) {
  const int tid = threadIdx.x;
  uint64_t fixed[P], o0[P], s0[P];
  uint32_t no[P], ns[P];  // clamped to kSizeElems + 1 / kSizeSigs + 1 (more: the loops)
#pragma unroll
  for (int q4 = 0; q4 < P; q4 += 4) {  // heads four records at a time (13 loads each), all in flight
    __builtin_amdgcn_sched_barrier(0);
    Head h[4];
#pragma unroll
    for (int r = 0; r < 4 && q4 + r < P; ++r) {
      const uint64_t i = t0 + (uint64_t)(q4 + r) * T + tid;
      load_head_flat(a, i < a.n ? i : a.n - 1, h[r]);
    }
#pragma unroll
    for (int r = 0; r < 4 && q4 + r < P; ++r) {
      const int q = q4 + r;
      const uint64_t i = t0 + (uint64_t)q * T + tid;
      uint64_t f = 0;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        f += h[r].v[k] ? 1 + vlen(h[r].v[k]) : 0;
        f += h[r].bl[k] ? 1 + vlen(h[r].bl[k]) + h[r].bl[k] : 0;
      }
      fixed[q] = i < a.n ? f : 0;
      o0[q] = h[r].o0;
      s0[q] = h[r].s0;
      no[q] = (uint32_t)min(h[r].o1 - h[r].o0, (uint64_t)kSizeElems + 1);
      ns[q] = (uint32_t)min(h[r].s1 - h[r].s0, (uint64_t)kSizeSigs + 1);
    }
  }
  const uint64_t* any = reinterpret_cast<const uint64_t*>(a.status);  // (a valid address; the value is masked)
  uint32_t longs = 0;
#pragma unroll
  for (int g = 0; g < P; g += G) {
    __builtin_amdgcn_sched_barrier(0);  // (one group's loads live at a time: hoisting them all spills)
    // element offsets: the first and the last as 64-bit words, the ones between as their low
    // words (a record whose elements total 2^32 bytes or more takes the loops, so every
    // length is exact as a 32-bit difference)
    typedef const __attribute__((address_space(1))) uint32_t gu32;
    uint64_t ofirst[G], olast[G], sv[G][kSizeSigs];
    uint32_t lw[G][kSizeElems - 1];
#pragma unroll
    for (int r = 0; r < G; ++r) {
      const int q = g + r;
      const uint64_t* ob = a.ooff ? a.ooff + o0[q] : any;
      const uint32_t ol = a.ooff ? min(no[q], kSizeElems) : 0;
      gu32* obw = reinterpret_cast<gu32*>((uintptr_t)ob);
      ofirst[r] = ob[0];
      olast[r] = ob[ol];
#pragma unroll
      for (uint32_t e = 1; e < kSizeElems; ++e) lw[r][e - 1] = obw[2 * min(e, ol)];
      const uint64_t* sb = ns[q] ? a.sig + s0[q] : any;
      const uint32_t sl = ns[q] ? min(ns[q], kSizeSigs) - 1 : 0;
#pragma unroll
      for (uint32_t e = 0; e < kSizeSigs; ++e) sv[r][e] = sb[min(e, sl)];
    }
#pragma unroll
    for (int r = 0; r < G; ++r) {
      const int q = g + r;
      const uint64_t i = t0 + (uint64_t)q * T + tid;
      const uint64_t total = olast[r] - ofirst[r];
      uint32_t vl = 0, prev = (uint32_t)ofirst[r];
#pragma unroll
      for (uint32_t e = 0; e < kSizeElems; ++e) {
        const uint32_t next = e + 1 < kSizeElems ? lw[r][e] : (uint32_t)olast[r];
        vl += e < no[q] ? vlen32(next - prev) : 0;
        prev = next;
      }
      uint64_t sigb = 0;
#pragma unroll
      for (uint32_t e = 0; e < kSizeSigs; ++e) sigb += e < ns[q] ? vlen(sv[r][e]) : 0;
      const uint64_t obl = no[q] + vl + total;
      const uint64_t body = fixed[q] + obl + (sigb ? 1 + vlen(sigb) + sigb : 0);
      sz[q] = i >= a.n ? 0 : a.field ? a.tag_len + vlen(body) + body : body;
      longs |= (i < a.n && (no[q] > kSizeElems || ns[q] > kSizeSigs || (total >> 32))) ? 1u << q : 0u;
    }
  }
  // records with more elements or values than the loads above: the loops
  if (__builtin_amdgcn_read_exec() & __ballot(longs != 0)) {
#pragma unroll
    for (int q = 0; q < P; ++q)
      if (longs & (1u << q)) sz[q] = record_size(a, t0 + (uint64_t)q * T + tid);
  }
}

// Block-wide exclusive scan of one value per thread; *total receives the sum.
template <int T>
__device__ __forceinline__ uint64_t block_excl(uint64_t x, uint64_t* s_wave, uint64_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t incl = wscan(x);
  if (lane == 63) s_wave[w] = incl;
  __syncthreads();
  uint64_t before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < T / 64; ++k) {
    before += k < w ? s_wave[k] : 0;
    all += s_wave[k];
  }
  __syncthreads();  // (s_wave is rewritten by the next scan)
  *total = all;
  return before + incl - x;
}

// The tile's exclusive base: thread t watches predecessor tile - 1 - t (T a round); the nearest
// inclusive prefix (P) ends the walk, the aggregates (A) nearer than it are added.
template <int T>
__device__ uint64_t lookback_tiles(uint64_t* status, uint64_t tile, uint32_t* s_first, uint64_t* s_part) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint64_t prefix = 0;
  for (int64_t j = (int64_t)tile - 1;; j -= T) {
    const int64_t idx = j - tid;
    uint64_t v = idx >= 0 ? ld_status(status + idx) : kFlagP;  // before tile 0: prefix 0
    for (uint32_t spins = 0; !(v >> 62); ++spins) {
      __builtin_amdgcn_s_sleep(1);
      v = spins < 256 ? ld_status(status + idx) : ld_status_fresh(status + idx);
    }
    if (tid == 0) *s_first = T;
    __syncthreads();
    if ((v >> 62) == 2) atomicMin(s_first, (uint32_t)tid);
    __syncthreads();
    const uint32_t first = *s_first;
    const uint64_t part = wsum((uint32_t)tid <= first ? (v & kVal) : 0);
    if (lane == 0) s_part[w] = part;
    __syncthreads();
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < T / 64; ++k) sum += s_part[k];
    __syncthreads();  // s_first / s_part are rewritten by the next window
    prefix += sum;
    if (first < (uint32_t)T) return prefix;
  }
}

// Launch 1: every record's size, the tile's scan, its base by look-back, offsets out.
template <int T, int P, bool LOOPS = false>
__device__ __forceinline__ void size_body(const AttArgs& a) {
  __shared__ uint64_t s_wave[T / 64], s_part[T / 64];
  __shared__ uint32_t s_first, s_tile;
  const int tid = threadIdx.x;
  if (tid == 0) s_tile = atomicAdd(a.ticket, 1u);
  __syncthreads();
  const uint64_t tile = s_tile, t0 = tile * (uint64_t)(T * P);
  uint64_t sz[P];
  if (LOOPS) {  // (A/B: round 5's first form, each record's loops in turn)
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const uint64_t i = t0 + (uint64_t)q * T + tid;
      sz[q] = i < a.n ? record_size(a, i) : 0;
    }
  } else {
    size_records<T, P, 2>(a, t0, sz);
  }
  uint64_t ex[P], run = 0;
  if (LOOPS) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      uint64_t tot;
      ex[q] = run + block_excl<T>(sz[q], s_wave, &tot);
      run += tot;
    }
  } else {
    // the P rows' scans together: P independent wave scans (their shuffles interleave), one
    // barrier, then each row's offset from the waves' totals -- where a block scan per row
    // took two barriers each
    __shared__ uint64_t s_rows[P][T / 64];
    const int lane = tid & 63, w = tid >> 6;
    uint64_t incl[P];
#pragma unroll
    for (int q = 0; q < P; ++q) incl[q] = wscan(sz[q]);
    if (lane == 63) {
#pragma unroll
      for (int q = 0; q < P; ++q) s_rows[q][w] = incl[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < P; ++q) {
      uint64_t before = 0, all = 0;
#pragma unroll
      for (int k = 0; k < T / 64; ++k) {
        const uint64_t x = s_rows[q][k];
        before += k < w ? x : 0;
        all += x;
      }
      ex[q] = run + before + incl[q] - sz[q];
      run += all;
    }
  }
  if (tid == 0) st_status(a.status + tile, (tile == 0 ? kFlagP : kFlagA) | run);
  const uint64_t base = tile == 0 ? 0 : lookback_tiles<T>(a.status, tile, &s_first, s_part);
  if (tid == 0 && tile > 0) st_status(a.status + tile, kFlagP | (base + run));
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const uint64_t i = t0 + (uint64_t)q * T + tid;
    if (i < a.n) a.offs[i + 1] = base + ex[q] + sz[q];
  }
  if (tile == 0 && tid == 0) a.offs[0] = 0;
}

extern "C" __global__ void __launch_bounds__(kSizeThreads) pz_wire_att_size_kernel(AttArgs a) {
  size_body<kSizeThreads, kSizePer>(a);
}
#ifdef PZ_AB_BUILD
extern "C" __global__ void __launch_bounds__(512) pz_wire_att_size_512x4_kernel(AttArgs a) { size_body<512, 4>(a); }
extern "C" __global__ void __launch_bounds__(256) pz_wire_att_size_256x8_kernel(AttArgs a) { size_body<256, 8>(a); }
extern "C" __global__ void __launch_bounds__(1024) pz_wire_att_size_1024x2_kernel(AttArgs a) { size_body<1024, 2>(a); }
extern "C" __global__ void __launch_bounds__(kSizeThreads) pz_wire_att_size_loops_kernel(AttArgs a) {
  size_body<kSizeThreads, kSizePer, true>(a);
}
#endif

// Launch 2: four records per wave, one per DPP row.  63 VGPRs; left alone the SGPRs (about
// 100) hold it at 7 waves per SIMD.  Capped at 8 (28 SGPRs spill to VGPR lanes): 0.432 ->
// 0.383 ms per 1M-record encode (tools/wire_att_probe.py r2t, same-process A/B).
#define PZ_ATT_WRITE(NAME, DST, NTF)                                                                 \
  extern "C" __global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(8, 8)))  \
  NAME(AttArgs a) {                                                                                  \
    __shared__ __attribute__((aligned(16))) uint8_t stage[kWaves][kRecs][kStageAlloc];              \
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                                  \
    wire_att_write_rows<DST, NTF>(a, stage[w], ((uint64_t)blockIdx.x * kWaves + w) * kRecs);         \
  }
PZ_ATT_WRITE(pz_wire_att_write_kernel, 2, 0)
#ifdef PZ_AB_BUILD
PZ_ATT_WRITE(pz_wire_att_write_bytes_kernel, 0, 0)
PZ_ATT_WRITE(pz_wire_att_write_aligned_kernel, 1, 0)
PZ_ATT_WRITE(pz_wire_att_write_sigloop_kernel, 3, 0)  // the product with the byte-loop signature varints
PZ_ATT_WRITE(pz_wire_att_write_nts_kernel, 2, 1)  // nontemporal 16-B output stores
PZ_ATT_WRITE(pz_wire_att_write_ntsl_kernel, 2, 3)  // + nontemporal head loads
// 1 round 4's three launches, 2 this scan + byte-wise stage, 3-5 other sizing tiles, 6 the
// aligned-dword stage, 7 the sizing loops, 8 byte-loop signature varints, 9 nontemporal output
// stores, 10 + nontemporal head loads
int g_att_variant = 0;
#endif

uint64_t att_tiles(uint64_t n) { return (n + 2047) / 2048; }  // (scratch: the smallest tile of any geometry)

hipError_t launch_write(const AttArgs& a, bool dst, hipStream_t s) {
  if (!a.n) return hipSuccess;
  const void* k = (const void*)pz_wire_att_write_kernel;
#ifdef PZ_AB_BUILD
  if (!dst) k = (const void*)pz_wire_att_write_bytes_kernel;
  if (g_att_variant == 6) k = (const void*)pz_wire_att_write_aligned_kernel;
  if (g_att_variant == 8) k = (const void*)pz_wire_att_write_sigloop_kernel;
  if (g_att_variant == 9) k = (const void*)pz_wire_att_write_nts_kernel;
  if (g_att_variant == 10) k = (const void*)pz_wire_att_write_ntsl_kernel;
#else
  (void)dst;
#endif
  void* args[] = {const_cast<AttArgs*>(&a)};
  return hipLaunchKernel(k, dim3((uint32_t)((a.n + kRecs * kWaves - 1) / (kRecs * kWaves))), dim3(kThreads), args, 0,
                         s);
}

// sizes + offsets (status words reset first), then the writes
hipError_t launch_two(AttArgs a, void* scratch, bool dst, hipStream_t s) {
  if (!a.n) return hipMemsetAsync(a.offs, 0, 8, s);
  const void* k = (const void*)pz_wire_att_size_kernel;
  uint32_t T = kSizeThreads, tile = kSizeTile;
#ifdef PZ_AB_BUILD
  if (g_att_variant == 3) k = (const void*)pz_wire_att_size_512x4_kernel, T = 512, tile = 2048;
  if (g_att_variant == 4) k = (const void*)pz_wire_att_size_256x8_kernel, T = 256, tile = 2048;
  if (g_att_variant == 5) k = (const void*)pz_wire_att_size_1024x2_kernel, T = 1024, tile = 2048;
  if (g_att_variant == 7) k = (const void*)pz_wire_att_size_loops_kernel;
#endif
  const uint64_t tiles = (a.n + tile - 1) / tile;
  a.status = static_cast<uint64_t*>(scratch);
  a.ticket = reinterpret_cast<uint32_t*>(a.status + tiles);
  hipError_t e = hipMemsetAsync(scratch, 0, tiles * 8 + 8, s);
  if (e != hipSuccess) return e;
  void* args[] = {&a};
  if ((e = hipLaunchKernel(k, dim3((uint32_t)tiles), dim3(T), args, 0, s)) != hipSuccess) return e;
  return launch_write(a, dst, s);
}

#ifdef PZ_AB_BUILD
// ---- round 4's three launches: size kernel, rocPRIM scan, byte-wise write kernel ----------------
extern "C" __global__ void __launch_bounds__(kThreads) pz_wire_att_size_r4_kernel(AttArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= a.n) return;
  Head h;
  load_head(a, i, h);
  uint64_t body = 0, sigb = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    body += h.v[k] ? 1 + vlen(h.v[k]) : 0;
    body += h.bl[k] ? 1 + vlen(h.bl[k]) + h.bl[k] : 0;
  }
#pragma unroll 4
  for (uint64_t e = h.o0; e < h.o1; ++e) {
    const uint64_t l = a.ooff[e + 1] - a.ooff[e];
    body += 1 + vlen(l) + l;
  }
#pragma unroll 4
  for (uint64_t e = h.s0; e < h.s1; ++e) sigb += vlen(a.sig[e]);
  body += sigb ? 1 + vlen(sigb) + sigb : 0;
  a.sizes[i] = a.field ? a.tag_len + vlen(body) + body : body;
}


size_t scan_bytes(uint64_t n) {
  size_t bytes = 0;
  (void)rocprim::inclusive_scan(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)n,
                                rocprim::plus<uint64_t>(), (hipStream_t)0);
  return (bytes + 255) & ~size_t(255);
}

hipError_t launch_three(AttArgs a, void* scratch, hipStream_t s) {
  a.sizes = static_cast<uint64_t*>(scratch);
  hipError_t e = hipMemsetAsync(a.offs, 0, 8, s);
  if (e != hipSuccess || !a.n) return e;
  hipLaunchKernelGGL(pz_wire_att_size_r4_kernel, dim3((uint32_t)((a.n + kThreads - 1) / kThreads)), dim3(kThreads), 0, s,
                     a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  size_t bytes = scan_bytes(a.n);
  e = rocprim::inclusive_scan(static_cast<uint8_t*>(scratch) + ((a.n * 8 + 255) & ~uint64_t(255)), bytes, a.sizes,
                              a.offs + 1, (size_t)a.n, rocprim::plus<uint64_t>(), s);
  if (e != hipSuccess) return e;
  return launch_write(a, false, s);
}

#endif

int att_args(const pz_attestation_cols* c, uint64_t n, uint32_t field_num, AttArgs* a) {
  if (!c) return fail(PZ_EINVAL, "columns are null");
  if (field_num >= (1u << 29)) return fail(PZ_EINVAL, "field number %u out of range", field_num);
  *a = AttArgs{};
  a->col[0] = c->slot;
  a->col[1] = c->shard_id;
  a->col[2] = c->justified_slot;
  a->bdat[0] = c->justified_block_hash;
  a->boff[0] = c->justified_block_hash_offs;
  a->bdat[1] = c->shard_block_hash;
  a->boff[1] = c->shard_block_hash_offs;
  a->bdat[2] = c->attester_bitfield;
  a->boff[2] = c->attester_bitfield_offs;
  a->odat = c->oblique_parent_hashes;
  a->ooff = c->oblique_offs;
  a->ofirst = c->oblique_first;
  a->sig = c->aggregate_sig;
  a->sfirst = c->aggregate_sig_first;
  for (int k = 0; k < 3; ++k)
    if (a->boff[k] && !a->bdat[k]) return fail(PZ_EINVAL, "bytes column without data");
  if (a->ofirst && (!a->ooff || !a->odat)) return fail(PZ_EINVAL, "oblique elements without data");
  if (a->sfirst && !a->sig) return fail(PZ_EINVAL, "signature ranges without values");
  a->n = n;
  a->field = field_num;
  uint64_t tag = ((uint64_t)field_num << 3) | 2;
  a->tag_len = 1;
  while (tag >= 0x80) {
    tag >>= 7;
    ++a->tag_len;
  }
  return PZ_OK;
}

hipError_t launch_encode(const AttArgs& a, void* scratch, hipStream_t s) {
#ifdef PZ_AB_BUILD
  if (g_att_variant == 1) return launch_three(a, scratch, s);
  if (g_att_variant == 2) return launch_two(a, scratch, false, s);
#endif
  return launch_two(a, scratch, true, s);
}

}  // namespace
}  // namespace pz

using namespace pz;

extern "C" {

uint64_t pz_wire_attestations_scratch_bytes(uint64_t n) {
  const uint64_t two = ((att_tiles(n) * 8 + 8 + 255) & ~uint64_t(255));
#ifdef PZ_AB_BUILD
  return std::max<uint64_t>(two, ((n * 8 + 255) & ~uint64_t(255)) + scan_bytes(n));
#else
  return std::max<uint64_t>(two, 256);
#endif
}

uint64_t pz_wire_attestations_bound(uint64_t n, uint64_t bytes_total, uint64_t n_oblique, uint64_t n_sig) {
  // frame 5+10, fields 1-3 3x11, fields 4-6 3x(1+10), field 8 header 11, per element 11, per value 10
  return n * (15 + 33 + 33 + 11) + bytes_total + n_oblique * 11 + n_sig * 10;
}

int pz_dev_wire_attestations(const pz_attestation_cols* c, uint64_t n, uint32_t field_num, uint8_t* d_out,
                             uint64_t* d_offsets, void* d_scratch, void* stream) {
  AttArgs a;
  int rc = att_args(c, n, field_num, &a);
  if (rc) return rc;
  if (!d_offsets || !d_scratch || (n && !d_out)) return fail(PZ_EINVAL, "null device pointer");
  a.out = d_out;
  a.offs = d_offsets;
  const hipError_t e = launch_encode(a, d_scratch, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_wire_att kernels");
}

int pz_wire_attestations(const pz_attestation_cols* c, uint64_t n, uint32_t field_num, uint8_t* out, uint64_t cap,
                         uint64_t* offsets, uint64_t* len) {
  if (!len) return fail(PZ_EINVAL, "len is null");
  *len = 0;
  AttArgs a;
  int rc = att_args(c, n, field_num, &a);
  if (rc) return rc;
  if (n == 0) {
    if (offsets) offsets[0] = 0;
    return PZ_OK;
  }
  for (int k = 0; k < 3; ++k)
    if (a.boff[k] && (rc = check_csr(a.boff[k], n, "bytes column"))) return rc;
  if (a.ofirst && (rc = check_csr(a.ofirst, n, "oblique ranges"))) return rc;
  if (a.sfirst && (rc = check_csr(a.sfirst, n, "signature ranges"))) return rc;
  const uint64_t ne = a.ofirst ? c->oblique_first[n] : 0, ns = a.sfirst ? c->aggregate_sig_first[n] : 0;
  if (a.ofirst && c->oblique_first[0] != 0) return fail(PZ_EINVAL, "oblique ranges must start at 0");
  if (a.sfirst && c->aggregate_sig_first[0] != 0) return fail(PZ_EINVAL, "signature ranges must start at 0");
  if (ne && (rc = check_csr(c->oblique_offs, ne, "oblique elements"))) return rc;
  DeviceCtx* ctx;
  if ((rc = acquire(&ctx))) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if ((rc = ctx->ensure_stream())) return rc;
  Stager st{ctx, ctx->stream};
  uint64_t bytes_total = 0;
  std::vector<uint64_t> rb[3];
  for (int k = 0; k < 3; ++k) {
    if (a.col[k]) a.col[k] = st.up(a.col[k], n);
    if (a.boff[k]) {
      rb[k] = rebase(a.boff[k], n);
      a.bdat[k] = st.up(a.bdat[k] + a.boff[k][0], rb[k][n]);
      a.boff[k] = st.up(rb[k].data(), n + 1);
      bytes_total += rb[k][n];
    }
  }
  std::vector<uint64_t> oo;
  if (a.ofirst) {
    a.ofirst = st.up(a.ofirst, n + 1);
    if (ne) {
      oo = rebase(c->oblique_offs, ne);
      a.odat = st.up(c->oblique_parent_hashes + c->oblique_offs[0], oo[ne]);
      a.ooff = st.up(oo.data(), ne + 1);
      bytes_total += oo[ne];
    } else {
      a.ooff = st.up(c->oblique_offs, 1);
    }
  }
  if (a.sfirst) {
    a.sfirst = st.up(a.sfirst, n + 1);
    a.sig = st.up(c->aggregate_sig, std::max<uint64_t>(ns, 1));
  }
  void* scratch = st.up<uint8_t>(nullptr, pz_wire_attestations_scratch_bytes(n));
  a.offs = st.zeros<uint64_t>(n + 1);
  a.out = st.up<uint8_t>(nullptr, pz_wire_attestations_bound(n, bytes_total, ne, ns));
  if (st.rc) return st.rc;
  // one pass into the bound-sized device buffer; the length is known once it has run
  st.check(launch_encode(a, scratch, st.s), "pz_wire_att kernels");
  uint64_t total = 0;
  st.down(&total, a.offs + n, 1);
  if (st.sync()) return st.rc;
  *len = total;
  if (total > cap) return fail(PZ_ERANGE, "output needs %llu bytes, capacity %llu", (unsigned long long)total,
                               (unsigned long long)cap);
  if (!out) return fail(PZ_EINVAL, "out is null");
  st.down(out, a.out, total);
  if (offsets) st.down(offsets, a.offs, n + 1);
  return st.sync();
}

}  // extern "C"

#ifdef PZ_AB_BUILD
extern "C" int pz_debug_set_att_write_variant(int v) {
  const int old = pz::g_att_variant;
  pz::g_att_variant = v;
  return old;
}
#endif
