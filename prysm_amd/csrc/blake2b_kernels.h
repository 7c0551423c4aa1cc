// Launchers for the BLAKE2b batch kernels (blake2b.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pz {
hipError_t launch_b2b_fixed(const uint8_t* msgs, uint64_t stride, uint64_t len, uint64_t n,
                            uint8_t* out, uint32_t out_bytes, hipStream_t stream);
hipError_t launch_b2b_csr(const uint8_t* msgs, const uint64_t* offsets, uint64_t n, uint8_t* out,
                          uint32_t out_bytes, hipStream_t stream);
// message i = msgs[begs[i], ends[i]) (spans may overlap; 4 readable bytes past each end)
hipError_t launch_b2b_spans(const uint8_t* msgs, const uint64_t* begs, const uint64_t* ends, uint64_t n, uint8_t* out,
                            uint32_t out_bytes, hipStream_t stream);
// One processAttestation message: its 10-byte header, where its 64 signed parent ids are
// (trail[wstart, wstart + nw), then 64 - nw oblique ids at var[vo..]) and its ShardBlockHash
// (sl bytes right after those ids).  32 bytes, appended by the walk into pinned memory.
struct AttMsg {
  uint8_t hdr[10];
  uint16_t nw;
  uint32_t wstart;
  uint32_t sl;
  uint32_t pad;
  uint64_t vo;  // byte offset into var (a multiple of 4)
};
static_assert(sizeof(AttMsg) == 32, "AttMsg is 32 bytes");
// processAttestation message digests (64 B each) from the engine's device hash log:
// message i = hdr | 64 x (hlog[id(i, r)] | ' ') | ShardBlockHash.
hipError_t launch_b2b_attmsg(const uint8_t* hlog, const uint32_t* trail, const AttMsg* rec, const uint8_t* var, uint64_t n,
                             uint8_t* out, hipStream_t stream);
}  // namespace pz

namespace pz {
// Kernel variant for the fixed-length path (1: persistent LDS-DMA, 0: plain grid); returns the
// previous one.  Exposed for in-process A/B timing (pz_debug_set_hash_variant).
#ifdef PZ_AB_BUILD
int set_fixed_variant(int v);
#endif
}  // namespace pz
