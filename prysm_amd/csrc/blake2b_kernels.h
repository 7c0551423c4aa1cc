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
// Where message i's 64 signed parent ids are: trail[wstart, wstart + nw), then oids[ooff, ooff + 64 - nw).
struct AttMsgRef {
  uint32_t wstart, nw, ooff, pad;
};
// processAttestation message digests (64 B each) from the engine's device hash log:
// message i = hdr[16 i .. 16 i + 10) | 64 x (hlog[id(i, r)] | ' ') | sbh[sbh_offs[i]..sbh_offs[i+1]).
hipError_t launch_b2b_attmsg(const uint8_t* hlog, const uint32_t* trail, const AttMsgRef* ref, const uint32_t* oids,
                             const uint8_t* hdr, const uint8_t* sbh, const uint64_t* sbh_offs, uint64_t n, uint8_t* out,
                             hipStream_t stream);
}  // namespace pz

namespace pz {
// Kernel variant for the fixed-length path (1: persistent LDS-DMA, 0: plain grid); returns the
// previous one.  Exposed for in-process A/B timing (pz_debug_set_hash_variant).
int set_fixed_variant(int v);
}  // namespace pz
