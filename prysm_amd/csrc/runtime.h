// Internal runtime helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <vector>

#include "../../include/prysm_hip.h"

namespace pz {

// Grow-only device allocation (padded by 256 B so CSR readers may over-read 4 bytes).
struct DevBuf {
  void* ptr = nullptr;
  size_t cap = 0;
  int reserve(size_t bytes);
  void release();
};

struct DeviceCtx {
  int device = 0;
  bool checked = false;  // gfx950 verified
  std::mutex mu;
  hipStream_t stream = nullptr;
  DevBuf in, out, aux;
  DevBuf slot[24];  // staging for the T/R host-pointer entry points
  static DeviceCtx* get(int dev);
  int ensure_stream();
};

int fail(int code, const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);
int acquire(DeviceCtx** out);
int device_ctx(int device, DeviceCtx** out);

// Copies host arrays into the context's staging slots and tracks the stream.
struct Stager {
  DeviceCtx* c;
  hipStream_t s;
  int next = 0;
  int rc = PZ_OK;

  template <typename T>
  T* up(const T* host, size_t count) {
    if (rc) return nullptr;
    DevBuf& b = c->slot[next++];
    size_t bytes = count * sizeof(T);
    if ((rc = b.reserve(bytes ? bytes : 16))) return nullptr;
    if (bytes && host) {
      hipError_t e = hipMemcpyAsync(b.ptr, host, bytes, hipMemcpyHostToDevice, s);
      if (e != hipSuccess) { rc = hip_fail(e, "hipMemcpyAsync H2D"); return nullptr; }
    }
    return static_cast<T*>(b.ptr);
  }
  template <typename T>
  T* zeros(size_t count, int byte = 0) {
    if (rc) return nullptr;
    DevBuf& b = c->slot[next++];
    size_t bytes = count * sizeof(T);
    if ((rc = b.reserve(bytes ? bytes : 16))) return nullptr;
    if (bytes) {
      hipError_t e = hipMemsetAsync(b.ptr, byte, bytes, s);
      if (e != hipSuccess) { rc = hip_fail(e, "hipMemsetAsync"); return nullptr; }
    }
    return static_cast<T*>(b.ptr);
  }
  template <typename T>
  int down(T* host, const T* dev, size_t count) {
    if (rc || !count) return rc;
    hipError_t e = hipMemcpyAsync(host, dev, count * sizeof(T), hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) rc = hip_fail(e, "hipMemcpyAsync D2H");
    return rc;
  }
  int sync() {
    if (rc) return rc;
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize");
    return rc;
  }
  int check(hipError_t e, const char* what) {
    if (!rc && e != hipSuccess) rc = hip_fail(e, what);
    return rc;
  }
};

// Host CSR offsets rebased to 0 (so device buffers hold only the referenced bytes).
inline std::vector<uint64_t> rebase(const uint64_t* offs, uint64_t n) {
  std::vector<uint64_t> r(n + 1);
  for (uint64_t i = 0; i <= n; ++i) r[i] = offs[i] - offs[0];
  return r;
}

inline int check_csr(const uint64_t* offs, uint64_t n, const char* what) {
  if (!offs) return fail(PZ_EINVAL, "%s offsets are null", what);
  for (uint64_t i = 0; i < n; ++i)
    if (offs[i + 1] < offs[i]) return fail(PZ_EINVAL, "%s offsets not monotone at %llu", what, (unsigned long long)i);
  return PZ_OK;
}

}  // namespace pz
