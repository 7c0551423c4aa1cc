// Internal runtime helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <mutex>

#include "../../include/prysm_hip.h"

namespace pz {

// Grow-only device allocation (padded by 256 B so CSR readers may over-read 4 bytes).
struct DevBuf {
  void* ptr = nullptr;
  size_t cap = 0;
  int reserve(size_t bytes);
};

struct DeviceCtx {
  int device = 0;
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

}  // namespace pz
