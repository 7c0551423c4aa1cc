// C-ABI runtime: device contexts, staging buffers, error reporting and the host-pointer
// (Go drop-in) entry points of include/prysm_hip.h.  Thread-safe: one mutex and one
// library-owned stream per device; the host-pointer API never retains caller pointers.
#include "runtime.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "blake2b_kernels.h"
#include "serial_hash.h"

namespace pz {

static thread_local std::string g_err;
static thread_local int g_device = -1;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(PZ_EDEVICE, "%s: %s", what, hipGetErrorString(e));
}

static std::mutex g_ctx_mu;
static std::vector<DeviceCtx*> g_ctx;

DeviceCtx* DeviceCtx::get(int dev) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if ((int)g_ctx.size() <= dev) g_ctx.resize(dev + 1, nullptr);
  if (!g_ctx[dev]) {
    DeviceCtx* c = new DeviceCtx();
    c->device = dev;
    g_ctx[dev] = c;
  }
  return g_ctx[dev];
}

int DeviceCtx::ensure_stream() {
  if (stream) return PZ_OK;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
  if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
  return PZ_OK;
}

int DevBuf::reserve(size_t bytes) {
  if (bytes <= cap) return PZ_OK;
  if (ptr) (void)hipFree(ptr);
  ptr = nullptr;
  cap = 0;
  size_t want = bytes + 256;  // padding: CSR readers may touch 4 bytes past the end
  hipError_t e = hipMalloc(&ptr, want);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc");
  cap = bytes;
  return PZ_OK;
}

void DevBuf::release() {
  if (ptr) (void)hipFree(ptr);
  ptr = nullptr;
  cap = 0;
}

// A device's library context, after checking that it is a gfx950 (no fallback to anything
// else); does not change the calling thread's default device.
int device_ctx(int device, DeviceCtx** out) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return fail(PZ_EDEVICE, "no HIP device available (%s)", e != hipSuccess ? hipGetErrorString(e) : "0 devices");
  if (device < 0 || device >= n) return fail(PZ_EINVAL, "device %d out of range [0,%d)", device, n);
  DeviceCtx* c = DeviceCtx::get(device);
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->checked) {
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      return fail(PZ_EDEVICE, "device %d is %s; this library is built for gfx950 only", device, prop.gcnArchName);
    c->checked = true;
  }
  int rc = c->ensure_stream();
  if (rc) return rc;
  *out = c;
  return PZ_OK;
}

// Resolve the calling thread's device and lock it.  Fails loudly when no device exists.
int acquire(DeviceCtx** out) {
  if (g_device < 0) {
    int rc = pz_init(0);
    if (rc != PZ_OK) return rc;
  }
  DeviceCtx* c = DeviceCtx::get(g_device);
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  *out = c;
  return PZ_OK;
}

}  // namespace pz

using namespace pz;

extern "C" {

int pz_version(void) { return 1; }

const char* pz_last_error(void) { return g_err.c_str(); }

int pz_device_count(int* count) {
  if (!count) return fail(PZ_EINVAL, "count is null");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return hip_fail(e, "hipGetDeviceCount");
  }
  *count = n;
  return PZ_OK;
}

int pz_init(int device) {
  DeviceCtx* c;
  int rc = device_ctx(device, &c);
  if (rc) return rc;
  g_device = device;
  return PZ_OK;
}

void pz_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  for (DeviceCtx*& c : g_ctx) {
    if (!c) continue;
    {
      std::lock_guard<std::mutex> l2(c->mu);
      (void)hipSetDevice(c->device);
      if (c->stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
      }
      c->in.release();
      c->out.release();
      c->aux.release();
      for (DevBuf& b : c->slot) b.release();
    }
    delete c;
    c = nullptr;
  }
  g_ctx.clear();
  g_device = -1;
}

// ---- H -------------------------------------------------------------------------------------
int pz_dev_blake2b512_fixed(const uint8_t* d_msgs, uint64_t stride, uint64_t len, uint64_t n,
                            uint8_t* d_out, uint32_t out_bytes, void* stream) {
  if (out_bytes != 32 && out_bytes != 64) return fail(PZ_EINVAL, "out_bytes must be 32 or 64");
  if (n == 0) return PZ_OK;
  if (!d_msgs || !d_out) return fail(PZ_EINVAL, "null pointer");
  if (stride % 16 || stride < len || stride >= (1ull << 26) || (reinterpret_cast<uintptr_t>(d_msgs) & 15) ||
      (reinterpret_cast<uintptr_t>(d_out) & 15))
    return fail(PZ_EINVAL, "fixed layout needs 16-B aligned buffers, stride %% 16 == 0, len <= stride < 64 MiB");
  hipError_t e = launch_b2b_fixed(d_msgs, stride, len, n, d_out, out_bytes, (hipStream_t)stream);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_b2b_fixed_kernel");
}

int pz_dev_blake2b512_batch(const uint8_t* d_msgs, const uint64_t* d_offsets, uint64_t n,
                            uint8_t* d_out, uint32_t out_bytes, void* stream) {
  if (out_bytes != 32 && out_bytes != 64) return fail(PZ_EINVAL, "out_bytes must be 32 or 64");
  if (n == 0) return PZ_OK;
  if (!d_msgs || !d_offsets || !d_out) return fail(PZ_EINVAL, "null pointer");
  if (reinterpret_cast<uintptr_t>(d_out) & 15) return fail(PZ_EINVAL, "d_out must be 16-B aligned");
  hipError_t e = launch_b2b_csr(d_msgs, d_offsets, n, d_out, out_bytes, (hipStream_t)stream);
  return e == hipSuccess ? PZ_OK : hip_fail(e, "pz_b2b_csr_kernel");
}

}  // extern "C"

namespace pz {
// The batch hash on one device's context (arguments already validated).
int hash_batch_on(DeviceCtx* c, const uint8_t* msgs, const uint64_t* offsets, uint64_t n, uint8_t* out,
                  uint32_t out_bytes) {
  if (n == 0) return PZ_OK;
  hipError_t e0 = hipSetDevice(c->device);
  if (e0 != hipSuccess) return hip_fail(e0, "hipSetDevice");
  const uint64_t base = offsets[0], total = offsets[n] - offsets[0];
  int rc;

  // A small batch (a drop-in Hash() call hashes ONE 100-600 B message, types/block.go:67-77)
  // costs a few compressions, ~1 us on one host core, against tens of microseconds of launch,
  // PCIe copies and stream sync on the GPU route: below the measured crossover it is hashed
  // on the calling thread (profiles/r02/hash_latency*.json).
  if (n <= small_batch_threshold()) {
    uint64_t comps = 0;
    for (uint64_t i = 0; i < n && comps <= small_batch_threshold(); ++i)
      comps += (offsets[i + 1] - offsets[i] + 127) / 128 + (offsets[i + 1] == offsets[i]);
    if (comps <= small_batch_threshold()) {
      std::vector<uint64_t> all(n);
      for (uint64_t i = 0; i < n; ++i) all[i] = i;
      host_blake2b512_many(msgs, offsets, all, out, out_bytes, 1);
      return PZ_OK;
    }
  }

  // Long messages (serial chains) go to host threads while the GPU hashes the rest.
  std::vector<uint64_t> lng = long_messages(offsets, n);
  if (!lng.empty()) {
    SerialHashJob job;
    job.start(msgs, offsets, lng, out, out_bytes);
    if (lng.size() == n) return PZ_OK;  // joined by the destructor
    std::vector<uint8_t> cat;
    std::vector<uint64_t> co{0}, idx;
    size_t k = 0;
    for (uint64_t i = 0; i < n; ++i) {
      if (k < lng.size() && lng[k] == i) {
        ++k;
        continue;
      }
      cat.insert(cat.end(), msgs + offsets[i], msgs + offsets[i + 1]);
      co.push_back(cat.size());
      idx.push_back(i);
    }
    std::vector<uint8_t> part(idx.size() * out_bytes);
    rc = hash_batch_on(c, cat.data(), co.data(), idx.size(), part.data(), out_bytes);
    job.join();
    if (rc) return rc;
    for (size_t j = 0; j < idx.size(); ++j) std::memcpy(out + idx[j] * out_bytes, &part[j * out_bytes], out_bytes);
    return PZ_OK;
  }

  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = c->ensure_stream())) return rc;
  hipStream_t s = c->stream;

  // Uniform records at a 16-B multiple stride use the LDS-staged fixed-length kernel.
  const uint64_t len0 = offsets[1] - offsets[0];
  bool uniform = (len0 % 16 == 0) && len0 > 0 && len0 < (1ull << 26);
  for (uint64_t i = 1; uniform && i < n; ++i) uniform = (offsets[i + 1] - offsets[i]) == len0;

  if ((rc = c->in.reserve(total + 16))) return rc;
  if ((rc = c->out.reserve(n * out_bytes))) return rc;
  hipError_t e;
  if (total) {
    e = hipMemcpyAsync(c->in.ptr, msgs + base, total, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync H2D");
  }
  if (uniform) {
    e = launch_b2b_fixed((const uint8_t*)c->in.ptr, len0, len0, n, (uint8_t*)c->out.ptr, out_bytes, s);
  } else {
    std::vector<uint64_t> rel(n + 1);
    for (uint64_t i = 0; i <= n; ++i) rel[i] = offsets[i] - base;
    if ((rc = c->aux.reserve((n + 1) * sizeof(uint64_t)))) return rc;
    e = hipMemcpyAsync(c->aux.ptr, rel.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync H2D offsets");
    // the pageable source must stay alive until the copy completes
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    e = launch_b2b_csr((const uint8_t*)c->in.ptr, (const uint64_t*)c->aux.ptr, n,
                       (uint8_t*)c->out.ptr, out_bytes, s);
  }
  if (e != hipSuccess) return hip_fail(e, "blake2b launch");
  e = hipMemcpyAsync(out, c->out.ptr, n * out_bytes, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync D2H");
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  return PZ_OK;
}

static int check_batch_args(const uint8_t* msgs, const uint64_t* offsets, uint64_t n, uint8_t* out,
                            uint32_t out_bytes) {
  if (out_bytes != 32 && out_bytes != 64) return fail(PZ_EINVAL, "out_bytes must be 32 or 64");
  if (n == 0) return PZ_OK;
  if (!offsets || !out) return fail(PZ_EINVAL, "null pointer");
  if (offsets[n] != offsets[0] && !msgs) return fail(PZ_EINVAL, "null msgs");
  for (uint64_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return fail(PZ_EINVAL, "offsets not monotone at %llu", (unsigned long long)i);
  return PZ_OK;
}
}  // namespace pz

extern "C" {

int pz_blake2b512_batch(const uint8_t* msgs, const uint64_t* offsets, uint64_t n, uint8_t* out,
                        uint32_t out_bytes) {
  int rc = check_batch_args(msgs, offsets, n, out, out_bytes);
  if (rc || n == 0) return rc;
  DeviceCtx* c;
  if ((rc = acquire(&c))) return rc;
  return hash_batch_on(c, msgs, offsets, n, out, out_bytes);
}

int pz_comm_blake2b512_batch(const pz_comm* comm, const uint8_t* msgs, const uint64_t* offsets, uint64_t n,
                             uint8_t* out, uint32_t out_bytes) {
  if (!comm) return fail(PZ_EINVAL, "comm is null");
  int rc = check_batch_args(msgs, offsets, n, out, out_bytes);
  if (rc || n == 0) return rc;
  int world = 1, nlocal = 1, first = 0;
  pz_comm_size(comm, &world, &nlocal, &first);
  std::vector<int> rcs(nlocal, PZ_OK);
  std::vector<std::string> errs(nlocal);
  auto work = [&](int i) {
    const uint64_t r = (uint64_t)(first + i);
    const uint64_t a = n * r / world, b = n * (r + 1) / world;
    int dev = 0;
    DeviceCtx* c;
    int k = pz_comm_device(comm, i, &dev);
    if (!k) k = device_ctx(dev, &c);
    if (!k && b > a) k = hash_batch_on(c, msgs, offsets + a, b - a, out + a * out_bytes, out_bytes);
    rcs[i] = k;
    if (k) errs[i] = g_err;
  };
  if (nlocal == 1) {
    work(0);
  } else {  // one host thread per local rank: the devices hash concurrently
    std::vector<std::thread> th;
    for (int i = 0; i < nlocal; ++i) th.emplace_back(work, i);
    for (std::thread& t : th) t.join();
  }
  for (int i = 0; i < nlocal; ++i)
    if (rcs[i]) return fail(rcs[i], "local rank %d: %s", i, errs[i].c_str());
  return PZ_OK;
}

uint64_t pz_set_serial_threshold(uint64_t bytes) { return set_serial_threshold(bytes); }
uint32_t pz_set_host_threads(uint32_t n) { return set_host_threads(n); }
uint64_t pz_set_small_batch_threshold(uint64_t compressions) { return set_small_batch_threshold(compressions); }

}  // extern "C"

#ifdef PZ_AB_BUILD
// The A/B library only: select the fixed-length hash kernel variant for in-process A/B timing.
extern "C" int pz_debug_set_hash_variant(int v) { return pz::set_fixed_variant(v); }
#endif
