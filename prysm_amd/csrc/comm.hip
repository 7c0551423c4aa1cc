// pz_comm: RCCL (over xGMI) and loopback communicators, and their C-ABI entry points
// (include/prysm_hip.h, "multi-GPU").  See comm.h for the design.
#include "comm.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>

#include "runtime.h"

namespace pz {

namespace {

std::once_flag g_rccl_once;
RcclApi g_rccl;
int g_rccl_rc = PZ_OK;
char g_rccl_err[256] = "";

template <typename F>
bool bind(void* h, const char* name, F* fn) {
  *fn = reinterpret_cast<F>(dlsym(h, name));
  return *fn != nullptr;
}

void load_rccl() {
  // The copy already in the process first: under PyTorch-ROCm that is torch's librccl, built
  // against the same HIP runtime this library binds to (see prysm_amd/_lib.py); otherwise
  // /opt/rocm's.
  const char* names[] = {"librccl.so", "librccl.so.1"};
  void* h = nullptr;
  for (const char* n : names)
    if ((h = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) { g_rccl.origin = "already loaded"; break; }
  if (!h && (h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL))) g_rccl.origin = "librccl.so.1";
  if (!h && (h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL))) g_rccl.origin = "/opt/rocm/lib/librccl.so.1";
  if (!h) {
    snprintf(g_rccl_err, sizeof g_rccl_err, "librccl not found: %s", dlerror());
    g_rccl_rc = PZ_EDEVICE;
    return;
  }
  bool ok = bind(h, "ncclGetUniqueId", &g_rccl.GetUniqueId) && bind(h, "ncclCommInitRank", &g_rccl.CommInitRank) &&
            bind(h, "ncclCommInitAll", &g_rccl.CommInitAll) && bind(h, "ncclCommDestroy", &g_rccl.CommDestroy) &&
            bind(h, "ncclAllReduce", &g_rccl.AllReduce) && bind(h, "ncclAllGather", &g_rccl.AllGather) &&
            bind(h, "ncclGroupStart", &g_rccl.GroupStart) && bind(h, "ncclGroupEnd", &g_rccl.GroupEnd) &&
            bind(h, "ncclGetErrorString", &g_rccl.GetErrorString);
  if (!ok) {
    snprintf(g_rccl_err, sizeof g_rccl_err, "librccl lacks an entry point: %s", dlerror());
    g_rccl_rc = PZ_EDEVICE;
  }
}

int nccl_fail(const RcclApi* api, ncclResult_t r, const char* what) {
  return fail(PZ_EDEVICE, "%s: %s", what, api && api->GetErrorString ? api->GetErrorString(r) : "RCCL error");
}

// Sum of the loopback ranks' buffers, written back to every one of them.
constexpr int kMaxLoopback = 64;
struct LoopPtrs {
  uint64_t* p[kMaxLoopback];
};

extern "C" __global__ void __launch_bounds__(256)
pz_loopback_sum_kernel(LoopPtrs ptrs, int world, uint64_t count) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  uint64_t s = 0;
  for (int r = 0; r < world; ++r) s += ptrs.p[r][i];
  for (int r = 0; r < world; ++r) ptrs.p[r][i] = s;
}

struct LoopPtrs32 {
  uint32_t* p[kMaxLoopback];
};

extern "C" __global__ void __launch_bounds__(256)
pz_loopback_min_kernel(LoopPtrs32 ptrs, int world, uint64_t count) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  uint32_t m = 0xFFFFFFFFu;
  for (int r = 0; r < world; ++r) m = min(m, ptrs.p[r][i]);
  for (int r = 0; r < world; ++r) ptrs.p[r][i] = m;
}

}  // namespace

int rccl_api(const RcclApi** out) {
  std::call_once(g_rccl_once, load_rccl);
  if (g_rccl_rc) return fail(g_rccl_rc, "%s", g_rccl_err);
  *out = &g_rccl;
  return PZ_OK;
}

}  // namespace pz

using namespace pz;

// Orders the collective stream of every local rank after its compute stream.
static int order_after(pz_comm* c, const hipStream_t* compute) {
  for (int i = 0; i < c->nlocal; ++i) {
    hipError_t e = hipSetDevice(c->dev[i]);
    if (e == hipSuccess) e = hipEventRecord(c->ev_in[i], compute[i]);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->cs(i), c->ev_in[i], 0);
    if (e != hipSuccess) return hip_fail(e, "collective ordering");
  }
  return PZ_OK;
}

static hipEvent_t timing_event(pz_comm* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// With timing on: the start of a collective on every local rank's collective stream (after
// order_after, so the wait for the compute stream is not counted).
static int time_begin(pz_comm* c) {
  if (!c->timing) return PZ_OK;
  c->timed.emplace_back();
  c->time_open = true;
  pz_comm::TimedOp& t = c->timed.back();
  for (int i = 0; i < c->nlocal; ++i) {
    (void)hipSetDevice(c->dev[i]);
    t.t0.push_back(timing_event(c));
    t.t1.push_back(timing_event(c));
    hipError_t e = hipEventRecord(t.t0.back(), c->cs(i));
    if (e != hipSuccess) return hip_fail(e, "collective timing event");
  }
  return PZ_OK;
}

static int mark_done(pz_comm* c, hipEvent_t* done) {
  for (int i = 0; i < c->nlocal; ++i) {
    hipError_t e = hipSetDevice(c->dev[i]);
    if (e == hipSuccess && c->time_open) e = hipEventRecord(c->timed.back().t1[i], c->cs(i));
    if (e == hipSuccess) e = hipEventRecord(done[i], c->cs(i));
    if (e != hipSuccess) return hip_fail(e, "collective completion event");
  }
  c->time_open = false;
  return PZ_OK;
}

// SHM: the local rank's buffer to host memory, through the process group, and back -- on the
// collective stream, which is drained on both sides (the group is synchronous).
template <typename F>
static int shm_run(pz_comm* c, void* dbuf, size_t down_bytes, size_t up_bytes, size_t up_offset, F&& collective) {
  (void)hipSetDevice(c->dev[0]);
  c->shm_stage.resize(std::max(down_bytes, up_offset + up_bytes));
  hipError_t e = hipSuccess;
  if (down_bytes) e = hipMemcpyAsync(c->shm_stage.data(), dbuf, down_bytes, hipMemcpyDeviceToHost, c->cstream[0]);
  if (e == hipSuccess) e = hipStreamSynchronize(c->cstream[0]);
  if (e != hipSuccess) return hip_fail(e, "shm collective: D2H");
  std::string err;
  int rc = collective(c->shm_stage.data(), &err);
  if (rc) return fail(rc, "%s", err.c_str());
  if (up_bytes) e = hipMemcpyAsync(dbuf, c->shm_stage.data() + up_offset, up_bytes, hipMemcpyHostToDevice, c->cstream[0]);
  if (e == hipSuccess) e = hipStreamSynchronize(c->cstream[0]);
  if (e != hipSuccess) return hip_fail(e, "shm collective: H2D");
  return PZ_OK;
}

int pz_comm::allreduce_u64(uint64_t* const* bufs, size_t count, const hipStream_t* compute, hipEvent_t* done) {
  int rc = order_after(this, compute);
  if (!rc) rc = time_begin(this);
  if (rc) return rc;
  if (count && world > 1) {
    if (kind == LOOPBACK) {
      LoopPtrs p;
      for (int r = 0; r < world; ++r) p.p[r] = bufs[r];
      (void)hipSetDevice(dev[0]);
      hipLaunchKernelGGL(pz_loopback_sum_kernel, dim3((uint32_t)((count + 255) / 256)), dim3(256), 0, cstream[0], p,
                         world, (uint64_t)count);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return hip_fail(e, "pz_loopback_sum_kernel");
    } else if (kind == SHM) {
      rc = shm_run(this, bufs[0], count * 8, count * 8, 0, [&](uint8_t* h, std::string* err) {
        return shm->sum_u64(reinterpret_cast<uint64_t*>(h), count, err);
      });
      if (rc) return rc;
    } else {
      if (nlocal > 1) api->GroupStart();
      ncclResult_t r = ncclSuccess;
      for (int i = 0; i < nlocal && r == ncclSuccess; ++i) {
        (void)hipSetDevice(dev[i]);
        r = api->AllReduce(bufs[i], bufs[i], count, ncclUint64, ncclSum, nccl[i], cstream[i]);
      }
      ncclResult_t g = nlocal > 1 ? api->GroupEnd() : ncclSuccess;
      if (r != ncclSuccess) return nccl_fail(api, r, "ncclAllReduce");
      if (g != ncclSuccess) return nccl_fail(api, g, "ncclGroupEnd");
    }
  }
  return mark_done(this, done);
}

int pz_comm::allreduce_sum_min(uint64_t* const* sbufs, size_t scount, uint32_t* const* mbufs, size_t mcount,
                               const hipStream_t* compute, hipEvent_t* done) {
  int rc = order_after(this, compute);
  if (!rc) rc = time_begin(this);
  if (rc) return rc;
  if (world > 1 && (scount || mcount)) {
    if (kind == LOOPBACK) {
      (void)hipSetDevice(dev[0]);
      if (scount) {
        LoopPtrs p;
        for (int r = 0; r < world; ++r) p.p[r] = sbufs[r];
        hipLaunchKernelGGL(pz_loopback_sum_kernel, dim3((uint32_t)((scount + 255) / 256)), dim3(256), 0, cstream[0],
                           p, world, (uint64_t)scount);
      }
      if (mcount) {
        LoopPtrs32 p;
        for (int r = 0; r < world; ++r) p.p[r] = mbufs[r];
        hipLaunchKernelGGL(pz_loopback_min_kernel, dim3((uint32_t)((mcount + 255) / 256)), dim3(256), 0, cstream[0],
                           p, world, (uint64_t)mcount);
      }
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return hip_fail(e, "loopback sum/min");
    } else if (kind == SHM) {
      // both buffers through one group round sequence: stage = [sum words][min words]
      (void)hipSetDevice(dev[0]);
      shm_stage.resize(scount * 8 + mcount * 4);
      hipError_t e = hipSuccess;
      if (scount) e = hipMemcpyAsync(shm_stage.data(), sbufs[0], scount * 8, hipMemcpyDeviceToHost, cstream[0]);
      if (e == hipSuccess && mcount)
        e = hipMemcpyAsync(shm_stage.data() + scount * 8, mbufs[0], mcount * 4, hipMemcpyDeviceToHost, cstream[0]);
      if (e == hipSuccess) e = hipStreamSynchronize(cstream[0]);
      if (e != hipSuccess) return hip_fail(e, "shm collective: D2H");
      std::string err;
      rc = shm->sum_min(reinterpret_cast<uint64_t*>(shm_stage.data()), scount,
                        reinterpret_cast<uint32_t*>(shm_stage.data() + scount * 8), mcount, &err);
      if (rc) return fail(rc, "%s", err.c_str());
      if (scount) e = hipMemcpyAsync(sbufs[0], shm_stage.data(), scount * 8, hipMemcpyHostToDevice, cstream[0]);
      if (e == hipSuccess && mcount)
        e = hipMemcpyAsync(mbufs[0], shm_stage.data() + scount * 8, mcount * 4, hipMemcpyHostToDevice, cstream[0]);
      if (e == hipSuccess) e = hipStreamSynchronize(cstream[0]);
      if (e != hipSuccess) return hip_fail(e, "shm collective: H2D");
    } else {
      api->GroupStart();
      ncclResult_t r = ncclSuccess;
      for (int i = 0; i < nlocal && r == ncclSuccess; ++i) {
        (void)hipSetDevice(dev[i]);
        if (scount) r = api->AllReduce(sbufs[i], sbufs[i], scount, ncclUint64, ncclSum, nccl[i], cstream[i]);
        if (r == ncclSuccess && mcount)
          r = api->AllReduce(mbufs[i], mbufs[i], mcount, ncclUint32, ncclMin, nccl[i], cstream[i]);
      }
      ncclResult_t g = api->GroupEnd();
      if (r != ncclSuccess) return nccl_fail(api, r, "ncclAllReduce (sum/min)");
      if (g != ncclSuccess) return nccl_fail(api, g, "ncclGroupEnd");
    }
  }
  return mark_done(this, done);
}

int pz_comm::allgather(const void* const* send, void* const* recv, size_t bytes, const hipStream_t* compute,
                       hipEvent_t* done) {
  int rc = order_after(this, compute);
  if (!rc) rc = time_begin(this);
  if (rc) return rc;
  if (bytes) {
    if (kind == SHM && world > 1) {
      // D2H of this rank's contribution, the gather through the group, H2D of all of it
      (void)hipSetDevice(dev[0]);
      shm_stage.resize(bytes + (size_t)world * bytes);
      hipError_t e = hipMemcpyAsync(shm_stage.data(), send[0], bytes, hipMemcpyDeviceToHost, cstream[0]);
      if (e == hipSuccess) e = hipStreamSynchronize(cstream[0]);
      if (e != hipSuccess) return hip_fail(e, "shm all-gather: D2H");
      std::string err;
      rc = shm->allgather(shm_stage.data(), shm_stage.data() + bytes, bytes, &err);
      if (rc) return fail(rc, "%s", err.c_str());
      e = hipMemcpyAsync(recv[0], shm_stage.data() + bytes, (size_t)world * bytes, hipMemcpyHostToDevice, cstream[0]);
      if (e == hipSuccess) e = hipStreamSynchronize(cstream[0]);
      if (e != hipSuccess) return hip_fail(e, "shm all-gather: H2D");
    } else if (kind == LOOPBACK || world == 1) {
      for (int i = 0; i < nlocal; ++i) {
        (void)hipSetDevice(dev[i]);
        for (int r = 0; r < world; ++r) {
          hipError_t e = hipMemcpyAsync(static_cast<uint8_t*>(recv[i]) + (size_t)r * bytes, send[r], bytes,
                                        hipMemcpyDeviceToDevice, cs(i));
          if (e != hipSuccess) return hip_fail(e, "loopback all-gather copy");
        }
      }
    } else {
      if (nlocal > 1) api->GroupStart();
      ncclResult_t r = ncclSuccess;
      for (int i = 0; i < nlocal && r == ncclSuccess; ++i) {
        (void)hipSetDevice(dev[i]);
        r = api->AllGather(send[i], recv[i], bytes, ncclUint8, nccl[i], cstream[i]);
      }
      ncclResult_t g = nlocal > 1 ? api->GroupEnd() : ncclSuccess;
      if (r != ncclSuccess) return nccl_fail(api, r, "ncclAllGather");
      if (g != ncclSuccess) return nccl_fail(api, g, "ncclGroupEnd");
    }
  }
  return mark_done(this, done);
}

pz_comm::~pz_comm() {
  for (size_t i = 0; i < cstream.size(); ++i) {
    (void)hipSetDevice(dev[i]);
    if (cstream[i]) {
      (void)hipStreamSynchronize(cstream[i]);
      (void)hipStreamDestroy(cstream[i]);
    }
    if (i < ev_in.size() && ev_in[i]) (void)hipEventDestroy(ev_in[i]);
  }
  if (api)
    for (ncclComm_t n : nccl)
      if (n) api->CommDestroy(n);
  for (TimedOp& t : timed) {
    for (hipEvent_t e : t.t0) (void)hipEventDestroy(e);
    for (hipEvent_t e : t.t1) (void)hipEventDestroy(e);
  }
  for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
  delete shm;
}

// Creates the per-local-rank streams/events after dev[] is set.
static int comm_setup(pz_comm* c) {
  c->cstream.assign(c->nlocal, nullptr);
  c->ev_in.assign(c->nlocal, nullptr);
  for (int i = 0; i < c->nlocal; ++i) {
    DeviceCtx* dc;
    int rc = device_ctx(c->dev[i], &dc);  // gfx950 check + the device's library context
    if (rc) return rc;
    hipError_t e = hipSetDevice(c->dev[i]);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->cstream[i], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_in[i], hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(e, "communicator stream/event");
  }
  return PZ_OK;
}

extern "C" {

int pz_comm_unique_id(uint8_t id[PZ_COMM_ID_BYTES]) {
  if (!id) return fail(PZ_EINVAL, "id is null");
  const RcclApi* api;
  int rc = rccl_api(&api);
  if (rc) return rc;
  ncclUniqueId u;
  ncclResult_t r = api->GetUniqueId(&u);
  if (r != ncclSuccess) return nccl_fail(api, r, "ncclGetUniqueId");
  static_assert(sizeof(u.internal) == PZ_COMM_ID_BYTES, "unique id size");
  std::memcpy(id, u.internal, PZ_COMM_ID_BYTES);
  return PZ_OK;
}

int pz_comm_init_rank(const uint8_t id[PZ_COMM_ID_BYTES], int world, int rank, int device, pz_comm** out) {
  if (!id || !out) return fail(PZ_EINVAL, "null pointer");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return fail(PZ_EINVAL, "rank %d of world %d", rank, world);
  const RcclApi* api;
  int rc = rccl_api(&api);
  if (rc) return rc;
  pz_comm* c = new pz_comm();
  c->kind = pz_comm::RCCL;
  c->api = api;
  c->world = world;
  c->nlocal = 1;
  c->rank0 = rank;
  c->dev = {device};
  if ((rc = comm_setup(c))) {
    delete c;
    return rc;
  }
  ncclUniqueId u;
  std::memcpy(u.internal, id, PZ_COMM_ID_BYTES);
  c->nccl.assign(1, nullptr);
  (void)hipSetDevice(device);
  ncclResult_t r = api->CommInitRank(&c->nccl[0], world, u, rank);
  if (r != ncclSuccess) {
    c->nccl.clear();
    delete c;
    return nccl_fail(api, r, "ncclCommInitRank");
  }
  *out = c;
  return PZ_OK;
}

int pz_init_devices(int ndev, const int* devices, pz_comm** out) {
  if (!out) return fail(PZ_EINVAL, "out is null");
  *out = nullptr;
  int n = 0;
  if (pz_device_count(&n)) return PZ_EDEVICE;
  if (ndev < 1 || ndev > n) return fail(PZ_EINVAL, "ndev %d of %d devices", ndev, n);
  const RcclApi* api;
  int rc = rccl_api(&api);
  if (rc) return rc;
  pz_comm* c = new pz_comm();
  c->kind = pz_comm::RCCL;
  c->api = api;
  c->world = c->nlocal = ndev;
  c->rank0 = 0;
  for (int i = 0; i < ndev; ++i) c->dev.push_back(devices ? devices[i] : i);
  if ((rc = comm_setup(c))) {
    delete c;
    return rc;
  }
  c->nccl.assign(ndev, nullptr);
  ncclResult_t r = api->CommInitAll(c->nccl.data(), ndev, c->dev.data());
  if (r != ncclSuccess) {
    c->nccl.clear();
    delete c;
    return nccl_fail(api, r, "ncclCommInitAll");
  }
  *out = c;
  return PZ_OK;
}

int pz_comm_init_loopback(int world, int device, pz_comm** out) {
  if (!out) return fail(PZ_EINVAL, "out is null");
  *out = nullptr;
  if (world < 1 || world > kMaxLoopback) return fail(PZ_EINVAL, "loopback world %d not in [1, %d]", world, kMaxLoopback);
  pz_comm* c = new pz_comm();
  c->kind = pz_comm::LOOPBACK;
  c->world = c->nlocal = world;
  c->rank0 = 0;
  c->dev.assign(world, device);
  int rc = comm_setup(c);
  if (rc) {
    delete c;
    return rc;
  }
  *out = c;
  return PZ_OK;
}

int pz_comm_init_shm(const char* name, int world, int rank, int device, uint32_t timeout_ms, pz_comm** out) {
  if (!name || !out) return fail(PZ_EINVAL, "null pointer");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return fail(PZ_EINVAL, "rank %d of world %d", rank, world);
  pz_comm* c = new pz_comm();
  c->kind = pz_comm::SHM;
  c->world = world;
  c->nlocal = 1;
  c->rank0 = rank;
  c->dev = {device};
  int rc = comm_setup(c);
  if (rc) {
    delete c;
    return rc;
  }
  std::string err;
  rc = ShmGroup::open(name, world, rank, timeout_ms ? timeout_ms : 60000, uint64_t(8) << 20, &c->shm, &err);
  if (rc) {
    delete c;
    return fail(rc, "%s", err.c_str());
  }
  *out = c;
  return PZ_OK;
}

int pz_comm_set_timing(pz_comm* c, int on) {
  if (!c) return fail(PZ_EINVAL, "comm is null");
  c->timing = on != 0;
  return PZ_OK;
}

int pz_comm_collective_time(pz_comm* c, double* ms, uint64_t* count) {
  if (!c || !ms || !count) return fail(PZ_EINVAL, "null pointer");
  // every elapsed time first; the events go back to the pool only once all were read, so an
  // error leaves each event owned by `timed` alone (the destructor destroys it once)
  double sum = 0;
  for (pz_comm::TimedOp& t : c->timed) {
    float mx = 0;
    for (size_t i = 0; i < t.t0.size(); ++i) {
      (void)hipSetDevice(c->dev[i]);
      hipError_t e = hipEventSynchronize(t.t1[i]);
      float v = 0;
      if (e == hipSuccess) e = hipEventElapsedTime(&v, t.t0[i], t.t1[i]);
      if (e != hipSuccess) return hip_fail(e, "collective timing");
      mx = std::max(mx, v);
    }
    sum += mx;
  }
  for (pz_comm::TimedOp& t : c->timed)
    for (size_t i = 0; i < t.t0.size(); ++i) {
      c->ev_pool.push_back(t.t0[i]);
      c->ev_pool.push_back(t.t1[i]);
    }
  *ms = sum;
  *count = c->timed.size();
  c->timed.clear();
  return PZ_OK;
}

int pz_comm_size(const pz_comm* c, int* world, int* nlocal, int* first_rank) {
  if (!c) return fail(PZ_EINVAL, "comm is null");
  if (world) *world = c->world;
  if (nlocal) *nlocal = c->nlocal;
  if (first_rank) *first_rank = c->rank0;
  return PZ_OK;
}

int pz_comm_device(const pz_comm* c, int local, int* device) {
  if (!c || !device) return fail(PZ_EINVAL, "null pointer");
  if (local < 0 || local >= c->nlocal) return fail(PZ_EINVAL, "local rank %d of %d", local, c->nlocal);
  *device = c->dev[local];
  return PZ_OK;
}

void pz_comm_free(pz_comm* c) { delete c; }

}  // extern "C"
