// ShmGroup: host-staged collectives through POSIX shared memory (see shm_group.h).
#include "shm_group.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <new>

#include "../../include/prysm_hip.h"

namespace pz {

namespace {

constexpr uint64_t kMagic = 0x707a5f73686d3031ULL;  // "pz_shm01"

struct alignas(64) RankCtl {
  std::atomic<uint64_t> posted;    // last round whose chunk and descriptor are in the slot
  std::atomic<uint64_t> consumed;  // last round this rank has finished reading
  std::atomic<uint32_t> joined;
  uint32_t op;
  uint64_t a, b, chunk;
};

struct Header {
  std::atomic<uint64_t> magic;  // written last by rank 0
  uint32_t world;
  uint32_t pad;
  uint64_t slot_bytes;
  std::atomic<int32_t> aborted;  // 0, or 1 + the rank that aborted the group
  RankCtl r[ShmGroup::kMaxWorld];
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "cross-process atomics need lock-free words");

size_t data_offset() { return (sizeof(Header) + 4095) & ~size_t(4095); }

Header* hdr(void* base) { return static_cast<Header*>(base); }

uint8_t* slot(void* base, uint64_t slot_bytes, int q) {
  return static_cast<uint8_t*>(base) + data_offset() + (size_t)q * slot_bytes;
}

const char* op_name(uint32_t op) {
  switch (op) {
    case ShmGroup::kSumU64: return "all-reduce(u64 sum)";
    case ShmGroup::kMinU32: return "all-reduce(u32 min)";
    case ShmGroup::kSumMin: return "all-reduce(u64 sum + u32 min)";
    case ShmGroup::kAllGather: return "all-gather";
    default: return "?";
  }
}

using Clock = std::chrono::steady_clock;

// Spins briefly, then yields, then sleeps: a collective partner is usually a few µs behind,
// but a rank in a long host phase (a chain's walk) may be many ms behind.
struct Backoff {
  uint32_t k = 0;
  void pause() {
    if (k < 256) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    } else if (k < 1024) {
      sched_yield();
    } else {
      usleep(20);
    }
    ++k;
  }
};

}  // namespace

int ShmGroup::open(const char* name, int world, int rank, uint32_t timeout_ms, uint64_t slot_bytes, ShmGroup** out,
                   std::string* err) {
  char buf[512];
  *out = nullptr;
  if (!name || name[0] != '/' || std::strchr(name + 1, '/')) {
    *err = "shm name must be '/<name>' without further slashes";
    return PZ_EINVAL;
  }
  if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world) {
    snprintf(buf, sizeof buf, "rank %d of world %d (at most %d)", rank, world, kMaxWorld);
    *err = buf;
    return PZ_EINVAL;
  }
  slot_bytes = std::max<uint64_t>(4096, (slot_bytes + 4095) & ~uint64_t(4095));
  const auto t0 = Clock::now();
  const auto late = [&] { return Clock::now() - t0 > std::chrono::milliseconds(timeout_ms); };
  int fd = -1;
  size_t bytes = 0;
  if (rank == 0) {
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) {
      snprintf(buf, sizeof buf, "shm_open(%s) for rank 0: %s", name, strerror(errno));
      *err = buf;
      return PZ_EINVAL;
    }
    bytes = data_offset() + (size_t)world * slot_bytes;
    if (ftruncate(fd, (off_t)bytes) != 0) {
      snprintf(buf, sizeof buf, "ftruncate(%s, %zu): %s", name, bytes, strerror(errno));
      *err = buf;
      close(fd);
      shm_unlink(name);
      return PZ_EDEVICE;
    }
  } else {
    // rank 0 may not have created it yet; it is complete once its size covers every slot
    Backoff bo;
    for (;;) {
      fd = shm_open(name, O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size >= data_offset() + (size_t)world * slot_bytes) {
          bytes = (size_t)st.st_size;
          break;
        }
        close(fd);
        fd = -1;
      }
      if (late()) {
        snprintf(buf, sizeof buf, "rank %d: shm segment %s not created by rank 0 within %u ms", rank, name, timeout_ms);
        *err = buf;
        return PZ_EDEVICE;
      }
      bo.pause();
    }
  }
  void* base = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base == MAP_FAILED) {
    snprintf(buf, sizeof buf, "mmap(%s): %s", name, strerror(errno));
    *err = buf;
    if (rank == 0) shm_unlink(name);
    return PZ_EDEVICE;
  }
  Header* h = hdr(base);
  if (rank == 0) {
    new (h) Header();  // the segment is zero-filled; construct the atomics in place
    h->world = (uint32_t)world;
    h->slot_bytes = slot_bytes;
    h->magic.store(kMagic, std::memory_order_release);
  } else {
    Backoff bo;
    while (h->magic.load(std::memory_order_acquire) != kMagic) {
      if (late()) {
        snprintf(buf, sizeof buf, "rank %d: shm segment %s never initialised", rank, name);
        *err = buf;
        munmap(base, bytes);
        return PZ_EDEVICE;
      }
      bo.pause();
    }
    if (h->world != (uint32_t)world || h->slot_bytes != slot_bytes) {
      snprintf(buf, sizeof buf, "rank %d: segment %s has world %u / slot %llu, this rank asked for %d / %llu", rank,
               name, h->world, (unsigned long long)h->slot_bytes, world, (unsigned long long)slot_bytes);
      *err = buf;
      munmap(base, bytes);
      return PZ_EINVAL;
    }
  }
  h->r[rank].joined.store(1, std::memory_order_release);
  Backoff bo;
  for (int q = 0; q < world; ++q) {
    while (!h->r[q].joined.load(std::memory_order_acquire)) {
      if (late() || h->aborted.load(std::memory_order_relaxed)) {
        snprintf(buf, sizeof buf, "rank %d: rank %d did not join shm group %s within %u ms", rank, q, name,
                 timeout_ms);
        *err = buf;
        h->aborted.store(1 + rank, std::memory_order_relaxed);
        munmap(base, bytes);
        if (rank == 0) shm_unlink(name);
        return PZ_EDEVICE;
      }
      bo.pause();
    }
  }
  if (rank == 0) shm_unlink(name);  // every rank holds a mapping: the name is no longer needed
  ShmGroup* g = new ShmGroup();
  g->world_ = world;
  g->rank_ = rank;
  g->timeout_ms_ = timeout_ms;
  g->slot_bytes_ = slot_bytes;
  g->base_ = base;
  g->map_bytes_ = bytes;
  *out = g;
  return PZ_OK;
}

ShmGroup::~ShmGroup() {
  if (base_) munmap(base_, map_bytes_);
}

void ShmGroup::abort_group() {
  int32_t zero = 0;
  hdr(base_)->aborted.compare_exchange_strong(zero, 1 + rank_, std::memory_order_relaxed);
}

int ShmGroup::wait_all(bool posted, uint64_t s, std::string* err) {
  Header* h = hdr(base_);
  const auto t0 = Clock::now();
  Backoff bo;
  for (int q = 0; q < world_; ++q) {
    const std::atomic<uint64_t>& w = posted ? h->r[q].posted : h->r[q].consumed;
    while (w.load(std::memory_order_acquire) < s) {
      const int32_t ab = h->aborted.load(std::memory_order_relaxed);
      const bool late = (bo.k & 63) == 63 && Clock::now() - t0 > std::chrono::milliseconds(timeout_ms_);
      if (ab || late) {
        char buf[384];
        if (ab)
          snprintf(buf, sizeof buf, "shm collective round %llu: rank %d aborted the group (see its error)",
                   (unsigned long long)s, ab - 1);
        else
          snprintf(buf, sizeof buf,
                   "shm collective round %llu: rank %d waited %u ms for rank %d to %s it (rank %d is at round %llu): "
                   "the ranks' collective sequences diverged or that rank stopped",
                   (unsigned long long)s, rank_, timeout_ms_, q, posted ? "post" : "consume", q,
                   (unsigned long long)w.load(std::memory_order_relaxed));
        *err = buf;
        abort_group();
        return PZ_EDEVICE;
      }
      bo.pause();
    }
  }
  return PZ_OK;
}

template <typename F>
int ShmGroup::round(const void* mine, size_t bytes, const Desc& d, F&& combine, std::string* err) {
  Header* h = hdr(base_);
  const uint64_t s = ++seq_;
  if (int rc = wait_all(false, s - 1, err)) return rc;  // my slot is free
  if (bytes) std::memcpy(slot(base_, slot_bytes_, rank_), mine, bytes);
  RankCtl& me = h->r[rank_];
  me.op = d.op;
  me.a = d.a;
  me.b = d.b;
  me.chunk = d.chunk;
  me.posted.store(s, std::memory_order_release);
  if (int rc = wait_all(true, s, err)) return rc;
  for (int q = 0; q < world_; ++q) {
    const RankCtl& o = h->r[q];
    if (o.op != d.op || o.a != d.a || o.b != d.b || o.chunk != d.chunk) {
      char buf[384];
      snprintf(buf, sizeof buf,
               "collective sequences diverged at shm round %llu: rank %d issued %s(%llu, %llu) chunk %llu, rank %d "
               "issued %s(%llu, %llu) chunk %llu",
               (unsigned long long)s, rank_, op_name(d.op), (unsigned long long)d.a, (unsigned long long)d.b,
               (unsigned long long)d.chunk, q, op_name(o.op), (unsigned long long)o.a, (unsigned long long)o.b,
               (unsigned long long)o.chunk);
      *err = buf;
      abort_group();
      return PZ_EINVAL;
    }
  }
  const uint8_t* slots[kMaxWorld];
  for (int q = 0; q < world_; ++q) slots[q] = slot(base_, slot_bytes_, q);
  combine(slots);
  me.consumed.store(s, std::memory_order_release);
  return PZ_OK;
}

int ShmGroup::sum_u64(uint64_t* buf, size_t n, std::string* err) {
  const size_t per = slot_bytes_ / 8;
  uint64_t k = 0;
  for (size_t off = 0; off < n || (n == 0 && k == 0); off += per, ++k) {
    const size_t c = std::min(per, n - off);
    int rc = round(buf + off, c * 8, Desc{kSumU64, n, 0, k}, [&](const uint8_t* const* sl) {
      for (size_t i = 0; i < c; ++i) {
        uint64_t v = 0;
        for (int q = 0; q < world_; ++q) v += reinterpret_cast<const uint64_t*>(sl[q])[i];  // mod 2^64, any order
        buf[off + i] = v;
      }
    }, err);
    if (rc) return rc;
    if (n == 0) break;
  }
  return PZ_OK;
}

int ShmGroup::min_u32(uint32_t* buf, size_t n, std::string* err) {
  const size_t per = slot_bytes_ / 4;
  uint64_t k = 0;
  for (size_t off = 0; off < n || (n == 0 && k == 0); off += per, ++k) {
    const size_t c = std::min(per, n - off);
    int rc = round(buf + off, c * 4, Desc{kMinU32, n, 0, k}, [&](const uint8_t* const* sl) {
      for (size_t i = 0; i < c; ++i) {
        uint32_t v = UINT32_MAX;
        for (int q = 0; q < world_; ++q) v = std::min(v, reinterpret_cast<const uint32_t*>(sl[q])[i]);
        buf[off + i] = v;
      }
    }, err);
    if (rc) return rc;
    if (n == 0) break;
  }
  return PZ_OK;
}

int ShmGroup::sum_min(uint64_t* s, size_t ns, uint32_t* m, size_t nm, std::string* err) {
  // the sum's chunks, then the minimum's, every round carrying both counts
  const size_t per64 = slot_bytes_ / 8, per32 = slot_bytes_ / 4;
  uint64_t k = 0;
  for (size_t off = 0; off < ns; off += per64, ++k) {
    const size_t c = std::min(per64, ns - off);
    int rc = round(s + off, c * 8, Desc{kSumMin, ns, nm, k}, [&](const uint8_t* const* sl) {
      for (size_t i = 0; i < c; ++i) {
        uint64_t v = 0;
        for (int q = 0; q < world_; ++q) v += reinterpret_cast<const uint64_t*>(sl[q])[i];
        s[off + i] = v;
      }
    }, err);
    if (rc) return rc;
  }
  for (size_t off = 0; off < nm; off += per32, ++k) {
    const size_t c = std::min(per32, nm - off);
    int rc = round(m + off, c * 4, Desc{kSumMin, ns, nm, k}, [&](const uint8_t* const* sl) {
      for (size_t i = 0; i < c; ++i) {
        uint32_t v = UINT32_MAX;
        for (int q = 0; q < world_; ++q) v = std::min(v, reinterpret_cast<const uint32_t*>(sl[q])[i]);
        m[off + i] = v;
      }
    }, err);
    if (rc) return rc;
  }
  if (ns == 0 && nm == 0) return round(nullptr, 0, Desc{kSumMin, 0, 0, 0}, [](const uint8_t* const*) {}, err);
  return PZ_OK;
}

int ShmGroup::allgather(const void* send, void* recv, size_t bytes, std::string* err) {
  const uint8_t* src = static_cast<const uint8_t*>(send);
  uint8_t* dst = static_cast<uint8_t*>(recv);
  uint64_t k = 0;
  for (size_t off = 0; off < bytes || (bytes == 0 && k == 0); off += slot_bytes_, ++k) {
    const size_t c = std::min<size_t>(slot_bytes_, bytes - off);
    int rc = round(src + off, c, Desc{kAllGather, bytes, 0, k}, [&](const uint8_t* const* sl) {
      for (int q = 0; q < world_; ++q) std::memcpy(dst + (size_t)q * bytes + off, sl[q], c);
    }, err);
    if (rc) return rc;
    if (bytes == 0) break;
  }
  return PZ_OK;
}

}  // namespace pz

// ---- host-only test entry points (the A/B library; no device involved; tests/test_shm_group.py)
#ifdef PZ_AB_BUILD
using pz::ShmGroup;

extern "C" {

static thread_local std::string g_shm_err;

const char* pz_debug_shm_error(void) { return g_shm_err.c_str(); }

int pz_debug_shm_open(const char* name, int world, int rank, uint32_t timeout_ms, uint64_t slot_bytes, void** out) {
  ShmGroup* g = nullptr;
  int rc = ShmGroup::open(name, world, rank, timeout_ms, slot_bytes, &g, &g_shm_err);
  *out = g;
  return rc;
}

int pz_debug_shm_sum_u64(void* g, uint64_t* buf, uint64_t n) {
  return static_cast<ShmGroup*>(g)->sum_u64(buf, n, &g_shm_err);
}

int pz_debug_shm_min_u32(void* g, uint32_t* buf, uint64_t n) {
  return static_cast<ShmGroup*>(g)->min_u32(buf, n, &g_shm_err);
}

int pz_debug_shm_sum_min(void* g, uint64_t* s, uint64_t ns, uint32_t* m, uint64_t nm) {
  return static_cast<ShmGroup*>(g)->sum_min(s, ns, m, nm, &g_shm_err);
}

int pz_debug_shm_allgather(void* g, const void* send, void* recv, uint64_t bytes) {
  return static_cast<ShmGroup*>(g)->allgather(send, recv, bytes, &g_shm_err);
}

void pz_debug_shm_close(void* g) { delete static_cast<ShmGroup*>(g); }

}  // extern "C"
#endif  // PZ_AB_BUILD
