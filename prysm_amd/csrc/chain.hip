// Native block pipeline: the reference's ChainService.blockProcessing (beacon-chain/
// blockchain/service.go:229-363) + updateHead (:170-227) over BeaconChain (core.go), fed with
// serialized blocks, with every data-parallel step on the GPU.
//
// The walk over the blocks is sequential host code (scalar checks, hash-map lookups, small
// copies); the device work is batched per call:
//   * block / attestation Hash / attestation Key digests: one CSR BLAKE2b launch, before the
//     walk (blocks are immutable inputs);
//   * processAttestation message digests (core.go:277-290, 64 bytes): one launch, after it;
//   * calculateBlockVoteCache (core.go:300-345): tally items queued during the walk, run by
//     the vote kernel on the HBM-resident cache before every stateRecalc and at the end;
//   * stateRecalc's processCrosslinks + CalculateRewards + next-cycle balance: one epoch
//     instance (epoch.hip) on the HBM-resident validator arrays.
// Reference semantics kept on purpose (each changes hashed bytes) are listed in DESIGN.md §7;
// oracle/replay.py restates the same pipeline for the parity tests.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <ctime>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <pthread.h>
#include <condition_variable>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "blake2b_kernels.h"
#include "comm.h"
#include "serial_hash.h"
#include "epoch.h"
#include "runtime.h"
#include "votes.h"
#include "wire.h"

namespace pz {
namespace chain {

constexpr uint64_t kCycle = PZ_CYCLE_LENGTH;

struct H32 {
  uint8_t b[32];
  bool operator==(const H32& o) const { return std::memcmp(b, o.b, 32) == 0; }
};
struct H32Hash {
  size_t operator()(const H32& h) const {
    uint64_t x;
    std::memcpy(&x, h.b, 8);
    return (size_t)(x ^ (x >> 29));
  }
};
static const H32 kZero = {};

// Open-addressing table keyed by 32-byte hashes: linear probing, power-of-two capacity, load
// at most 1/2.  The probed array holds 16-B slots {tag, value, used}: a 64-bit tag of the key
// rejects a mismatch without touching the key, which sits in a parallel array.  The walk
// inserts every block hash (the saved set) and every logged hash (the vote-cache slots);
// node-based std::unordered_* paid a malloc per insert and a pointer chase per probe (~8 % of
// the walk), 40-B inline entries a cache miss per probe (tools/walk_sampler.py, profiles/r03).
template <typename V>
struct H32Table {
  struct Slot {
    uint64_t tag;
    V v;
    uint8_t used;
  };
  std::vector<Slot> t;
  std::vector<H32> keys;
  size_t n = 0, mask = 0;
  // digests are uniform, but BytesToHash of a short oblique hash is zero-padded on the left:
  // both ends go into the tag, and the slot index takes its high bits after a multiply
  static uint64_t tag_of(const H32& h) {
    uint64_t a, b;
    std::memcpy(&a, h.b, 8);
    std::memcpy(&b, h.b + 24, 8);
    return a ^ (b * 0x9E3779B97F4A7C15ull);
  }
  size_t index(uint64_t tag) const { return (size_t)((tag * 0xD6E8FEB86659FD93ull) >> 32) & mask; }
  size_t size() const { return n; }
  void clear() {
    t.clear();
    keys.clear();
    n = mask = 0;
  }
  void grow(size_t cap = 0) {
    std::vector<Slot> old;
    std::vector<H32> oldk;
    old.swap(t);
    oldk.swap(keys);
    if (!cap) cap = old.empty() ? 1024 : 2 * old.size();
    t.assign(cap, Slot{0, V{}, 0});
    keys.resize(cap);
    mask = cap - 1;
    for (size_t j = 0; j < old.size(); ++j)
      if (old[j].used) {
        size_t i = index(old[j].tag);
        while (t[i].used) i = (i + 1) & mask;
        t[i] = old[j];
        keys[i] = oldk[j];
      }
  }
  void reserve(size_t m) {
    size_t cap = t.empty() ? 1024 : t.size();
    while (2 * m > cap) cap *= 2;
    if (cap > t.size()) grow(cap);  // one rehash
  }
  const V* find(const H32& k) const {
    if (!n) return nullptr;
    const uint64_t tg = tag_of(k);
    for (size_t i = index(tg);; i = (i + 1) & mask) {
      if (!t[i].used) return nullptr;
      if (t[i].tag == tg && keys[i] == k) return &t[i].v;
    }
  }
  bool count(const H32& k) const { return find(k) != nullptr; }
  // inserts (k, v) unless k is present; returns the stored value
  V insert(const H32& k, V v) {
    if (2 * (n + 1) > t.size()) grow();
    const uint64_t tg = tag_of(k);
    size_t i = index(tg);
    for (; t[i].used; i = (i + 1) & mask)
      if (t[i].tag == tg && keys[i] == k) return t[i].v;
    t[i] = Slot{tg, v, 1};
    keys[i] = k;
    ++n;
    return v;
  }
};

// go-ethereum common.BytesToHash: last 32 bytes, right-aligned.
static H32 bytes_to_hash(const uint8_t* p, size_t n) {
  H32 h;
  if (n >= 32) {
    std::memcpy(h.b, p + n - 32, 32);
    return h;
  }
  h = kZero;
  if (n > 32) {
    p += n - 32;
    n = 32;
  }
  if (n) std::memcpy(h.b + 32 - n, p, n);
  return h;
}
// `var h [32]byte; copy(h[:], b)`: left-aligned, truncated.
static H32 copy32(const uint8_t* p, size_t n) {
  H32 h = kZero;
  if (n) std::memcpy(h.b, p, n < 32 ? n : 32);
  return h;
}

// ---- proto3 ---------------------------------------------------------------------------------
static void put_varint(std::string& o, uint64_t x) {
  while (x >= 0x80) {
    o.push_back((char)((x & 0x7f) | 0x80));
    x >>= 7;
  }
  o.push_back((char)x);
}
static void put_u(std::string& o, uint32_t f, uint64_t v) {
  if (v) {
    put_varint(o, (uint64_t)f << 3);
    put_varint(o, v);
  }
}
static void put_b(std::string& o, uint32_t f, const uint8_t* p, size_t n) {
  if (n) {
    put_varint(o, ((uint64_t)f << 3) | 2);
    put_varint(o, n);
    o.append((const char*)p, n);
  }
}
static void put_msg(std::string& o, uint32_t f, const uint8_t* p, size_t n) {
  put_varint(o, ((uint64_t)f << 3) | 2);
  put_varint(o, n);
  o.append((const char*)p, n);
}

// Streaming proto3 reader that also checks canonical form: the reference hashes
// proto.Marshal of the DECODED message, so the engine accepts exactly the inputs that equal
// the re-encoding of their own decoding.  Instead of re-encoding, every rule Marshal applies
// is checked while reading: minimal varints (keys, values, lengths), ascending field numbers
// (a repeated field only repeats in a run), zero scalars and empty singular bytes omitted,
// a packed repeated field never empty, and no unknown fields.
struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  bool more() const { return ok && p < e; }
  // a minimal varint (a 10-byte one must end in 0x01: only bit 63 left)
  uint64_t varint() {
    uint64_t x = 0;
    for (int i = 0, s = 0; i < 10; ++i, s += 7) {
      if (p >= e) { ok = false; return 0; }
      const uint8_t b = *p++;
      x |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) {
        if ((i > 0 && b == 0) || (i == 9 && b != 1)) ok = false;
        return x;
      }
    }
    ok = false;
    return 0;
  }
  bool span(const uint8_t** q, size_t* n) {
    const uint64_t len = varint();
    if (!ok || len > (uint64_t)(e - p)) { ok = false; return false; }
    *q = p;
    *n = (size_t)len;
    p += len;
    return true;
  }
  void skip(uint32_t wt) {  // (only for counting; canonical form is checked by the parsers)
    const uint8_t* q;
    size_t n;
    if (wt == 0) varint();
    else if (wt == 2) span(&q, &n);
    else if (wt == 1 && e - p >= 8) p += 8;
    else if (wt == 5 && e - p >= 4) p += 4;
    else ok = false;
  }
  // the next key: field f with wire type wt, after field `prev`; `rep` = f may repeat
  bool key(uint32_t prev, uint32_t* f, uint32_t* wt, uint32_t nfields, const uint32_t* types, uint32_t rep_mask) {
    const uint64_t k = varint();
    *f = (uint32_t)(k >> 3);
    *wt = (uint32_t)(k & 7);
    if (!ok || *f == 0 || *f > nfields || types[*f] != *wt) return ok = false;
    if (*f < prev || (*f == prev && !((rep_mask >> *f) & 1))) return ok = false;
    return true;
  }
};

// The oblique parent hashes of one attestation: (offset, length) pairs into its encoding,
// held in the call arena's pool.
struct OblSpan {
  const std::pair<uint32_t, uint32_t>* p = nullptr;
  uint32_t n = 0;
  const std::pair<uint32_t, uint32_t>* begin() const { return p; }
  const std::pair<uint32_t, uint32_t>* end() const { return p + n; }
  size_t size() const { return n; }
};

// One AttestationRecord (messages.proto:110-119): its canonical encoding is a span of the call
// arena's copy of the input blocks.  Records are referred to by plain pointers; the Engine
// keeps every arena that a live state's pending attestations point into (keep_arenas).
struct Att {
  const uint8_t* base = nullptr;  // the encoding
  uint32_t len = 0;
  uint64_t slot = 0, shard = 0, jslot = 0;
  uint32_t sbh_off = 0, sbh_len = 0, bf_off = 0, bf_len = 0;
  uint32_t obl_first = 0;  // its first pair in the arena pool (OblSpan bound after the parse)
  OblSpan obl;
  const uint8_t* at(uint32_t off) const { return base + off; }
};
using AttP = const Att*;

// A block's attestations: a run of the arena's record pointers.
struct AttSpan {
  const AttP* p = nullptr;
  uint32_t n = 0;
  const AttP* begin() const { return p; }
  const AttP* end() const { return p + n; }
  size_t size() const { return n; }
  AttP operator[](size_t i) const { return p[i]; }
};

// One pz_chain_process_blocks call's input: a copy of its serialized blocks and every
// attestation record parsed from them, allocated once (per-record allocations made the parse
// allocator-bound).  The Engine keeps it while a live state's pending attestations point in.
// Record storage allocated without constructing anything: the parse threads construct their own
// ranges (a value-initialised std::vector<Att> zeroed and faulted in 4.4 MB per 10,000 blocks
// on the calling thread before any parse thread started).
struct AttStore {
  Att* p = nullptr;
  size_t n = 0;
  AttStore() = default;
  AttStore(const AttStore&) = delete;
  AttStore& operator=(const AttStore&) = delete;
  ~AttStore() { std::free(p); }
  void alloc(size_t count) {  // (Att is trivially destructible: nothing to destroy first)
    std::free(p);
    p = nullptr;
    n = count;
    if (count && !(p = static_cast<Att*>(std::malloc(count * sizeof(Att))))) throw std::bad_alloc();
  }
  Att* data() const { return p; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  Att& operator[](size_t i) const { return p[i]; }
};
static_assert(std::is_trivially_destructible<Att>::value && std::is_trivially_copyable<Att>::value,
              "AttStore places records without destructors");

struct CallArena {
  using Pool = std::vector<std::pair<uint32_t, uint32_t>>;
  uint8_t* bytes = nullptr;  // (not zero-filled) the Engine's pinned arena, or `own`
  std::unique_ptr<uint8_t[]> own;
  AttStore atts;  // sized to the exact count: block i's records at [first[i], first[i+1])
  std::vector<AttP> ptrs;  // &atts[j]: each Block's AttSpan is a run of it
  std::vector<uint64_t> first;  // per block, its first record (a prefix of the per-block counts)
  // one pool per range parsed by one thread, each reserved to a bound (an element takes >= 2
  // bytes): Att::obl points into it
  std::vector<Pool> obl;
};

// messages.pb.go:889-896: 1-3 varint, 4-6 bytes, 7 repeated bytes, 8 packed varints
static bool parse_att(const uint8_t* p, size_t n, Att* a, CallArena::Pool& pool) {
  static const uint32_t kTypes[9] = {9, 0, 0, 0, 2, 2, 2, 2, 2};
  a->base = p;
  a->len = (uint32_t)n;
  a->obl_first = (uint32_t)pool.size();
  const uint8_t* base = p;
  Reader r{base, base + n};
  uint32_t prev = 0, f, wt;
  const uint8_t* q;
  size_t len;
  while (r.more()) {
    if (!r.key(prev, &f, &wt, 8, kTypes, 1u << 7)) return false;
    prev = f;
    if (f <= 3) {
      const uint64_t v = r.varint();
      if (!v) return false;  // a zero scalar is omitted by Marshal
      (f == 1 ? a->slot : f == 2 ? a->shard : a->jslot) = v;
    } else if (!r.span(&q, &len)) {
      return false;
    } else if (f <= 6) {
      if (!len) return false;  // an empty singular bytes field is omitted
      if (f == 5) { a->sbh_off = (uint32_t)(q - base); a->sbh_len = (uint32_t)len; }
      if (f == 6) { a->bf_off = (uint32_t)(q - base); a->bf_len = (uint32_t)len; }
    } else if (f == 7) {
      if (pool.size() == pool.capacity()) return false;  // (the bound makes this unreachable)
      pool.push_back({(uint32_t)(q - base), (uint32_t)len});
      ++a->obl.n;
    } else {  // f == 8: packed, never empty
      if (!len) return false;
      Reader s{q, q + len};
      while (s.more()) s.varint();
      if (!s.ok) return false;
    }
  }
  a->obl.p = pool.data() + a->obl_first;  // the pool never reallocates (reserved to a bound)
  return r.ok;
}

struct Block {
  const uint8_t* data;
  size_t len;
  uint64_t slot = 0;
  H32 parent = kZero;  // Block.ParentHash(): copy into [32]byte (types/block.go:80-84)
  AttSpan atts;
};

// messages.pb.go:224-232: 1 bytes, 2 varint, 3-6 bytes, 7 Timestamp, 8 repeated records
// Block i's records go to ar->atts[first[i], first[i+1]).
static bool parse_block(const uint8_t* p, size_t n, Block* b, CallArena* ar, uint64_t i, CallArena::Pool& pool) {
  static const uint32_t kTypes[9] = {9, 2, 0, 2, 2, 2, 2, 2, 2};
  static const uint32_t kTsTypes[3] = {9, 0, 0};
  b->data = p;
  b->len = n;
  const uint64_t a0 = ar->first[i], a1 = ar->first[i + 1];
  b->atts.p = ar->ptrs.data() + a0;
  b->atts.n = 0;
  Reader r{p, p + n};
  uint32_t prev = 0, f, wt;
  const uint8_t* q;
  size_t len;
  while (r.more()) {
    if (!r.key(prev, &f, &wt, 8, kTypes, 1u << 8)) return false;
    prev = f;
    if (f == 2) {
      if (!(b->slot = r.varint())) return false;
    } else if (!r.span(&q, &len)) {
      return false;
    } else if (f == 1 || f <= 6) {
      if (!len) return false;
      if (f == 1) b->parent = copy32(q, len);
    } else if (f == 7) {  // Timestamp {int64 seconds = 1; int32 nanos = 2}; may be empty
      Reader t{q, q + len};
      uint32_t tp = 0, tf, twt;
      while (t.more()) {
        if (!t.key(tp, &tf, &twt, 2, kTsTypes, 0)) return false;
        tp = tf;
        const uint64_t v = t.varint();
        if (!v) return false;
        // int32: Marshal sign-extends the decoded 32-bit value
        if (tf == 2 && v != (uint64_t)(int64_t)(int32_t)(uint32_t)v) return false;
      }
      if (!t.ok) return false;
    } else {  // f == 8
      if (a0 + b->atts.n >= a1) return false;  // more records than counted (unreachable)
      Att* a = new (&ar->atts[a0 + b->atts.n]) Att();  // (constructed here, on the parsing thread)
      if (!parse_att(q, len, a, pool)) return false;
      ar->ptrs[a0 + b->atts.n] = a;
      ++b->atts.n;
    }
  }
  return r.ok && b->atts.n == a1 - a0;
}

// ---- chain state ----------------------------------------------------------------------------
struct Crosslink {
  uint64_t dynasty = 0, slot = 0;
  std::string hash;
};

struct AState {               // types.ActiveState
  std::vector<AttP> pending;  // PendingAttestations
  // RecentBlockHashes (normalised) as hash-log ids: Engine::trail[tail - len, tail).  The
  // states of one chain push onto the trail's end in turn, so a window is a range of it, not a
  // copy per state (push_recent re-appends a window that is not at the end).
  uint64_t tail = 0;
  uint32_t len = 0;
  bool recent_raw_empty = false;  // genesis: every entry is a zero-length byte slice
  bool cache_nil = false;     // the shared vote-cache map, or nil (SetBlockVoteCache(nil))
};
using AP = std::shared_ptr<AState>;

struct CState {  // types.CrystallizedState (validators and committees live in the Engine)
  uint64_t lsr = 0, streak = 0, jslot = 0, fslot = 0, dynasty = 0, start_shard = 0, tdep = 0, seed_reset = 0;
  std::string seed;  // DynastySeed (empty at genesis; stateRecalc does not carry it)
  std::shared_ptr<std::vector<Crosslink>> xl;  // shared with the next state (mutated in place)
};
using CP = std::shared_ptr<CState>;

template <typename T>
struct DevArr {
  T* p = nullptr;
  size_t n = 0;
  int alloc(size_t count) {
    if (count <= n && p) return PZ_OK;
    T* q = nullptr;
    hipError_t e = hipMalloc((void**)&q, (count ? count : 1) * sizeof(T) + 256);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc");
    if (p) (void)hipFree(p);
    p = q;
    n = count;
    return PZ_OK;
  }
  ~DevArr() {
    if (p) (void)hipFree(p);
  }
};

// Pinned host memory is slow to get (its pages are locked and mapped for the device: ~ms per
// 10 MB), so freed PinBufs go to a process-wide pool that later chains of the process reuse
// (sizes rounded up to powers of two, at most kPinPoolBytes kept).  The pool is never
// destroyed: it outlives static destructors that may run after the HIP runtime's.
constexpr size_t kPinPoolBytes = size_t(1) << 30;
struct PinPool {
  std::mutex mu;
  std::multimap<size_t, void*> free;
  size_t bytes = 0;
};
static PinPool& pin_pool() {
  static PinPool* p = new PinPool();
  return *p;
}

// Grow-only pinned host buffer, for asynchronous-capable H2D / D2H and device-mapped reads.
struct PinBuf {
  uint8_t* p = nullptr;
  size_t n = 0;
  // its device address for each device that reads it, looked up once per device (a runtime
  // call per use showed in the walk).  hipHostMalloc memory is mapped into every device's
  // address space, but the device address is asked of the device that will use it: a chain
  // over several devices (pz_chain_new_comm) reads the tally arena from every rank's device.
  std::vector<std::pair<int, void*>> d;
  int reserve(size_t bytes) {
    if (bytes <= n && p) return PZ_OK;
    release();
    size_t want = 4096;
    while (want < bytes) want *= 2;
    PinPool& pool = pin_pool();
    {
      std::lock_guard<std::mutex> lk(pool.mu);
      auto it = pool.free.lower_bound(want);
      if (it != pool.free.end() && it->first <= 4 * want) {
        p = static_cast<uint8_t*>(it->second);
        n = it->first;
        pool.bytes -= it->first;
        pool.free.erase(it);
        return PZ_OK;
      }
    }
    hipError_t e = hipHostMalloc((void**)&p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      p = nullptr;
      return hip_fail(e, "hipHostMalloc");
    }
    n = want;
    return PZ_OK;
  }
  // (the calling thread's current device must be `device`: hipHostGetDevicePointer answers
  // for the current device)
  int dev(int device, void** out) {
    for (const auto& x : d)
      if (x.first == device) {
        *out = x.second;
        return PZ_OK;
      }
    void* q = nullptr;
    hipError_t e = hipHostGetDevicePointer(&q, p, 0);
    if (e != hipSuccess) return hip_fail(e, "hipHostGetDevicePointer");
    d.emplace_back(device, q);
    *out = q;
    return PZ_OK;
  }
  void release() {
    if (!p) return;
    PinPool& pool = pin_pool();
    {
      std::lock_guard<std::mutex> lk(pool.mu);
      if (pool.bytes + n <= kPinPoolBytes) {
        pool.free.emplace(n, p);
        pool.bytes += n;
        p = nullptr;
      }
    }
    if (p) (void)hipHostFree(p);
    p = nullptr;
    d.clear();
    n = 0;
  }
  ~PinBuf() { release(); }
};

// Append-only pinned array for data that asynchronous H2D copies read while the walk keeps
// appending: growing copies into a new buffer and keeps the old ones alive until reset(), which
// the caller makes only once no copy is in flight.
template <typename T>
struct PinVec {
  std::vector<std::unique_ptr<PinBuf>> bufs;  // the last one is current
  size_t n = 0;
  T* data() const { return bufs.empty() ? nullptr : reinterpret_cast<T*>(bufs.back()->p); }
  // the current buffer's address on `device` (the calling thread's current device), or null
  const T* dev(int device) const {
    if (bufs.empty()) return nullptr;
    void* q = nullptr;
    if (int rc = bufs.back()->dev(device, &q)) throw rc;
    return static_cast<const T*>(q);
  }
  size_t cap() const { return bufs.empty() ? 0 : bufs.back()->n / sizeof(T); }
  void reserve(size_t c) {
    if (c <= cap()) return;
    auto nb = std::make_unique<PinBuf>();
    if (int rc = nb->reserve(c * sizeof(T))) throw rc;
    if (n) std::memcpy(nb->p, bufs.back()->p, n * sizeof(T));
    bufs.push_back(std::move(nb));
  }
  T* grow(size_t k) {  // k more elements at the end
    if (n + k > cap()) reserve(std::max(2 * cap(), n + k));
    T* p = data() + n;
    n += k;
    return p;
  }
  void trim() {  // drop the outgrown buffers (no copy may still read them)
    if (bufs.size() > 1) bufs.erase(bufs.begin(), bufs.end() - 1);
  }
  void reset() {
    n = 0;
    trim();
  }
  // the std::vector subset the hash log and the trail use
  size_t size() const { return n; }
  size_t capacity() const { return cap(); }
  T& operator[](size_t i) { return data()[i]; }
  const T& operator[](size_t i) const { return data()[i]; }
  void push_back(const T& x) { *grow(1) = x; }
  void resize(size_t k) {
    if (k > n) grow(k - n);
    else n = k;
  }
  void assign(size_t k, const T& x) {
    n = 0;
    T* p = grow(k);
    for (size_t i = 0; i < k; ++i) p[i] = x;
  }
};

[[maybe_unused]] constexpr uint64_t kVoteTraceFlushes = 256, kVoteTraceWaves = 512;  // (A/B: PZ_VOTE_TRACE)

// The walk's per-call switches (read_knobs), set once per pz_chain_process_blocks call: the
// product's choices plus pz_chain_options; the A/B library (make ab, -DPZ_AB_BUILD) also reads the
// measured-and-dropped forms from the environment there.
struct Knobs {
  int vote_path = 2;            // (A/B: PZ_VOTE_PATH; VotePath: 0 segments, 1 packed, 2 direct)
  bool vote_groups = true;      // pz_chain_options.tally_forms bit 0: the per-attestation tally
  bool vote_trace = false;      // (A/B: PZ_VOTE_TRACE, tools/vote_trace.py)
  bool epoch_pack_direct = false;  // (A/B: PZ_EPOCH_PACK=direct)
  bool epoch_prep_after = true;    // (A/B: PZ_EPOCH_PREP=merged: false)
};

// A recent window's parent ids as a run (votes.h VoteRec) over its positions [0, nw): shared by
// every attestation that signs the same window (trail[wstart, wstart + nw) at generation gen).
struct WindowRun {
  uint64_t wstart = ~0ull, nw = 0, gen = ~0ull;
  uint64_t step = 0, absent = 0;
  uint32_t s0 = UINT32_MAX, prev = 0;
  bool run = true;
};

enum ProfSlot {
  kProfParse, kProfHash1, kProfCheck, kProfQueue, kProfFlush, kProfRecalc, kProfMsgHash, kProfWalk, kProfProcess,
  kProfCount, kProfFlushWait, kProfMsgSend, kProfMsgLog, kProfMsgWait,
  kProfTotalsWait,    // the walk waiting for a transition's justification totals (inside state_recalc)
  kProfPollFallback,  // a count, not seconds: sequence-word polls that fell back to the event wait
  kProfIdRows,        // a count: queued attestations whose parent ids are no run (an explicit id row)
  kProfSlots
};

// Queued attestations that force a tally flush before the next stateRecalc.  Flushing more
// often overlaps the tally with the walk but pays ~20 us of host launch work per flush:
// every 16 / 64 / 256 attestations gave 57k / 86k / 97k blocks/s against 102k for
// flushing only at the transitions (10,000 blocks, 65,536 validators).
constexpr size_t kFlushAtts = 1 << 16;

// The pipelined walk's producer runs at most kRing chunks of kChunk blocks ahead (Feeder).
constexpr uint64_t kChunk = 512;
constexpr int kRing = 4;

// Staging of one digest batch (pinned host buffers and their device copies).
struct DigestBufs {
  PinBuf msgs, offs, dig;
  DevArr<uint8_t> d_in, d_out;
  DevArr<uint64_t> d_offs;
};

// One local rank's device state.  An unsharded chain has one rank holding every validator;
// a chain over a pz_comm (pz_chain_new_comm) gives each rank the
// 64-aligned validator range [lo, hi): its balances, its columns of every vote-cache voter
// bitmap and its partial VoteTotalDeposit sums, and its part of every epoch.
// Device buffers a growth replaced: not freed at the growth (a hipFree waits for the whole
// device, and the copies out of the old buffer are still queued) but at the end of the
// pz_chain_process_blocks call, once its streams have drained (release_retired), so a long-lived
// chain holds no dead generations between calls.
struct Retired {
  std::vector<void*> p;
  void keep(void* x) {
    if (x) p.push_back(x);
  }
  void release() {
    for (void* x : p) (void)hipFree(x);
    p.clear();
  }
  ~Retired() { release(); }
};

struct RankDev {
  int dev = 0, grank = 0;
  hipStream_t s = nullptr;
  uint64_t lo = 0, hi = 0, n = 0;
  // validators [lo, hi) (shared by every CrystallizedState, like the Go pointer slice)
  DevArr<uint64_t> balance, start, end;
  // field 11 of the CrystallizedState for this range, encoded on the device (wire.hip)
  DevArr<uint8_t> w_out;
  DevArr<uint64_t> w_scratch, w_total;
  // ShardAndCommitteesForSlots, replicated; and the members inside [lo, hi) with their
  // committee positions (the sharded epoch's crosslink partial sums)
  DevArr<uint32_t> committee, lcomm, lcpos;
  DevArr<uint64_t> coffs, lcoffs;
  // the vote cache, voter-major (votes.h VoteWordArgs): bm[w * n + v] holds this range's
  // validator v's votes for ids 64 w .. 64 w + 63; partial totals and present flags per id
  DevArr<uint64_t> bm;
  DevArr<uint64_t> totals;
  DevArr<uint8_t> present;
  DevArr<uint8_t> d_qpack;
  DevArr<uint64_t> d_err;      // sticky tally panic flag
  DevArr<uint32_t> v_ticket;   // the fused gather's arrival ticket (left zero)
  DevArr<uint64_t> v_trace;    // (PZ_VOTE_TRACE, tools/ only) per flush and wave, the tally's phase stamps
  // sharded (world > 1): the transition's one all-reduce buffer, [totals + panic flag (65) |
  // TotalDeposits slot (1) | the epoch's {scal, vote, total} partials], and this rank's
  // post-reward next-cycle partial waiting for the next all-reduce (sharded_reduce_enqueue)
  DevArr<uint64_t> xred, nbp;
  // epoch scratch: red = {scal[8], vote[natt], total[natt]} (one all-reduce when sharded)
  DevArr<uint64_t> e_red, e_mask;
  DevArr<uint32_t> e_blk, e_list, e_win;
  DevArr<uint8_t> e_pack;      // one H2D per transition: bitfields, offsets, committees, ... (sharded)
  DevArr<uint32_t> e_ticket;   // one rank: the reward pass's hand-off ticket (left zero)
  hipEvent_t q_ev = nullptr;   // this rank's copy of the pinned tally arena is done (staged path)
  hipEvent_t vq_ev[2] = {};    // this rank's last reader of Engine::vq[i] is done
  hipEvent_t ev_epoch = nullptr, ev_t64 = nullptr;
};

struct Engine {
  uint64_t nval = 0;
  int device = 0;
  hipStream_t s = nullptr;  // local rank 0's stream: hashing, the digest and message batches
  hipStream_t s2 = nullptr;  // local rank 0's second stream: the pipelined digest batches
  DigestBufs dbatch;         // the digest batch of an unpipelined call
  DigestBufs ring[kRing];    // the pipelined calls' digest batches, reused chunk after chunk
  hipEvent_t ring_ev[kRing] = {};
  // the batch path's digest batch runs on s2 in two parts: the block digests (the walk waits
  // for ev_dblk) and the attestations' Hash / Key (results only: collected after the walk)
  hipEvent_t ev_dblk = nullptr, ev_datt = nullptr;
  pz_comm* comm = nullptr;  // null: one device, every validator
  int world = 1;
  std::vector<RankDev> rk;
  std::mutex mu;
  bool poisoned = false;
  std::vector<uint64_t> h_balance, h_start, h_end;  // genesis / reloaded values (uploaded once)
  // the other ValidatorRecord fields, resident (on rank 0) only when a reloaded state has them
  // non-zero (reloading is unsharded)
  DevArr<uint64_t> pubkey, wshard, wa_offs, rc_offs;
  DevArr<uint8_t> wa, rc;
  bool has_pk = false, has_ws = false, has_wa = false, has_rc = false;
  uint64_t val_bytes = 0;  // total withdrawal_address + randao_commitment bytes
  // field 11 of the CrystallizedState, re-encoded only after rewards changed a balance
  std::string val_enc;
  bool val_enc_valid = false;
  // ShardAndCommitteesForSlots (immutable in this reference: stateRecalc copies it)
  std::vector<uint64_t> csize;
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> lookup;  // [array] -> (shard, committee id)
  std::string arrays_enc;  // field 12 of the CrystallizedState, every array
  // block vote cache (one map shared by every ActiveState)
  H32Table<uint32_t> slot_of;
  std::vector<H32> slot_hash;
  uint64_t cap = 0;
  // pending tally work: per queued attestation its committee's members, its bitfield and the
  // vote-cache ids of its 64 signed parent hashes (votes.h VoteWordArgs).  The walk writes the queue straight into pinned memory: two queues, the walk
  // filling one while a flush's kernels may still read the other (RankDev::vq_ev).
  struct VoteQueue {
    PinVec<VoteRec> rec;      // per attestation (votes.h VoteRec)
    PinVec<uint32_t> slots;   // the explicit 64-id rows (kVoteIdsRow records)
    PinVec<uint8_t> bits;     // the bitfield rows when they are not inline (bits_inline false)
    uint32_t chunks = 1;  // max ceil(k / 256) over the queue
    // the queue's attestations grouped by committee (votes.h VoteGroup), built as they queue;
    // `groupable` false once a record is not in the run form, a bitfield is not inline, or the
    // groups outnumber kVoteMaxGroups
    struct Group {
      uint32_t c = 0, k = 0;
      uint32_t idlo = UINT32_MAX, idhi = 0;  // the parents' id range (inclusive)
      std::vector<uint32_t> atts;
    };
    std::vector<Group> grp;
    std::vector<int32_t> gof;  // per committee: its group + 1, 0 for none
    bool groupable = true;
    PinVec<uint32_t> perm;     // the flushed groups' record indices (VoteWordArgs.perm)
    bool busy = false;
    size_t natt() const { return rec.size(); }
  } vq[2];
  int vq_cur = 0;
  // flushes run asynchronously to the walk: the queue is packed into a pinned arena and
  // copied with one H2D per rank; the arena is reused once every rank's copy is done
  PinBuf q_arena;
  bool q_arena_busy = false;
  uint64_t ncomm = 0;
  std::vector<uint64_t> h_coffs;  // the committees' first member offsets (host copy)
  uint32_t bf_stride = 4;         // the vote queue's bitfield row: >= every committee's bytes, x4
  uint64_t trail_gen = 0;         // bumped whenever the trail is rebuilt (WindowRun's key)
  WindowRun wrun;                 // the last recent window's parent-id run (queue_vote_cache)
  Retired retired;                // grown-out device buffers (freed with the chain)
  Knobs kn;                       // (read_knobs)
  pz_chain_options opt{};         // pz_chain_set_options (every field 0: the product's choices)
  uint64_t calls = 0;             // pz_chain_process_blocks calls that reached the walk
  // sharded: the last epoch's next-cycle balance is still a partial per rank (nbp), summed by
  // the next all-reduce (a transition's or the call's final flush), then set as nb_dst's
  // TotalDeposits
  bool nb_pending = false, nb_carried = false;
  CP nb_dst;
  uint64_t kmax = 0;              // the largest committee
  bool bits_inline = true;        // every committee <= kVoteInlineBits: the bitfields ride in the records
  bool ids_rows = false;          // (pz_chain_options.tally_forms bit 2) every attestation's ids in an explicit row
  PinBuf e_pin, e_pin_out;   // the epoch inputs' pinned staging; the results' pinned landing
  PinBuf tot_pin;            // the gathered justification totals (65 words; + a sequence word)
  uint64_t gather_seq = 0;   // the last sequence number the fused gather was asked to write
  bool gather_poll = false;  // the current transition's totals arrive with their sequence word
  hipEvent_t ev_totals = nullptr;  // the tally flush + the totals' D2H of a transition are done
  // The epoch of the last transition, enqueued but not yet collected: its results (the
  // crosslink records, the next state's TotalDeposits, a panic) are first needed at the next
  // transition or by the state bytes/roots, so the walk never waits for it.
  struct DeferredEpoch {
    bool live = false;
    std::vector<AttP> pending;  // the attestations it ran over (a winner's ShardBlockHash)
    std::shared_ptr<CState> src, dst;  // the state it read (xl mutated in place), the new state
    uint64_t block_slot = 0;
    uint64_t block_index = 0;  // the transition block's index in the call (named by a panic)
    size_t nrec = 0;
    uint64_t seq = 0;  // one rank: the results arrive in g.e_pin_out with this sequence word
  } deferred;
  uint64_t epoch_seq = 0;
  // whether every validator is active at dynasty aa_dyn (the validators' dynasties never change
  // in a chain: stateRecalc does not rotate the set), cached per dynasty value
  uint64_t aa_dyn = UINT64_MAX;
  bool aa = false;
  // hashing scratch (rank 0)
  PinBuf pin_msgs, pin_offs, pin_dig;  // pinned staging of the digest batch
  DevArr<uint8_t> h_in, h_out;
  DevArr<uint64_t> h_offs;
  // chain
  AP A;
  CP C;
  bool has_cand = false;
  uint64_t cand_slot = 0;
  AP cand_A;
  CP cand_C;
  // saved block hashes (blockchain.go's SaveBlock): a flag per vote-cache slot (every block
  // digest is logged with a slot), plus a table for the hashes a reloaded chain starts with
  std::vector<uint8_t> slot_saved;
  H32Table<uint8_t> saved;
  // the call arenas whose records a live state still holds (pending attestations)
  std::vector<std::shared_ptr<CallArena>> arenas;
  // append-only hash log: every block digest and oblique parent hash the walk meets gets an
  // id; RecentBlockHashes carry ids too, so signed parent hashes are id ranges (no hashing of
  // 32-byte keys per vote) and the processAttestation messages are assembled on the device
  // (hlog and trail are pinned: the message batches' H2D of their new entries is a DMA that
  // neither stages through a host copy nor blocks the walk)
  PinVec<H32> hlog;
  std::vector<uint32_t> id_slot;  // vote-cache slot of each id (resolved when it is logged)
  PinVec<uint32_t> trail;         // the recent-hash windows of the states (AState::tail, len)
  DevArr<uint32_t> d_trail;
  uint64_t d_trail_n = 0;
  DevArr<uint8_t> d_hlog;
  uint64_t d_hlog_n = 0;
  // processAttestation messages of the call: a 32-byte record each, plus their oblique parent
  // ids and ShardBlockHash bytes in m_var, appended by the walk straight into pinned memory and
  // digested a batch at a time on stream ms while the walk goes on (msg_send)
  PinVec<AttMsg> m_rec;
  PinVec<uint8_t> m_var;
  uint64_t m_sent = 0, m_var_sent = 0;  // records / var bytes already sent this call
  bool m_busy = false;                  // ms may still be reading the pinned buffers
  hipStream_t ms = nullptr;             // local rank 0's message stream
  DevArr<AttMsg> d_mrec;
  DevArr<uint8_t> d_mvar, d_mout;
  PinBuf m_pin;  // the message digests' D2H
  PinBuf arena_pin;  // the call arena's bytes: parsed in place, H2D'd whole for the digest batch
  // wall-time accumulators (seconds) per phase, read by pz_debug_chain_profile
  double prof[kProfSlots] = {};
  uint64_t vtrace_n = 0;               // (PZ_VOTE_TRACE) flushes launched traced
  std::vector<uint64_t> vtrace_w;      //   and their wave counts (0: not recorded)
  // per transition (tools/replay_timeline.py, correlated with a rocprofv3 kernel trace):
  // CLOCK_MONOTONIC ns at the flush's start, after its tally launch returned, after the epoch's
  // launches, and when the totals' sequence word was seen
  std::vector<std::array<uint64_t, 4>> tl;
};
static uint64_t mono_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

// Accumulates the wall time of its scope into Engine::prof[slot].
struct PhaseTimer {
  double& acc;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit PhaseTimer(double& a) : acc(a) {}
  ~PhaseTimer() { acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
};
// Per-attestation phases (checks, vote queueing) are timed only when PZ_CHAIN_PROFILE is set:
// two clock reads per attestation cost ~4 ms per 10,000 blocks of the walk they measure.
static bool fine_profile() {
#ifdef PZ_AB_BUILD
  static const bool on = std::getenv("PZ_CHAIN_PROFILE") != nullptr;
  return on;
#else
  return false;
#endif
}
struct FineTimer {
  double* acc = nullptr;
  std::chrono::steady_clock::time_point t0;
  explicit FineTimer(double& a) {
    if (fine_profile()) {
      acc = &a;
      t0 = std::chrono::steady_clock::now();
    }
  }
  ~FineTimer() {
    if (acc) *acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
};

struct Panic {
  std::string what;
};
struct Rejected {
  int code;
};

static void check(int rc) {
  if (rc) throw rc;
}
static void hchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw hip_fail(e, what);
}

template <typename T>
static void upload(Engine& g, DevArr<T>& d, const T* h, size_t n) {
  check(d.alloc(n));
  if (n) hchk(hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, g.s), "H2D");
}
template <typename T>
static void upload(RankDev& r, DevArr<T>& d, const T* h, size_t n) {
  hchk(hipSetDevice(r.dev), "hipSetDevice");
  check(d.alloc(n));
  if (n) hchk(hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, r.s), "H2D");
}
// Ranks of the chain's partition this process drives (rank 0's device left current).
static void each_rank(Engine& g, const std::function<void(RankDev&)>& f) {
  for (RankDev& r : g.rk) {
    hchk(hipSetDevice(r.dev), "hipSetDevice");
    f(r);
  }
  hchk(hipSetDevice(g.rk[0].dev), "hipSetDevice");
}
static void sync_ranks(Engine& g) {
  each_rank(g, [](RankDev& r) { hchk(hipStreamSynchronize(r.s), "sync"); });
}

// Many messages -> 64-byte digests (one CSR launch).  Blocks until done.
static void hash_many(Engine& g, const std::string& data, const std::vector<uint64_t>& offs, std::vector<uint8_t>& out) {
  const size_t n = offs.size() - 1;
  out.resize(n * 64);
  if (!n) return;
  // long messages (state roots: one serial chain each) on host threads, overlapping the GPU
  std::vector<uint64_t> lng = long_messages(offs.data(), n);
  SerialHashJob job;
  job.start((const uint8_t*)data.data(), offs.data(), lng, out.data(), 64);
  if (lng.size() == n) return;  // joined by the destructor
  const std::string* src = &data;
  const std::vector<uint64_t>* so = &offs;
  std::string cat;
  std::vector<uint64_t> co, idx;
  if (!lng.empty()) {  // compact the batchable messages
    co.push_back(0);
    size_t k = 0;
    for (uint64_t i = 0; i < n; ++i) {
      if (k < lng.size() && lng[k] == i) {
        ++k;
        continue;
      }
      cat.append(data, offs[i], offs[i + 1] - offs[i]);
      co.push_back(cat.size());
      idx.push_back(i);
    }
    src = &cat;
    so = &co;
  }
  const size_t m = so->size() - 1;
  std::vector<uint8_t> part;
  uint8_t* dst = out.data();
  if (!lng.empty()) {
    part.resize(m * 64);
    dst = part.data();
  }
  check(g.h_in.alloc(src->size() + 16));
  check(g.h_out.alloc(m * 64));
  upload(g, g.h_offs, so->data(), so->size());
  if (!src->empty()) hchk(hipMemcpyAsync(g.h_in.p, src->data(), src->size(), hipMemcpyHostToDevice, g.s), "H2D msgs");
  hchk(launch_b2b_csr(g.h_in.p, g.h_offs.p, m, g.h_out.p, 64, g.s), "blake2b csr");
  hchk(hipMemcpyAsync(dst, g.h_out.p, m * 64, hipMemcpyDeviceToHost, g.s), "D2H digests");
  hchk(hipStreamSynchronize(g.s), "sync");
  job.join();
  for (size_t j = 0; j < idx.size(); ++j) std::memcpy(&out[idx[j] * 64], &part[j * 64], 64);
}

// ---- vote cache -------------------------------------------------------------------------------
// Every rank's vote-cache arrays grown to nc slots, keeping their contents (outside a flush).
static void grow_slots(Engine& g, uint64_t nc) {
  if (nc <= g.cap) return;
  nc = (nc + 63) & ~63ull;  // whole id words
  {
    each_rank(g, [&](RankDev& r) {
      DevArr<uint64_t> bm;
      DevArr<uint64_t> tt;
      DevArr<uint8_t> pr;
      check(bm.alloc(nc / 64 * r.n + 1));
      check(tt.alloc(nc));
      check(pr.alloc(nc));
      hchk(hipMemsetAsync(bm.p, 0, (nc / 64 * r.n + 1) * 8, r.s), "memset");
      hchk(hipMemsetAsync(tt.p, 0, nc * 8, r.s), "memset");
      hchk(hipMemsetAsync(pr.p, 0, nc, r.s), "memset");
      if (g.cap) {  // the old id words are a prefix of the new rows
        if (r.n) hchk(hipMemcpyAsync(bm.p, r.bm.p, g.cap / 64 * r.n * 8, hipMemcpyDeviceToDevice, r.s), "D2D");
        hchk(hipMemcpyAsync(tt.p, r.totals.p, g.cap * 8, hipMemcpyDeviceToDevice, r.s), "D2D");
        hchk(hipMemcpyAsync(pr.p, r.present.p, g.cap, hipMemcpyDeviceToDevice, r.s), "D2D");
      }
      // (no stream sync: the old arrays are kept until the chain goes, so the queued copies and
      // tallies still reading them are safe)
      std::swap(r.bm.p, bm.p);
      std::swap(r.bm.n, bm.n);
      std::swap(r.totals.p, tt.p);
      std::swap(r.totals.n, tt.n);
      std::swap(r.present.p, pr.p);
      std::swap(r.present.n, pr.n);
      g.retired.keep(bm.p);
      g.retired.keep(tt.p);
      g.retired.keep(pr.p);
      bm.p = nullptr;
      tt.p = nullptr;
      pr.p = nullptr;
    });
    g.cap = nc;
  }
}

static uint32_t vote_slot(Engine& g, const H32& h) {
  const uint32_t s = (uint32_t)g.slot_hash.size();
  const uint32_t got = g.slot_of.insert(h, s);
  if (got != s) return got;
  g.slot_hash.push_back(h);
  g.slot_saved.push_back(0);
  if (s >= g.cap) grow_slots(g, std::max<uint64_t>(64, 2 * g.cap));
  return s;
}

static bool is_saved(const Engine& g, const H32& h) {
  const uint32_t* sl = g.slot_of.find(h);
  if (sl && g.slot_saved[*sl]) return true;
  return g.saved.size() && g.saved.count(h);
}

// Every logged hash gets its vote-cache slot at once (a slot is storage; whether the Go map
// has an entry for the hash is the slot's `present` flag, set by the tally).  A slot costs
// nval/8 bytes of voter bitmap + 9 bytes in HBM: 8 KiB per block at 65,536 validators (80 MB
// for configs[4]'s 10,000 blocks), 512 KiB at 4M; Go's VoteCache keeps a []uint32 of up to
// nval voter indices per signed hash (core.go:322-340), 32x the bitmap when fully voted, and
// in a live chain every block hash is signed.  Creating slots on a hash's first tally instead
// (measured in round 2) put a resolve loop over every queued (attestation, parent) item in the
// flush and cost 40 ms per 10,000 blocks (153 -> 88 k blocks/s, tools/gpu_replay_ab.sh).  `votable` is
// false for an id that can never be tallied: a 32-byte oblique parent hash is only ever a
// parent of its own attestation, which skips it (core.go:313-320).
static void msg_drain(Engine& g);
static uint32_t log_hash(Engine& g, const H32& h, bool votable = true) {
  g.hlog.push_back(h);
  g.id_slot.push_back(votable ? vote_slot(g, h) : UINT32_MAX);
  return (uint32_t)(g.hlog.size() - 1);
}

// Enqueue the pending tally items on every rank; no host wait (the pinned arena and its
// per-rank events make the H2D asynchronous).  Balances only change in stateRecalc's epoch,
// which each rank's stream orders after every flush, so a flush may run any time before it.
// With `gq` (a stateRecalc's flush on one rank), the tally's last block also gathers the 64
// justification totals into g.tot_pin (polled by their sequence word): returns true when it
// did so (tally_gather_enqueue's work is then done).
// One rank's stateRecalc epoch, prepared on the host (the pack in g.e_pin, the arguments) by the
// transition's vote flush before its tally launch, whose count blocks ride in that launch
// (pz_vote_words_count_kernel), reading the pinned pack in place: two launches less per
// transition.  `staged` / `counted`: done (else epoch_launch_rest does them).
struct EpochLaunch {
  EpochArgs a;
  EpochHandoff ho;
  size_t total = 0;      // pack bytes (a multiple of 16)
  bool win = false;      // crosslink winners to form
  bool staged = false, counted = false;
  bool ready = false;    // prepared (by the flush's hook, or by state_recalc when nothing was flushed)
};
using EpochPrep = std::function<EpochLaunch*()>;

// How a flush reaches the device (PZ_VOTE_PATH, read per call so that one test process can
// run every path; A/B knob):
//   direct (product)    no copy: the tally reads the walk's pinned queue in place (one 64-B
//                       record per attestation, votes.h VoteRec);
//   segments            the queue arrays copied into a device pack by ONE multi-segment stage
//                       kernel, then the tally (one launch more per flush: 1-3 % slower,
//                       profiles/r04/replay_ab_words_r4k.txt);
//   packed              round 3: the queue memcpy'd into one pinned arena first, one stage copy.
enum VotePath { kVoteSegments, kVotePacked, kVoteDirect };
static void read_knobs(Engine& g) {
  g.kn = Knobs{};
  g.kn.vote_groups = !(g.opt.tally_forms & PZ_TALLY_PER_ATTESTATION);
#ifdef PZ_AB_BUILD
  auto is = [](const char* name, const char* v) {
    const char* e = std::getenv(name);
    return e && !std::strcmp(e, v);
  };
  g.kn.vote_path = is("PZ_VOTE_PATH", "packed") ? kVotePacked : is("PZ_VOTE_PATH", "segments") ? kVoteSegments : kVoteDirect;
  g.kn.vote_trace = std::getenv("PZ_VOTE_TRACE") != nullptr;
  g.kn.epoch_pack_direct = is("PZ_EPOCH_PACK", "direct");
  g.kn.epoch_prep_after = !is("PZ_EPOCH_PREP", "merged");
#endif
}

static bool flush_votes_enqueue(Engine& g, const VoteGatherSlots* gq = nullptr, const EpochPrep* prep = nullptr) {
  Engine::VoteQueue& Q = g.vq[g.vq_cur];
  if (Q.natt() == 0) return false;
  const bool gather = gq && g.world == 1;
  const VotePath path = (VotePath)g.kn.vote_path;
  const bool staged = path != kVoteDirect;  // a device copy of the queue
  PhaseTimer pt(g.prof[kProfFlush]);
  const uint64_t natt = Q.natt();
  auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
  // the device pack: rec | slots | bits
  const size_t o_rec = 0, o_slots = o_rec + natt * sizeof(VoteRec), o_bits = o_slots + al(Q.slots.size() * 4),
               total = staged ? o_bits + al(Q.bits.size()) : 0;
  if (path == kVotePacked) {
    if (g.q_arena_busy) {
      FineTimer pw(g.prof[kProfFlushWait]);
      for (RankDev& r : g.rk) hchk(hipEventSynchronize(r.q_ev), "event sync");
      g.q_arena_busy = false;
    }
    check(g.q_arena.reserve(total));
    uint8_t* qa = g.q_arena.p;
    std::memcpy(qa + o_rec, Q.rec.data(), natt * sizeof(VoteRec));
    if (Q.slots.size()) std::memcpy(qa + o_slots, Q.slots.data(), Q.slots.size() * 4);
    if (Q.bits.size()) std::memcpy(qa + o_bits, Q.bits.data(), Q.bits.size());
  }
  // the grouped form (votes.h VoteGroup): the walk's queue read in place, every record in the run
  // form, each group within kVoteGroupWords id words (PZ_VOTE_GROUPS=0: A/B and test knob)
  bool grouped = path == kVoteDirect && Q.groupable && !Q.grp.empty() && g.kn.vote_groups;
  VoteGroup groups[kVoteMaxGroups];
  uint32_t nwaves = 0, ngroups = 0;
  if (grouped) {
    ngroups = (uint32_t)Q.grp.size();
    uint32_t* pm = Q.perm.grow(natt);
    uint32_t o = 0;
    for (size_t i = 0; i < Q.grp.size() && grouped; ++i) {
      const Engine::VoteQueue::Group& G = Q.grp[i];
      VoteGroup& d = groups[i];
      d.cb = (uint32_t)g.h_coffs[G.c];
      d.k = G.k;
      d.first = o;
      d.n = (uint32_t)G.atts.size();
      d.wlo = G.idlo == UINT32_MAX ? 0 : G.idlo >> 6;
      d.nw = G.idlo == UINT32_MAX ? 0 : (G.idhi >> 6) - d.wlo + 1;
      d.wave0 = nwaves;
      // (records at a fixed stride, as a block's attestations of its committees in order: no
      // index array to read)
      d.stride = 0;
      if (G.atts.size() == 1) {
        d.stride = 1;
      } else {
        const uint32_t st = G.atts[1] - G.atts[0];
        bool ap = st > 0;
        for (size_t j = 2; j < G.atts.size() && ap; ++j) ap = G.atts[j] - G.atts[j - 1] == st;
        if (ap) d.stride = st;
      }
      d.first = d.stride ? G.atts[0] : o;
      if (d.nw > (uint32_t)kVoteGroupWords) grouped = false;
      nwaves += std::max<uint32_t>(1, (G.k + 63) / 64);  // (an empty committee: one wave, its parents' map entries)
      std::memcpy(pm + o, G.atts.data(), G.atts.size() * 4);
      o += (uint32_t)G.atts.size();
    }
  }
  for (const Engine::VoteQueue::Group& G : Q.grp) Q.gof[G.c] = 0;
  Q.grp.clear();
  Q.groupable = true;
  each_rank(g, [&](RankDev& r) {
    // Growing a device buffer frees the old one, which in-flight flushes may still read:
    // drain the stream first (rare: the buffer doubles).
    if (total > r.d_qpack.n) {
      hchk(hipStreamSynchronize(r.s), "sync");
      check(r.d_qpack.alloc(std::max<uint64_t>(total, 2 * r.d_qpack.n)));
    }
    if (path == kVotePacked) {
      // the pack crosses PCIe in a kernel of this stream (a copy-engine H2D costs ~13 us more on
      // the transition's critical path: the kernel behind it waits for the engine's signal)
      void* src = nullptr;
      check(g.q_arena.dev(r.dev, &src));
      hchk(launch_stage_h2d(src, r.d_qpack.p, total, r.s), "stage H2D");
      if (!gather) {  // (gathering: the transition's totals, later in the stream, free the arena)
        if (!r.q_ev) hchk(hipEventCreateWithFlags(&r.q_ev, hipEventDisableTiming), "event");
        hchk(hipEventRecord(r.q_ev, r.s), "event");
      }
    }
#ifdef PZ_AB_BUILD
    else if (path == kVoteSegments) {
      // the queue's pinned arrays straight into the pack, one launch (no host-side copy)
      StageSegs sg;
      sg.nseg = 0;
      auto seg = [&](const void* src, size_t off, size_t bytes) {
        if (bytes) sg.seg[sg.nseg++] = StageSeg{src, r.d_qpack.p + off, (bytes + 15) / 16};
      };
      seg(Q.rec.dev(r.dev), o_rec, natt * sizeof(VoteRec));
      seg(Q.slots.dev(r.dev), o_slots, Q.slots.size() * 4);
      seg(Q.bits.dev(r.dev), o_bits, Q.bits.size());
      hchk(launch_stage_h2d_segs(sg, r.s), "stage H2D");
    }
#endif
    if (!r.d_err.p) {
      check(r.d_err.alloc(1));
      hchk(hipMemsetAsync(r.d_err.p, 0, 8, r.s), "memset");
    }
    if (!r.v_ticket.p) {
      check(r.v_ticket.alloc(1));
      hchk(hipMemsetAsync(r.v_ticket.p, 0, 4, r.s), "memset");
    }
    VoteWordArgs v;
    std::memset(&v, 0, sizeof v);
    v.committee = r.committee.p;
    if (staged) {
      v.rec = reinterpret_cast<const VoteRec*>(r.d_qpack.p + o_rec);
      v.slots = reinterpret_cast<const uint32_t*>(r.d_qpack.p + o_slots);
      v.bits = g.bits_inline ? nullptr : r.d_qpack.p + o_bits;
    } else {  // read in place (pinned, mapped into this rank's device)
      v.rec = Q.rec.dev(r.dev);
      v.slots = Q.slots.size() ? Q.slots.dev(r.dev) : nullptr;
      v.bits = g.bits_inline ? nullptr : Q.bits.dev(r.dev);
    }
    v.natt = natt;
    if (grouped) {
      v.ngroups = ngroups;
      std::memcpy(v.groups, groups, ngroups * sizeof(VoteGroup));
      v.nwaves = nwaves;
      v.perm = Q.perm.dev(r.dev);
    }
    v.bstride = g.bf_stride;
    v.chunks = Q.chunks;
    v.balance = r.balance.p;
    v.nval = r.n;
    v.val_offset = r.lo;
    v.nval_global = g.nval;
    v.bm = r.bm.p;
    v.totals = r.totals.p;
    v.present = r.present.p;
    v.err = r.d_err.p;  // sticky: read (and the chain poisoned) at the next sync point
    if (gather) {
      check(g.tot_pin.reserve((kJustifySlots + 2) * 8));
      void* dp = nullptr;
      check(g.tot_pin.dev(r.dev, &dp));
      v.gather_out = static_cast<uint64_t*>(dp);
      v.ticket = r.v_ticket.p;
      v.gq = *gq;
      v.gather_seq = ++g.gather_seq;
      // (pooled pinned memory holds old words: clear the sequence word before the launch)
      reinterpret_cast<volatile uint64_t*>(g.tot_pin.p)[kJustifySlots + 1] = 0;
    }
#ifdef PZ_AB_BUILD
    if (prep) {
      // (A/B, PZ_EPOCH_PREP=merged: the transition's epoch packed before the launch) the tally
      // with the epoch's count blocks in one launch
      EpochLaunch* el = (*prep)();
      hchk(launch_vote_words_count(v, el->a, r.s), "vote tally + epoch count");
      el->counted = true;
    } else if (g.kn.vote_trace && r.grank == 0) {
      // (tools/vote_trace.py: the first kVoteTraceFlushes flushes' per-wave phase stamps)
      if (!r.v_trace.p) {
        check(r.v_trace.alloc((size_t)kVoteTraceFlushes * kVoteTraceWaves * 8));
        hchk(hipMemsetAsync(r.v_trace.p, 0, (size_t)kVoteTraceFlushes * kVoteTraceWaves * 64, r.s), "memset");
      }
      const uint64_t waves = v.ngroups ? 4ull * v.nwaves : natt * Q.chunks;
      uint64_t* tr = g.vtrace_n < kVoteTraceFlushes && waves <= kVoteTraceWaves
                         ? r.v_trace.p + (size_t)g.vtrace_n * kVoteTraceWaves * 8
                         : nullptr;
      g.vtrace_w.push_back(tr ? waves : 0);
      ++g.vtrace_n;
      hchk(launch_vote_words_traced(v, tr, r.s), "vote tally");
    } else
#else
    (void)prep;
#endif
    {
      hchk(launch_vote_words(v, r.s), "vote tally");
    }
    if (!gather) {  // (gathering: the walk waits for the tally before any later flush)
      if (!r.vq_ev[g.vq_cur]) hchk(hipEventCreateWithFlags(&r.vq_ev[g.vq_cur], hipEventDisableTiming), "event");
      hchk(hipEventRecord(r.vq_ev[g.vq_cur], r.s), "event");
    }
  });
  if (path == kVotePacked) g.q_arena_busy = !gather;
  g.gather_poll = gather;
  // the walk goes on in the other queue, once the flush before last has stopped reading it (a
  // gathering flush is waited for by tally_gather_finish before the walk goes on)
  Q.busy = !gather;
  g.vq_cur ^= 1;
  Engine::VoteQueue& N = g.vq[g.vq_cur];
  if (N.busy) {
    FineTimer pw(g.prof[kProfFlushWait]);
    for (RankDev& r : g.rk)
      if (r.vq_ev[g.vq_cur]) hchk(hipEventSynchronize(r.vq_ev[g.vq_cur]), "event sync");
    N.busy = false;
  }
  N.rec.reset();
  N.perm.reset();
  N.slots.reset();
  N.bits.reset();
  N.chunks = 1;
  return gather;
}

// Enqueue, behind every rank's pending tallies, the gather of the 64 justification totals
// (slot UINT32_MAX: 0) and the sticky tally panic flag, then g.ev_totals: one rank straight
// into g.tot_pin; sharded, into each rank's xred, summed by one all-reduce (the partial
// VoteTotalDeposit sums of the validator ranges, with any pending next-cycle partial).
// sharded (world > 1): every rank's xred [totals + panic flag | TotalDeposits slot | epoch
// partials (nred words)] summed by ONE all-reduce, each rank's stream waiting for it, rank 0's
// first kJustifySlots + 2 words D2H into g.tot_pin, then g.ev_totals.  A pending next-cycle
// partial rode in the TotalDeposits slot: tally_gather_finish hands the sum to g.nb_dst.
static void sharded_allreduce(Engine& g, uint64_t nred) {
  check(g.tot_pin.reserve((kJustifySlots + 2) * 8));
  std::vector<uint64_t*> bufs;
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> evs;
  for (RankDev& r : g.rk) {
    if (!r.ev_t64) hchk(hipEventCreateWithFlags(&r.ev_t64, hipEventDisableTiming), "event");
    bufs.push_back(r.xred.p);
    streams.push_back(r.s);
    evs.push_back(r.ev_t64);
  }
  check(g.comm->allreduce_u64(bufs.data(), kJustifySlots + 2 + nred, streams.data(), evs.data()));
  for (RankDev& r : g.rk) {
    hchk(hipSetDevice(r.dev), "hipSetDevice");
    hchk(hipStreamWaitEvent(r.s, r.ev_t64, 0), "wait");
  }
  RankDev& r0 = g.rk[0];
  hchk(hipSetDevice(r0.dev), "hipSetDevice");
  hchk(hipMemcpyAsync(g.tot_pin.p, r0.xred.p, (kJustifySlots + 2) * 8, hipMemcpyDeviceToHost, r0.s), "D2H");
  if (!g.ev_totals) hchk(hipEventCreateWithFlags(&g.ev_totals, hipEventDisableTiming), "event");
  hchk(hipEventRecord(g.ev_totals, r0.s), "event");
  g.nb_carried = g.nb_pending;
  g.nb_pending = false;
}

// sharded: a rank's gather into its xred and the TotalDeposits slot (the pending next-cycle
// partial, else zero; a transition's epoch puts rank 0's known TotalDeposits there instead)
static void sharded_gather(Engine& g, RankDev& r, const VoteGatherSlots& q, uint64_t nred) {
  check(r.xred.alloc(kJustifySlots + 2 + nred));
  check(r.nbp.alloc(1));
  if (!r.d_err.p) {
    check(r.d_err.alloc(1));
    hchk(hipMemsetAsync(r.d_err.p, 0, 8, r.s), "memset");
  }
  hchk(launch_vote_gather(r.totals.p, q, r.d_err.p, r.xred.p, r.s), "vote gather");
  if (g.nb_pending)
    hchk(hipMemcpyAsync(r.xred.p + kJustifySlots + 1, r.nbp.p, 8, hipMemcpyDeviceToDevice, r.s), "D2D");
  else
    hchk(hipMemsetAsync(r.xred.p + kJustifySlots + 1, 0, 8, r.s), "memset");
}

static void tally_gather_enqueue(Engine& g, const VoteGatherSlots& q) {
  check(g.tot_pin.reserve((kJustifySlots + 2) * 8));
  if (g.world > 1) {  // (a call's final flush: the totals and any pending next-cycle partial)
    each_rank(g, [&](RankDev& r) { sharded_gather(g, r, q, 0); });
    sharded_allreduce(g, 0);
    return;
  }
  // one rank: the gather stores straight into the pinned totals (no D2H copy behind it)
  RankDev& r = g.rk[0];
  hchk(hipSetDevice(r.dev), "hipSetDevice");
  if (!r.d_err.p) {
    check(r.d_err.alloc(1));
    hchk(hipMemsetAsync(r.d_err.p, 0, 8, r.s), "memset");
  }
  void* dp = nullptr;
  check(g.tot_pin.dev(r.dev, &dp));
  hchk(launch_vote_gather(r.totals.p, q, r.d_err.p, static_cast<uint64_t*>(dp), r.s), "vote gather");
  if (!g.ev_totals) hchk(hipEventCreateWithFlags(&g.ev_totals, hipEventDisableTiming), "event");
  hchk(hipEventRecord(g.ev_totals, g.rk[0].s), "event");
}

// After g.ev_totals: raise the panic a tally detected.
static void tally_gather_wait(Engine& g);
static void tally_gather_finish(Engine& g) {
  tally_gather_wait(g);
  if (g.nb_carried) {  // sharded: the last epoch's next-cycle balance, summed over the ranks
    g.nb_carried = false;
    if (g.nb_dst) g.nb_dst->tdep = reinterpret_cast<const uint64_t*>(g.tot_pin.p)[kJustifySlots + 1];
    g.nb_dst.reset();
  }
}

static void tally_gather_wait(Engine& g) {
  PhaseTimer pt(g.prof[kProfTotalsWait]);
  const bool polled = g.gather_poll;  // (a gathering flush records no event: its fallback syncs the stream)
  if (g.gather_poll) {
    // The fused gather writes its sequence word last (system-scope release): spin on the pinned
    // word instead of sleeping in the event wait, whose wake-up took ~10-20 us of every
    // transition's critical path.  Bounded: past ~50 ms the event wait decides (an error
    // surfaces there).
    g.gather_poll = false;
    const volatile uint64_t* sq = reinterpret_cast<const volatile uint64_t*>(g.tot_pin.p) + kJustifySlots + 1;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0; *sq != g.gather_seq; ++k) {
      __builtin_ia32_pause();
      if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (*sq != g.gather_seq) g.prof[kProfPollFallback] += 1;  // reported, so a fallback is not silent
    if (*sq == g.gather_seq) {
      // every rank's flush is done: its stage kernel preceded the tally
      g.q_arena_busy = false;
      if (reinterpret_cast<const uint64_t*>(g.tot_pin.p)[kJustifySlots])
        throw Panic{"calculateBlockVoteCache: CheckBit / validator index out of range"};
      return;
    }
  }
  if (polled)
    hchk(hipStreamSynchronize(g.rk[0].s), "stream sync (vote totals)");
  else
    hchk(hipEventSynchronize(g.ev_totals), "event sync (vote totals)");
  g.q_arena_busy = false;  // every rank's flush is behind g.ev_totals
  if (reinterpret_cast<const uint64_t*>(g.tot_pin.p)[kJustifySlots])
    throw Panic{"calculateBlockVoteCache: CheckBit / validator index out of range"};
}

// Every queued tally done, its panic (if any) raised.
static void flush_votes(Engine& g) {
  flush_votes_enqueue(g);
  VoteGatherSlots q;
  for (int j = 0; j < kJustifySlots; ++j) q.slot[j] = UINT32_MAX;
  tally_gather_enqueue(g, q);
  PhaseTimer pt(g.prof[kProfFlush]);
  tally_gather_finish(g);
}

// ---- core.go ------------------------------------------------------------------------------------
// The signed parent hashes of an attestation (getSignedParentHashes, core.go:348-360) as
// hash-log ids: the window trail[wstart, wstart + nw) of RecentBlockHashes, then the oblique
// parent hashes (ids obl[0, nobl)); always 64 in all.
struct Parents {
  uint64_t wstart = 0;
  uint32_t nw = 0;
  std::vector<uint32_t> obl;
  uint32_t id(const Engine& g, size_t j) const;
};

uint32_t Parents::id(const Engine& g, size_t j) const { return j < nw ? g.trail[wstart + j] : obl[j - nw]; }

// Hash-log id i of the window of A (RecentBlockHashes[i]).
static inline uint32_t recent_id(const Engine& g, const AState& A, uint64_t i) { return g.trail[A.tail - A.len + i]; }

// RecentBlockHashes = append(RecentBlockHashes, id)[-2 * kCycle:] (computeNewActiveState,
// core.go:223-237): appended at the trail's end, after re-appending A's window if another
// state's pushes came after it.
static void push_recent(Engine& g, AState& A, uint32_t id) {
  if (A.tail != g.trail.size()) {
    const uint64_t b = A.tail - A.len, at = g.trail.size();
    g.trail.resize(at + A.len);
    for (uint32_t i = 0; i < A.len; ++i) g.trail[at + i] = g.trail[b + i];
    A.tail = g.trail.size();
  }
  g.trail.push_back(id);
  ++A.tail;
  A.len = (uint32_t)std::min<uint64_t>(A.len + 1, 2 * kCycle);
}

// Go slices up to cap, beyond len panics.
static void signed_parents(Engine& g, const AState& A, uint64_t block_slot, const Att& a, Parents& out) {
  const uint64_t start = block_slot - a.slot;
  const uint64_t end = block_slot - a.slot - (uint64_t)a.obl.size() + kCycle;
  if (start > end || end > A.len) throw Panic{"slice bounds out of range (core.go:353)"};
  out.wstart = A.tail - A.len + start;
  out.nw = (uint32_t)(end - start);
  out.obl.clear();
  for (auto& o : a.obl) out.obl.push_back(log_hash(g, bytes_to_hash(a.at(o.first), o.second), o.second != 32));
}

// getAttesterIndices (core.go:363-374) -> committee id.
static uint32_t attester_committee(const Engine& g, const CState& C, const Att& a) {
  const uint64_t idx = a.slot - C.lsr;  // uint64 wrap, like Go
  if (idx >= g.lookup.size()) throw Panic{"ShardAndCommitteesForSlots index out of range (core.go:367)"};
  for (auto& sc : g.lookup[idx])
    if (sc.first == a.shard) return sc.second;
  throw Rejected{PZ_ATT_NO_COMMITTEE};
}

// uvarint(x) at p (Go's binary.PutUvarint); returns the bytes written.
static size_t put_uvarint(uint8_t* p, uint64_t x) {
  size_t n = 0;
  while (x >= 0x80) {
    p[n++] = (uint8_t)(x | 0x80);
    x >>= 7;
  }
  p[n++] = (uint8_t)x;
  return n;
}

// What processAttestation found out about an attestation that calculateBlockVoteCache, run
// next on the same block state, would compute again: its signed parent hashes (hash-log ids)
// and its committee.
struct AttLookup {
  bool have = false;
  uint32_t comm = 0;
  Parents parents;
};

// processAttestation (core.go:240-297) -> builds the message whose digest the reference logs.
static void process_attestation(Engine& g, uint64_t block_slot, const Att& a, AttLookup& L) {
  L.have = false;
  if ((int64_t)a.slot > (int64_t)block_slot) throw Rejected{PZ_ATT_SLOT_HIGH};
  if ((int64_t)a.slot < (int64_t)block_slot - (int64_t)kCycle) throw Rejected{PZ_ATT_SLOT_LOW};
  if (a.jslot != g.C->jslot) throw Rejected{PZ_ATT_JUSTIFIED};
  Parents& parents = L.parents;
  signed_parents(g, *g.A, block_slot, a, parents);
  const uint32_t c = attester_committee(g, *g.C, a);
  L.comm = c;
  L.have = true;
  const uint64_t k = g.csize[c];
  if ((k + 7) / 8 != a.bf_len) throw Rejected{PZ_ATT_BITFIELD_LEN};  // core.go:379-382
  if (k % 8 && (a.at(a.bf_off)[a.bf_len - 1] & (0xFFu >> (k % 8)))) throw Rejected{PZ_ATT_TRAILING_BITS};
  // the message: a 10-byte buffer holding uvarint(slot % 64) overwritten by uvarint(shard)
  // at offset 0, then "parent ' '" x 64, then ShardBlockHash; assembled on the device
  uint8_t hdr[16] = {0};
  put_uvarint(hdr, a.slot % kCycle);
  put_uvarint(hdr, a.shard);
  const size_t nobl = parents.obl.size(), vb = (4 * nobl + a.sbh_len + 3) & ~size_t(3);
  AttMsg* m = g.m_rec.grow(1);
  std::memcpy(m->hdr, hdr, sizeof m->hdr);
  m->nw = (uint16_t)parents.nw;
  m->wstart = (uint32_t)parents.wstart;
  m->sl = (uint32_t)a.sbh_len;
  m->pad = 0;
  m->vo = g.m_var.n;
  uint8_t* v = g.m_var.grow(vb);
  if (nobl) std::memcpy(v, parents.obl.data(), 4 * nobl);
  std::memcpy(v + 4 * nobl, a.at(a.sbh_off), a.sbh_len);
  std::memset(v + 4 * nobl + a.sbh_len, 0, vb - 4 * nobl - a.sbh_len);
}

// calculateBlockVoteCache (core.go:300-345): queue one tally item per signed parent hash.
// The parents and committee come from processAttestation's lookup when it got that far (the
// block state is the same), else they are looked up here.
static void queue_vote_cache(Engine& g, uint64_t block_slot, const Att& a, AttLookup& L) {
  if (!L.have) {
    signed_parents(g, *g.A, block_slot, a, L.parents);
    L.comm = attester_committee(g, *g.C, a);
    L.have = true;
  }
  const Parents& parents = L.parents;
  const uint32_t c = L.comm;
  const uint64_t k = g.csize[c];
  // Parents equal to one of the raw oblique parent hashes are skipped (core.go:313-320); only
  // a 32-byte oblique can equal a [32]byte parent.  The parents are the recent window then the
  // obliques themselves (always 64 of them), so a 32-byte oblique's own position is skipped,
  // and any other parent with its bytes has the vote-cache slot its bytes were given (slots
  // are per distinct hash; a 32-byte oblique id has none, which no slot equals).
  const size_t nobl = a.obl.size(), np = parents.nw + nobl;
  uint64_t skip = 0;
  uint32_t match[64];
  int nmatch = 0;
  for (size_t i = 0; i < nobl; ++i) {
    const auto& o = a.obl.p[i];
    if (o.second != 32) continue;
    skip |= 1ull << (np - nobl + i);
    H32 h;
    std::memcpy(h.b, a.at(o.first), 32);
    if (const uint32_t* sl = g.slot_of.find(h)) match[nmatch++] = *sl;
  }
  Engine::VoteQueue& Q = g.vq[g.vq_cur];
  // the 64 parents' vote-cache ids, UINT32_MAX where a parent is not tallied, as a run (votes.h
  // VoteRec: s0, step, absent) when they make one
  uint64_t step = 0, absent = 0;
  bool run = !g.ids_rows;
  uint32_t s0 = UINT32_MAX, prev = 0;
  auto put = [&](size_t j, uint32_t sl) {
    if (((skip >> j) & 1) || sl == UINT32_MAX) {
      absent |= 1ull << j;
      return;
    }
    if (s0 == UINT32_MAX) s0 = sl;
    else if (sl == prev + 1) step |= 1ull << j;
    else if (sl != prev) run = false;
    prev = sl;
  };
  // (the trail's and the id table's base pointers hoisted: PinVec::operator[] is three dependent
  // loads)
  const uint32_t* tr = g.trail.data() + parents.wstart;
  const uint32_t* ids = g.id_slot.data();
  const size_t nw = parents.nw;
  auto id_at = [&](size_t j) -> uint32_t {
    return j < nw ? ids[tr[j]] : j < np ? ids[parents.obl[j - nw]] : UINT32_MAX;
  };
  if (nmatch == 0) {
    // The window part is the same for every attestation of a block (and its run summary for
    // every attestation over the same window): computed once per window (the walk's samples had
    // the 64-parent loop at 12 %), then the obliques' positions one by one.
    WindowRun& W = g.wrun;
    if (W.wstart != parents.wstart || W.nw != nw || W.gen != g.trail_gen) {
      W.wstart = parents.wstart;
      W.nw = nw;
      W.gen = g.trail_gen;
      for (size_t j = 0; j < nw && j < 64; ++j) put(j, id_at(j));
      W.step = step, W.absent = absent, W.s0 = s0, W.prev = prev, W.run = run;
    } else {
      step = W.step, absent = W.absent, s0 = W.s0, prev = W.prev, run = W.run && run;
    }
    for (size_t j = nw; j < 64; ++j) put(j, id_at(j));
  } else {
    for (size_t j = 0; j < 64; ++j) {
      const uint32_t sl = id_at(j);
      for (int m = 0; m < nmatch; ++m)
        if (sl == match[m]) skip |= 1ull << j;
      put(j, sl);
    }
  }
  if (skip == ~0ull) return;  // no map access at all
  if (g.A->cache_nil) throw Panic{"assignment to entry in nil map (core.go:323)"};
  // the member loop reaches CheckBit(bitfield, 8 * len) when the committee is longer
  if (k > 8ull * a.bf_len) throw Panic{"calculateBlockVoteCache: CheckBit index out of range (core.go:330)"};
  if (!run || !g.bits_inline) Q.groupable = false;
  if (Q.groupable) {
    if (Q.gof.size() < g.ncomm) Q.gof.assign(g.ncomm, 0);
    int32_t& gi = Q.gof[c];
    if (!gi) {
      if (Q.grp.size() >= (size_t)kVoteMaxGroups) {
        Q.groupable = false;
      } else {
        Q.grp.emplace_back();
        Q.grp.back().c = c;
        Q.grp.back().k = (uint32_t)k;
        gi = (int32_t)Q.grp.size();
      }
    }
    if (Q.groupable) {
      Engine::VoteQueue::Group& G = Q.grp[gi - 1];
      if (absent != ~0ull) {  // the run's ids: [s0, s0 + popcount(step)]
        G.idlo = std::min(G.idlo, s0);
        G.idhi = std::max(G.idhi, s0 + (uint32_t)__builtin_popcountll(step));
      }
      G.atts.push_back((uint32_t)Q.natt());
    }
  }
  VoteRec* rec = Q.rec.grow(1);
  rec->cb = (uint32_t)g.h_coffs[c];
  rec->k = (uint32_t)k;
  if (run) {
    rec->s0 = s0;
    rec->form = 0;
    rec->step = step;
    rec->absent = absent;
  } else {
    rec->s0 = (uint32_t)(Q.slots.size() / 64);
    rec->form = kVoteIdsRow;
    g.prof[kProfIdRows] += 1;
    rec->step = rec->absent = 0;
    uint32_t* row = Q.slots.grow(64);
    for (size_t j = 0; j < 64; ++j) row[j] = ((absent >> j) & 1) ? UINT32_MAX : id_at(j);
  }
  const uint8_t* bf = a.at(a.bf_off);
  const size_t nbf = (k + 7) / 8;
  if (g.bits_inline) {  // (k <= 256: at most 32 bytes)
    std::memset(rec->bits, 0, sizeof rec->bits);
    if (nbf) std::memcpy(rec->bits, bf, nbf);
  } else {
    // the bitfield at a fixed stride (VoteWordArgs.bstride), the rest of its row zero
    std::memset(rec->bits, 0, sizeof rec->bits);
    uint8_t* row = Q.bits.grow(g.bf_stride);
    if (nbf) std::memcpy(row, bf, nbf);
    std::memset(row + nbf, 0, g.bf_stride - nbf);
  }
  Q.chunks = std::max<uint32_t>(Q.chunks, (uint32_t)((k + 255) / 256));
  if (Q.natt() >= kFlushAtts || Q.bits.size() >= (1ull << 31))
    flush_votes_enqueue(g);  // bounds the queue (and its u32 offsets); no host wait
}

// One rank: the epoch's arguments over the pack in g.e_pin (already built), its device buffers,
// and the hand-off that returns its results.  The kernels read the pack from r.e_pack, which
// the transition's flush stages (or epoch_launch_rest); PZ_EPOCH_PACK=direct (A/B knob) lets
// them read the pinned pack in place instead.
static EpochLaunch epoch_prepare_args(Engine& g, CState& C, size_t na, size_t nrec, uint64_t nbits, size_t o_boffs,
                                      size_t o_rdyn, size_t o_small, size_t o_comm, size_t o_shard, size_t o_bits,
                                      size_t total, bool in_place) {
  EpochLaunch el;
  RankDev& r = g.rk[0];
  hchk(hipSetDevice(r.dev), "hipSetDevice");
  const uint64_t nred = kScal + 2 * (uint64_t)na;
  const uint64_t wn = (nrec + 1) / 2;
  const size_t had = r.e_red.n;
  check(r.e_red.alloc(nred + wn + 1));
  if (r.e_red.n != had) hchk(hipMemsetAsync(r.e_red.p, 0, kScal * 8, r.s), "memset");  // (once per growth)
  if (!r.e_ticket.p) {
    check(r.e_ticket.alloc(1));
    hchk(hipMemsetAsync(r.e_ticket.p, 0, 4, r.s), "memset");
  }
  check(g.e_pin_out.reserve((kScal + wn + 1) * 8));
  void *hp = nullptr, *op = nullptr;
  check(g.e_pin.dev(r.dev, &hp));
  check(g.e_pin_out.dev(r.dev, &op));
  reinterpret_cast<volatile uint64_t*>(g.e_pin_out.p)[kScal + wn] = 0;  // (pooled memory: old words)
  const bool direct = in_place || g.kn.epoch_pack_direct;
  uint8_t* d = static_cast<uint8_t*>(hp);
  if (!direct) {
    check(r.e_pack.alloc(total));
    d = r.e_pack.p;
  }
  el.total = total;
  el.staged = direct;  // nothing to stage when the kernels read the pinned pack
  EpochArgs& a = el.a;
  std::memset(&a, 0, sizeof a);
  a.ninst = 1;
  a.nval = r.n;
  a.val_offset = r.lo;
  a.nval_global = g.nval;
  a.kind = PZ_KIND_ACTIVE;
  a.balance = r.balance.p;
  a.start = r.start.p;
  a.end = r.end.p;
  a.dynasty = reinterpret_cast<const uint64_t*>(d + o_small);
  a.total_deposit = reinterpret_cast<const uint64_t*>(d + o_small) + 1;
  a.natt = (uint32_t)na;
  a.bits = d + o_bits;
  a.boffs = reinterpret_cast<const uint64_t*>(d + o_boffs);
  a.max_inst_bytes = nbits;
  a.pop_rank = 0;
  a.pop_world = 1;
  a.committee = r.committee.p;
  a.coffs = r.coffs.p;
  a.att_comm = reinterpret_cast<const uint32_t*>(d + o_comm);
  a.att_shard = reinterpret_cast<const uint32_t*>(d + o_shard);
  a.nrec = (uint32_t)nrec;
  a.rec_dynasty = reinterpret_cast<const uint64_t*>(d + o_rdyn);
  a.winner = reinterpret_cast<uint32_t*>(r.e_red.p + kScal);
  a.scal = r.e_red.p;
  a.vote = r.e_red.p + kScal + wn;
  a.total = r.e_red.p + kScal + wn + na;
  a.act_mask = r.e_mask.p;
  a.blk_cnt = r.e_blk.p;
  a.act_list = r.e_list.p;
  el.ho.ticket = r.e_ticket.p;
  el.ho.out = static_cast<uint64_t*>(op);
  el.ho.nrec = (uint32_t)nrec;
  el.ho.seq = ++g.epoch_seq;
  el.win = a.nrec > 0 && na > 0;
  if (g.aa_dyn != C.dynasty) {
    g.aa_dyn = C.dynasty;
    g.aa = true;
    for (uint64_t v = 0; v < g.nval && g.aa; ++v) g.aa = g.h_start[v] <= C.dynasty && C.dynasty < g.h_end[v];
  }
  g.deferred.nrec = nrec;
  g.deferred.seq = el.ho.seq;
  el.ready = true;
  return el;
}

// The launches of a prepared one-rank epoch that the flush did not take: the stage copy and the
// count pass (if the flush did not carry them), then winners + rewards + hand-off (one launch
// when every validator is active, else mid with the compaction, then rewards + hand-off).
static void epoch_launch_rest(Engine& g, EpochLaunch& el) {
  RankDev& r = g.rk[0];
  hchk(hipSetDevice(r.dev), "hipSetDevice");
  if (!el.staged) {
    void* hp = nullptr;
    check(g.e_pin.dev(r.dev, &hp));
    hchk(launch_stage_h2d(hp, r.e_pack.p, el.total, r.s), "stage H2D (epoch)");
  }
  if (!el.counted) hchk(launch_epoch_count(el.a, true, true, true, r.s), "epoch count");
  if (g.aa) {  // no compaction: the winners run beside the rewards (one launch)
    hchk(launch_epoch_reward_handoff(el.a, el.ho, el.win, r.s), "epoch reward");
  } else {
    hchk(launch_epoch_mid(el.a, el.win, true, r.s), "epoch mid");
    hchk(launch_epoch_reward_handoff(el.a, el.ho, false, r.s), "epoch reward");
  }
}

// processCrosslinks + CalculateRewards + next-cycle balance on the device: enqueued, its
// results landing in pinned memory behind g.ev_epoch (collected by epoch_collect).
// out (one rank): prepare only -- the pack and the arguments into *out, the kernels read the pack
// in place (in_place) or from the stage copy; the caller launches (the flush and
// epoch_launch_rest).
static void epoch_enqueue(Engine& g, CState& C, const std::vector<AttP>& pending, EpochLaunch* out = nullptr,
                          bool in_place = false, const VoteGatherSlots* q = nullptr) {
  const size_t na = pending.size();
  std::vector<Crosslink>& xl = *C.xl;
  const size_t nrec = xl.size();
  uint64_t nbits = 0;
  for (auto& p : pending) nbits += p->bf_len;
  // packed layout (16-byte aligned parts): boffs | rdyn | small | comm | shard | bits
  auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
  const size_t o_boffs = 0, o_rdyn = al((na + 1) * 8), o_small = o_rdyn + al(nrec * 8), o_comm = o_small + 16,
               o_shard = o_comm + al(na * 4), o_bits = o_shard + al(na * 4), total = o_bits + al(nbits) + 16;
  check(g.e_pin.reserve(total));
  uint8_t* h = g.e_pin.p;
  uint64_t* boffs = reinterpret_cast<uint64_t*>(h + o_boffs);
  uint32_t* comm = reinterpret_cast<uint32_t*>(h + o_comm);
  uint32_t* shard = reinterpret_cast<uint32_t*>(h + o_shard);
  uint8_t* bits = h + o_bits;
  boffs[0] = 0;
  for (size_t i = 0; i < na; ++i) {
    const Att& a = *pending[i];
    try {
      comm[i] = attester_committee(g, C, a);
    } catch (Rejected&) {  // stateRecalc returns an error; the caller dereferences a nil state
      throw Panic{"stateRecalc: committee lookup failed -> nil state dereference"};
    }
    if (a.shard > 0xffffffffull) throw Panic{"crosslink record index out of range"};
    shard[i] = (uint32_t)a.shard;
    std::memcpy(bits + boffs[i], a.at(a.bf_off), a.bf_len);
    boffs[i + 1] = boffs[i] + a.bf_len;
  }
  uint64_t* rdyn = reinterpret_cast<uint64_t*>(h + o_rdyn);
  for (size_t s = 0; s < nrec; ++s) rdyn[s] = xl[s].dynasty;
  uint64_t* small = reinterpret_cast<uint64_t*>(h + o_small);
  small[0] = C.dynasty;
  small[1] = C.tdep;
  // the previous epoch was collected (every rank's event completed), so the staging is free
  const uint64_t nred = kScal + 2 * (uint64_t)na;  // {scal, vote, total}: one all-reduce when sharded
  if (g.world == 1) {
    EpochLaunch el =
        epoch_prepare_args(g, C, na, nrec, nbits, o_boffs, o_rdyn, o_small, o_comm, o_shard, o_bits, total, in_place);
    if (out)
      *out = el;
    else
      epoch_launch_rest(g, el);
    return;
  }
  // sharded (world > 1): the transition's ONE collective.  Every rank's xred gets
  // its tally gather (sharded_gather: the justification totals, and in the TotalDeposits slot the
  // previous epoch's pending next-cycle partial -- or, with none pending, rank 0's known
  // TotalDeposits) and this epoch's count-pass partials {scal, vote, total} (every validator is
  // active in a sharded chain, so rank == index and no active-list gather is needed); one
  // all-reduce sums them; then on every range the winners (on the complete tallies) and the
  // rewards (TotalDeposits read from the reduced slot).  The post-reward next-cycle partial
  // waits in nbp for the next all-reduce (the next transition's, or the call's final flush),
  // which hands its sum to the new state (tally_gather_finish).
  if (!q) throw fail(PZ_EINVAL, "sharded epoch without its transition's gather");
  g.deferred.seq = 0;
  const uint64_t o_red = kJustifySlots + 2;
  std::vector<EpochArgs> args;
  const bool carry = g.nb_pending;
  each_rank(g, [&](RankDev& r) {
    sharded_gather(g, r, *q, nred);
    check(r.e_pack.alloc(total));
    hchk(hipMemcpyAsync(r.e_pack.p, h, total, hipMemcpyHostToDevice, r.s), "H2D epoch");
    if (!carry && r.grank == 0)  // (no partial pending: the known TotalDeposits, summed with the others' 0)
      hchk(hipMemcpyAsync(r.xred.p + kJustifySlots + 1, r.e_pack.p + o_small + 8, 8, hipMemcpyDeviceToDevice, r.s),
           "D2D");
    check(r.e_win.alloc(nrec + 1));
    uint64_t* red = r.xred.p + o_red;
    hchk(hipMemsetAsync(red, 0, kScal * 8, r.s), "memset");
    uint8_t* d = r.e_pack.p;
    EpochArgs a;
    std::memset(&a, 0, sizeof a);
    a.ninst = 1;
    a.nval = r.n;
    a.val_offset = r.lo;
    a.nval_global = g.nval;
    a.kind = PZ_KIND_ACTIVE;
    a.balance = r.balance.p;
    a.start = r.start.p;
    a.end = r.end.p;
    a.dynasty = reinterpret_cast<const uint64_t*>(d + o_small);
    a.total_deposit = r.xred.p + kJustifySlots + 1;  // (read by the reward pass, after the all-reduce)
    a.natt = (uint32_t)na;
    a.bits = d + o_bits;
    a.boffs = reinterpret_cast<const uint64_t*>(d + o_boffs);
    a.max_inst_bytes = nbits;
    a.pop_rank = (uint32_t)r.grank;
    a.pop_world = (uint32_t)g.world;
    // the members inside [lo, hi) with their committee positions (rank 0 also keeps any member
    // >= nval, whose processCrosslinks panic it raises)
    a.committee = r.lcomm.p;
    a.coffs = r.lcoffs.p;
    a.cpos = r.lcpos.p;
    a.att_comm = reinterpret_cast<const uint32_t*>(d + o_comm);
    a.att_shard = reinterpret_cast<const uint32_t*>(d + o_shard);
    a.nrec = (uint32_t)nrec;
    a.rec_dynasty = reinterpret_cast<const uint64_t*>(d + o_rdyn);
    a.winner = r.e_win.p;
    a.scal = red;
    a.vote = red + kScal;
    a.total = red + kScal + na;
    a.act_mask = r.e_mask.p;
    a.blk_cnt = r.e_blk.p;
    a.act_list = r.e_list.p;
    hchk(launch_epoch_count(a, true, true, true, r.s), "epoch count");
    args.push_back(a);
  });
  sharded_allreduce(g, nred);
  for (size_t i = 0; i < g.rk.size(); ++i) {
    RankDev& r = g.rk[i];
    hchk(hipSetDevice(r.dev), "hipSetDevice");
    hchk(launch_epoch_mid(args[i], args[i].nrec > 0 && na > 0, false, r.s), "epoch mid");
    hchk(launch_epoch_reward(args[i], r.s), "epoch reward");
    hchk(hipMemcpyAsync(r.nbp.p, args[i].scal + kNextBal, 8, hipMemcpyDeviceToDevice, r.s), "D2D");
  }
  RankDev& r0 = g.rk[0];
  hchk(hipSetDevice(r0.dev), "hipSetDevice");
  check(g.e_pin_out.reserve(kScal * 8 + nrec * 4 + 16));
  hchk(hipMemcpyAsync(g.e_pin_out.p, args[0].scal, kScal * 8, hipMemcpyDeviceToHost, r0.s), "D2H");
  if (nrec) hchk(hipMemcpyAsync(g.e_pin_out.p + kScal * 8, r0.e_win.p, nrec * 4, hipMemcpyDeviceToHost, r0.s), "D2H");
  each_rank(g, [&](RankDev& r) {
    if (!r.ev_epoch) hchk(hipEventCreateWithFlags(&r.ev_epoch, hipEventDisableTiming), "event");
    hchk(hipEventRecord(r.ev_epoch, r.s), "event");
  });
  g.deferred.nrec = nrec;
}

// The deferred epoch's results, once its event has completed: the reference's panics, the
// crosslink winners (core.go:549-555) and the next-cycle balance (TotalDeposits of the state
// it built).  Called before anything reads them: the next transition, the state bytes, the
// roots, and the end of every pz_chain_process_blocks call (so a panic fails that call).
static void epoch_collect(Engine& g) {
  Engine::DeferredEpoch& D = g.deferred;
  if (!D.live) return;
  D.live = false;
  if (D.seq) {  // one rank: poll the reward pass's sequence word (written last), bounded
    const volatile uint64_t* sq = reinterpret_cast<const volatile uint64_t*>(g.e_pin_out.p) + kScal + (D.nrec + 1) / 2;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0; *sq != D.seq; ++k) {
      __builtin_ia32_pause();
      if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
    }
    if (*sq != D.seq) {  // not yet (or an error): the stream decides
      g.prof[kProfPollFallback] += 1;
      hchk(hipStreamSynchronize(g.rk[0].s), "stream sync (epoch)");
      if (*sq != D.seq) throw (int)fail(PZ_EDEVICE, "epoch results never arrived (sequence %llu)", (unsigned long long)D.seq);
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  } else {
    for (RankDev& r : g.rk) hchk(hipEventSynchronize(r.ev_epoch), "event sync (epoch)");
  }
  uint64_t scal[kScal];
  std::memcpy(scal, g.e_pin_out.p, sizeof scal);
  const uint32_t* win = reinterpret_cast<const uint32_t*>(g.e_pin_out.p + sizeof scal);
  std::vector<AttP> pending;
  pending.swap(D.pending);
  CState& C = *D.src;
  std::vector<Crosslink>& xl = *C.xl;
  // The epoch is collected up to 63 blocks after its transition (or at the end of the call), so
  // a panic names the transition block; the result rows of the blocks after it are undefined
  // (the reference stops at that block; include/prysm_hip.h, pz_chain_process_blocks).
  char where[160];
  snprintf(where, sizeof where, " (stateRecalc of block %llu of this call, slot %llu; result rows after that block are undefined)",
           (unsigned long long)D.block_index, (unsigned long long)D.block_slot);
  if (scal[kErrXl])
    throw Panic{std::string("processCrosslinks: index out of range (committee member, bitfield or shard)") + where};
  const uint64_t dep = scal[kPop] * PZ_DEFAULT_BALANCE;
  const bool thr = dep * 3ull >= C.tdep * 2ull;
  if (thr && scal[kNact] > 0 && scal[kErrRwd])
    throw Panic{std::string("CalculateRewards: CheckBit index out of range (incentives.go:23)") + where};
  if (!pending.empty() && !xl.empty()) {
    for (size_t s = 0; s < xl.size() && s < D.nrec; ++s) {
      if (win[s] == 0xffffffffu) continue;
      const Att& w = *pending[win[s]];
      xl[s].dynasty = C.dynasty;
      xl[s].hash.assign((const char*)w.at(w.sbh_off), w.sbh_len);
      xl[s].slot = D.block_slot;
    }
  }
  if (scal[kApplied]) g.val_enc_valid = false;
  if (g.world == 1) D.dst->tdep = scal[kNextBal];  // (sharded: a partial per rank, summed by the next all-reduce)
  D.src.reset();
  D.dst.reset();
}

// stateRecalc (core.go:398-497) -> (new C, new A).
static void state_recalc(Engine& g, const CP& C, const AP& A, uint64_t block_slot, uint64_t block_index, CP* nc_out,
                         AP* na_out) {
  // The previous transition's epoch first: this one reads the crosslink records and the
  // TotalDeposits it produced (long since done: 64 blocks of walk have passed).
  epoch_collect(g);
  // The host waits only for what the justification loop reads (core.go:411-431): the pending
  // vote tallies and the D2H of their totals.  The device epoch (processCrosslinks,
  // CalculateRewards, next balance) does not depend on it and is enqueued behind them, to be
  // collected at the next transition; the stream orders every later tally after its rewards.
  VoteGatherSlots q;
  for (uint64_t i = 0; i < kCycle; ++i) {
    q.slot[i] = UINT32_MAX;
    if (!A->cache_nil && i < A->len) {
      if (const uint32_t* sl = g.slot_of.find(g.hlog[recent_id(g, *A, i)])) q.slot[i] = *sl;
    }
  }
  // one rank: the epoch is prepared inside the flush (before its tally launch)
  const bool one = g.world == 1;
  EpochLaunch el;
  const EpochPrep prep = [&]() -> EpochLaunch* {
    epoch_enqueue(g, *C, A->pending, &el, true);
    return &el;
  };
  // The tally is launched first and the epoch packed while it runs (its count pass then a
  // launch of its own): the pack's host time is off the justification loop's wait (totals_wait
  // 3.5 -> 2.4 ms per 10,000 blocks, profiles/r04/replay_prep_ab_r4n.txt).  PZ_EPOCH_PREP=merged
  // (A/B, read per call): pack first, the count blocks inside the tally launch.
  const bool prep_after = g.kn.epoch_prep_after;
  std::array<uint64_t, 4> tl{mono_ns(), 0, 0, 0};
  const bool gathered = flush_votes_enqueue(g, &q, one && !prep_after ? &prep : nullptr);
  tl[1] = mono_ns();
  PhaseTimer pt(g.prof[kProfRecalc]);
  uint64_t streak = C->streak, justified = C->jslot, finalized = C->fslot;
  const uint64_t lsr = C->lsr;
  std::vector<uint64_t> tot(kCycle, 0);
  if (one) {
    if (!gathered) tally_gather_enqueue(g, q);
    if (!el.ready) epoch_enqueue(g, *C, A->pending, &el);  // (nothing was flushed)
    epoch_launch_rest(g, el);
  } else {  // the gather, the epoch and ONE all-reduce
    epoch_enqueue(g, *C, A->pending, nullptr, false, &q);
  }
  tl[2] = mono_ns();
  auto nc = std::make_shared<CState>();
  g.deferred.live = true;
  g.deferred.pending = A->pending;
  g.deferred.src = C;
  g.deferred.dst = nc;
  g.deferred.block_slot = block_slot;
  g.deferred.block_index = block_index;
  // (the new ActiveState does not depend on the totals: built while the device tallies)
  auto na = std::make_shared<AState>();
  na->pending.reserve(A->pending.size());
  for (auto& p : A->pending)
    if (p->slot > lsr) na->pending.push_back(p);
  na->tail = A->tail;  // (the window is at most 2 * kCycle long)
  na->len = A->len;
  na->cache_nil = A->cache_nil;
  tally_gather_finish(g);  // (sharded: C's TotalDeposits, if its epoch's partials were pending, set here)
  if (!one) {  // this epoch's next-cycle partials now pending, for the new state
    g.nb_pending = true;
    g.nb_dst = nc;
  }
  tl[3] = mono_ns();
  if (g.tl.size() < (1u << 16)) g.tl.push_back(tl);
  std::memcpy(tot.data(), g.tot_pin.p, kCycle * 8);
  for (uint64_t i = 0; i < kCycle; ++i) {
    const uint64_t slot = lsr - kCycle + i;
    if (3ull * tot[i] >= 2ull * C->tdep) {
      if (slot > justified) justified = slot;
      ++streak;
    } else {
      streak = 0;
    }
    if (streak >= kCycle + 1 && slot - kCycle > finalized) finalized = slot - kCycle;
  }
  nc->lsr = lsr + kCycle;
  nc->jslot = justified;
  nc->streak = streak;
  nc->fslot = finalized;
  nc->start_shard = 0;
  nc->dynasty = 0;  // core.go:467-478 does not set CurrentDynasty
  nc->seed_reset = C->seed_reset;
  nc->tdep = 0;  // the epoch's next-cycle balance, set by epoch_collect
  nc->xl = C->xl;
  *nc_out = nc;
  *na_out = na;
}

// ---- serialization of the states (state roots) --------------------------------------------
static const std::string& validators_enc(Engine& g) {
  if (g.val_enc_valid) return g.val_enc;
  // each rank encodes its range (records are framed one by one, so the ranges' encodings
  // concatenate); across processes the ranges' bytes are all-gathered, padded to the largest
  std::vector<uint64_t> totals(g.rk.size(), 0);
  each_rank(g, [&](RankDev& r) {
    if (!r.n) return;
    pz_validator_cols v{};
    v.balance = r.balance.p;
    v.start_dynasty = r.start.p;
    v.end_dynasty = r.end.p;
    if (g.has_pk) v.public_key = g.pubkey.p;
    if (g.has_ws) v.withdrawal_shard = g.wshard.p;
    if (g.has_wa) { v.withdrawal_address = g.wa.p; v.withdrawal_address_offs = g.wa_offs.p; }
    if (g.has_rc) { v.randao_commitment = g.rc.p; v.randao_commitment_offs = g.rc_offs.p; }
    WireValArgs a;
    check(wire_val_args(&v, r.n, 11, &a));
    const uint64_t bound = pz_wire_validators_bound(r.n, g.val_bytes);
    check(r.w_out.alloc(bound));
    check(r.w_scratch.alloc(wire_tiles(r.n) + 1));
    check(r.w_total.alloc(1));
    a.out = r.w_out.p;
    a.total = r.w_total.p;
    hchk(launch_wire_validators(a, r.w_scratch.p, r.s), "pz_wire_val_kernel");
  });
  each_rank(g, [&](RankDev& r) {
    if (!r.n) return;
    uint64_t t = 0;
    hchk(hipMemcpyAsync(&t, r.w_total.p, 8, hipMemcpyDeviceToHost, r.s), "D2H");
    hchk(hipStreamSynchronize(r.s), "sync");
    totals[&r - g.rk.data()] = t;
  });
  g.val_enc.clear();
  if (g.world == (int)g.rk.size()) {  // every range is in this process
    for (size_t i = 0; i < g.rk.size(); ++i) {
      RankDev& r = g.rk[i];
      if (!totals[i]) continue;
      const size_t at = g.val_enc.size();
      g.val_enc.resize(at + totals[i]);
      hchk(hipSetDevice(r.dev), "hipSetDevice");
      hchk(hipMemcpyAsync(&g.val_enc[at], r.w_out.p, totals[i], hipMemcpyDeviceToHost, r.s), "D2H");
      hchk(hipStreamSynchronize(r.s), "sync");
    }
  } else {  // one local rank per process: all-gather the lengths, then the padded encodings
    RankDev& r = g.rk[0];
    hchk(hipSetDevice(r.dev), "hipSetDevice");
    DevArr<uint64_t> len1, lens;
    check(len1.alloc(1));
    check(lens.alloc(g.world));
    hchk(hipMemcpyAsync(len1.p, &totals[0], 8, hipMemcpyHostToDevice, r.s), "H2D");
    hipEvent_t ev;
    hchk(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
    const void* snd = len1.p;
    void* rcv = lens.p;
    int rc = g.comm->allgather(&snd, &rcv, 8, &r.s, &ev);
    std::vector<uint64_t> all(g.world);
    if (!rc) {
      hchk(hipStreamWaitEvent(r.s, ev, 0), "wait");
      hchk(hipMemcpyAsync(all.data(), lens.p, g.world * 8, hipMemcpyDeviceToHost, r.s), "D2H");
      hchk(hipStreamSynchronize(r.s), "sync");
    }
    uint64_t mx = 1;
    for (uint64_t x : all) mx = std::max(mx, x);
    DevArr<uint8_t> pad, gath;
    if (!rc) {
      check(pad.alloc(mx));
      check(gath.alloc(mx * g.world));
      if (totals[0]) hchk(hipMemcpyAsync(pad.p, r.w_out.p, totals[0], hipMemcpyDeviceToDevice, r.s), "D2D");
      const void* s2 = pad.p;
      void* r2 = gath.p;
      rc = g.comm->allgather(&s2, &r2, mx, &r.s, &ev);
    }
    if (!rc) {
      std::vector<uint8_t> hostg(mx * g.world);
      hchk(hipStreamWaitEvent(r.s, ev, 0), "wait");
      hchk(hipMemcpyAsync(hostg.data(), gath.p, hostg.size(), hipMemcpyDeviceToHost, r.s), "D2H");
      hchk(hipStreamSynchronize(r.s), "sync");
      for (int w = 0; w < g.world; ++w) g.val_enc.append((const char*)hostg.data() + (size_t)w * mx, all[w]);
    }
    (void)hipEventDestroy(ev);
    check(rc);
  }
  g.val_enc_valid = true;
  return g.val_enc;
}

static std::string encode_active(const Engine& g, const AState& A) {  // messages.proto:94-97
  std::string o;
  for (auto& p : A.pending) put_msg(o, 1, p->base, p->len);
  for (uint32_t i = 0; i < A.len; ++i) put_msg(o, 2, g.hlog[recent_id(g, A, i)].b, A.recent_raw_empty ? 0 : 32);
  return o;
}

static std::string encode_crystallized(Engine& g, const CState& C) {  // messages.proto:59-72
  const std::string& venc = validators_enc(g);
  std::string o;
  o.reserve(venc.size() + g.arrays_enc.size() + 16384);
  put_u(o, 1, C.lsr);
  put_u(o, 2, C.streak);
  put_u(o, 3, C.jslot);
  put_u(o, 4, C.fslot);
  put_u(o, 5, C.dynasty);
  put_u(o, 6, C.start_shard);
  put_u(o, 7, C.tdep);
  put_b(o, 8, (const uint8_t*)C.seed.data(), C.seed.size());
  put_u(o, 9, C.seed_reset);
  std::string r;
  for (auto& x : *C.xl) {
    r.clear();
    put_u(r, 1, x.dynasty);
    put_b(r, 2, (const uint8_t*)x.hash.data(), x.hash.size());
    put_u(r, 3, x.slot);
    put_msg(o, 10, (const uint8_t*)r.data(), r.size());
  }
  o += venc;  // ValidatorRecords
  o += g.arrays_enc;
  return o;
}

// Uploads the validators and committees and installs the chain's states: C, and the genesis
// ActiveState (types/state.go:46-57), which is also what NewBeaconChain keeps when it reloads
// a stored CrystallizedState (blockchain/core.go:59-64).
static void init_tail(Engine& g, const std::vector<uint32_t>& members, const std::vector<uint64_t>& offs, const CP& C) {
  const uint64_t n = g.nval;
  g.csize.resize(offs.size() - 1);
  for (size_t c = 0; c + 1 < offs.size(); ++c) g.csize[c] = offs[c + 1] - offs[c];
  g.ncomm = g.csize.size();
  g.h_coffs = offs;
  uint64_t kmax = 0;
  for (uint64_t k : g.csize) kmax = std::max(kmax, k);
  g.bf_stride = (uint32_t)std::max<uint64_t>(4, ((kmax + 7) / 8 + 3) & ~3ull);
  // (pz_chain_options.tally_forms, tests: every bitfield in the row array, every attestation's
  // ids in an explicit row)
  g.kmax = kmax;
  g.bits_inline = kmax <= kVoteInlineBits && !(g.opt.tally_forms & PZ_TALLY_BITS_ROWS);
  g.ids_rows = (g.opt.tally_forms & PZ_TALLY_ID_ROWS) != 0;
  if (offs.back() >= (1ull << 32)) throw (int)fail(PZ_EINVAL, "committee lists above 2^32 members");
  // 64-aligned validator ranges, as pz_epoch_state / pz_comm_vote_tally split them
  const uint64_t span = 64 * std::max<uint64_t>(1, (n + 64ull * g.world - 1) / (64ull * g.world));
  each_rank(g, [&](RankDev& r) {
    r.lo = std::min<uint64_t>(n, (uint64_t)r.grank * span);
    r.hi = std::min<uint64_t>(n, (uint64_t)(r.grank + 1) * span);
    if (g.world == 1) r.lo = 0, r.hi = n;
    r.n = r.hi - r.lo;
    upload(r, r.committee, members.data(), members.size());
    upload(r, r.coffs, offs.data(), offs.size());
    upload(r, r.balance, g.h_balance.data() + r.lo, r.n);
    upload(r, r.start, g.h_start.data() + r.lo, r.n);
    upload(r, r.end, g.h_end.data() + r.lo, r.n);
    if (g.world > 1) {  // the members inside [lo, hi) and their committee positions
      std::vector<uint32_t> mem, pos;
      std::vector<uint64_t> lo_offs(offs.size(), 0);
      for (size_t c = 0; c + 1 < offs.size(); ++c) {
        for (uint64_t k = offs[c]; k < offs[c + 1]; ++k) {
          const uint32_t v = members[k];
          if ((v >= r.lo && v < r.hi) || (r.grank == 0 && v >= n)) {
            mem.push_back(v);
            pos.push_back((uint32_t)(k - offs[c]));
          }
        }
        lo_offs[c + 1] = mem.size();
      }
      mem.push_back(0);
      pos.push_back(0);
      upload(r, r.lcomm, mem.data(), mem.size());
      upload(r, r.lcpos, pos.data(), pos.size());
      upload(r, r.lcoffs, lo_offs.data(), lo_offs.size());
    }
    check(r.e_mask.alloc((r.n + 63) / 64 + 1));
    check(r.e_blk.alloc(vblocks_per_inst(r.n) + 1));
    check(r.e_list.alloc(r.n + 1));
    hchk(hipStreamSynchronize(r.s), "sync");
  });
  auto A = std::make_shared<AState>();
  msg_drain(g);
  g.hlog.reset();
  g.id_slot.clear();
  g.d_hlog_n = 0;
  const uint32_t zero_id = log_hash(g, kZero);
  g.trail.assign(2 * kCycle, zero_id);
  ++g.trail_gen;
  g.d_trail_n = 0;
  A->tail = g.trail.size();
  A->len = (uint32_t)(2 * kCycle);
  A->recent_raw_empty = true;
  g.A = A;
  g.C = C;
}

// ---- genesis (types/state.go:44-112) -------------------------------------------------------
static int genesis(Engine& g) {
  const uint64_t n = g.nval;
  g.h_balance.assign(n, PZ_DEFAULT_BALANCE);
  g.h_start.assign(n, 0);
  g.h_end.assign(n, PZ_DEFAULT_END_DYNASTY);
  // ShuffleValidatorsToCommittees(BytesToHash(empty seed), validators, 1, 0) (sharding.go:11-21)
  std::vector<uint32_t> idx(n);
  for (uint64_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
  uint8_t seed[32] = {0};
  int rc = pz_shuffle_indices(seed, idx.data(), n);
  if (rc) return rc;
  // getCommitteeParams (sharding.go:60-73)
  uint64_t cps, spc = 1;
  if (n >= kCycle * PZ_MIN_COMMITTEE_SIZE) {
    cps = n / (kCycle * PZ_MIN_COMMITTEE_SIZE * 2) + 1;
  } else {
    cps = 1;
    while (n * spc < PZ_MIN_COMMITTEE_SIZE * kCycle && spc < kCycle) spc *= 2;
  }
  // splitBySlotShard (sharding.go:27-53): 64 slot arrays; the genesis repeats them 4 times
  std::vector<uint32_t> members;
  std::vector<uint64_t> offs{0};
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> base(kCycle);
  std::string arr_enc[kCycle];
  for (uint64_t i = 0; i < kCycle; ++i) {
    const uint64_t s0 = n * i / kCycle, s1 = n * (i + 1) / kCycle, len = s1 - s0;
    const uint64_t shard_start = i * cps / spc;
    for (uint64_t j = 0; j < cps; ++j) {
      const uint64_t c0 = s0 + len * j / cps, c1 = s0 + len * (j + 1) / cps;
      const uint64_t shard = (shard_start + j) % PZ_SHARD_COUNT;
      const uint32_t cid = (uint32_t)(offs.size() - 1);
      members.insert(members.end(), idx.begin() + (ptrdiff_t)c0, idx.begin() + (ptrdiff_t)c1);
      offs.push_back(members.size());
      base[i].push_back({shard, cid});
      std::string sc, packed;
      put_u(sc, 1, shard);
      for (uint64_t q = c0; q < c1; ++q) put_varint(packed, idx[q]);
      if (!packed.empty()) put_msg(sc, 2, (const uint8_t*)packed.data(), packed.size());
      put_msg(arr_enc[i], 1, (const uint8_t*)sc.data(), sc.size());
    }
  }
  g.lookup.clear();
  g.arrays_enc.clear();
  for (int rep = 0; rep < 4; ++rep)
    for (uint64_t i = 0; i < kCycle; ++i) {
      g.lookup.push_back(base[i]);
      put_msg(g.arrays_enc, 12, (const uint8_t*)arr_enc[i].data(), arr_enc[i].size());
    }
  auto C = std::make_shared<CState>();
  C->dynasty = 1;
  C->tdep = n * PZ_DEFAULT_BALANCE;
  C->xl = std::make_shared<std::vector<Crosslink>>(PZ_SHARD_COUNT);
  init_tail(g, members, offs, C);
  return PZ_OK;
}

// ---- reload: NewBeaconChain with a stored CrystallizedState (blockchain/core.go:86-95) -------
// proto.Unmarshal accepts any valid encoding (field order, unpacked repeated scalars, unknown
// fields), so this reader is lenient, unlike the canonical-only block Reader.
struct LRd {
  const uint8_t* p;
  const uint8_t* e;
  bool bad = false;
  uint64_t var() {
    uint64_t x = 0;
    for (int s = 0; s < 64 && p < e; s += 7) {
      const uint8_t c = *p++;
      x |= (uint64_t)(c & 0x7F) << s;
      if (!(c & 0x80)) return x;
    }
    bad = true;
    return 0;
  }
  LRd sub() {
    const uint64_t n = var();
    if (bad || (uint64_t)(e - p) < n) { bad = true; return LRd{p, p}; }
    LRd r{p, p + n};
    p += n;
    return r;
  }
  void skip(uint32_t wt) {
    if (wt == 0) var();
    else if (wt == 2) sub();
    else if (wt == 1 && e - p >= 8) p += 8;
    else if (wt == 5 && e - p >= 4) p += 4;
    else bad = true;
  }
};

static int reload(Engine& g, const uint8_t* data, uint64_t len) {
  auto C = std::make_shared<CState>();
  C->xl = std::make_shared<std::vector<Crosslink>>();
  std::vector<uint64_t> pk, ws;
  std::string wa_bytes, rc_bytes;
  std::vector<uint64_t> wa_offs{0}, rc_offs{0};
  // ShardAndCommitteesForSlots: arrays of (shard, members); identical committees share an id
  std::map<std::vector<uint32_t>, uint32_t> comm_id;
  std::vector<uint32_t> members;
  std::vector<uint64_t> offs{0};
  g.lookup.clear();
  g.arrays_enc.clear();
  LRd r{data, data + len};
  while (r.p < r.e && !r.bad) {
    const uint64_t key = r.var();
    const uint32_t f = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (wt == 0 && f >= 1 && f <= 9 && f != 8) {
      const uint64_t v = r.var();
      switch (f) {
        case 1: C->lsr = v; break;
        case 2: C->streak = v; break;
        case 3: C->jslot = v; break;
        case 4: C->fslot = v; break;
        case 5: C->dynasty = v; break;
        case 6: C->start_shard = v; break;
        case 7: C->tdep = v; break;
        default: C->seed_reset = v;
      }
    } else if (wt == 2 && f == 8) {
      LRd b = r.sub();
      C->seed.assign((const char*)b.p, b.e - b.p);
    } else if (wt == 2 && f == 10) {  // CrosslinkRecord (messages.pb.go:983-985)
      LRd m = r.sub();
      Crosslink x;
      while (m.p < m.e && !m.bad) {
        const uint64_t k = m.var();
        if (k == (1 << 3)) x.dynasty = m.var();
        else if (k == ((2 << 3) | 2)) { LRd b = m.sub(); x.hash.assign((const char*)b.p, b.e - b.p); }
        else if (k == (3 << 3)) x.slot = m.var();
        else m.skip((uint32_t)(k & 7));
      }
      r.bad |= m.bad;
      C->xl->push_back(std::move(x));
    } else if (wt == 2 && f == 11) {  // ValidatorRecord (messages.pb.go:803-809)
      LRd m = r.sub();
      uint64_t col[8] = {};
      std::string wab, rcb;
      while (m.p < m.e && !m.bad) {
        const uint64_t k = m.var();
        const uint32_t ff = (uint32_t)(k >> 3), ww = (uint32_t)(k & 7);
        if (ww == 0 && (ff == 1 || ff == 2 || (ff >= 5 && ff <= 7))) col[ff] = m.var();
        else if (ww == 2 && ff == 3) { LRd b = m.sub(); wab.assign((const char*)b.p, b.e - b.p); }
        else if (ww == 2 && ff == 4) { LRd b = m.sub(); rcb.assign((const char*)b.p, b.e - b.p); }
        else m.skip(ww);
      }
      r.bad |= m.bad;
      pk.push_back(col[1]);
      ws.push_back(col[2]);
      g.h_balance.push_back(col[5]);
      g.h_start.push_back(col[6]);
      g.h_end.push_back(col[7]);
      wa_bytes += wab;
      wa_offs.push_back(wa_bytes.size());
      rc_bytes += rcb;
      rc_offs.push_back(rc_bytes.size());
    } else if (wt == 2 && f == 12) {  // ShardAndCommitteeArray (messages.pb.go:559, 673-674)
      LRd m = r.sub();
      std::vector<std::pair<uint64_t, uint32_t>> arr;
      std::string arr_enc;
      while (m.p < m.e && !m.bad) {
        const uint64_t k = m.var();
        if (k != ((1 << 3) | 2)) { m.skip((uint32_t)(k & 7)); continue; }
        LRd q = m.sub();
        uint64_t shard = 0;
        std::vector<uint32_t> mem;
        while (q.p < q.e && !q.bad) {
          const uint64_t kk = q.var();
          if (kk == (1 << 3)) shard = q.var();
          else if (kk == ((2 << 3) | 2)) { LRd pk2 = q.sub(); while (pk2.p < pk2.e && !pk2.bad) mem.push_back((uint32_t)pk2.var()); q.bad |= pk2.bad; }
          else if (kk == (2 << 3)) mem.push_back((uint32_t)q.var());
          else q.skip((uint32_t)(kk & 7));
        }
        m.bad |= q.bad;
        auto it = comm_id.find(mem);
        uint32_t cid;
        if (it == comm_id.end()) {
          cid = (uint32_t)(offs.size() - 1);
          comm_id.emplace(mem, cid);
          members.insert(members.end(), mem.begin(), mem.end());
          offs.push_back(members.size());
        } else {
          cid = it->second;
        }
        arr.push_back({shard, cid});
        std::string sc, packed;
        put_u(sc, 1, shard);
        for (uint32_t v : mem) put_varint(packed, v);
        if (!packed.empty()) put_msg(sc, 2, (const uint8_t*)packed.data(), packed.size());
        put_msg(arr_enc, 1, (const uint8_t*)sc.data(), sc.size());
      }
      r.bad |= m.bad;
      g.lookup.push_back(std::move(arr));
      put_msg(g.arrays_enc, 12, (const uint8_t*)arr_enc.data(), arr_enc.size());
    } else {
      r.skip(wt);
    }
  }
  if (r.bad) return fail(PZ_EINVAL, "stored CrystallizedState does not decode (proto.Unmarshal error)");
  g.nval = g.h_balance.size();
  if (g.nval == 0 || g.nval > PZ_MAX_VALIDATORS)
    return fail(PZ_EINVAL, "stored state holds %llu validators", (unsigned long long)g.nval);
  // (a committee member >= len(validators) panics where Go indexes it, not here)
  auto any = [](const std::vector<uint64_t>& c) { for (uint64_t x : c) if (x) return true; return false; };
  g.has_pk = any(pk);
  g.has_ws = any(ws);
  g.has_wa = !wa_bytes.empty();
  g.has_rc = !rc_bytes.empty();
  g.val_bytes = wa_bytes.size() + rc_bytes.size();
  if (g.has_pk) upload(g, g.pubkey, pk.data(), pk.size());
  if (g.has_ws) upload(g, g.wshard, ws.data(), ws.size());
  if (g.has_wa) { upload(g, g.wa, (const uint8_t*)wa_bytes.data(), wa_bytes.size()); upload(g, g.wa_offs, wa_offs.data(), wa_offs.size()); }
  if (g.has_rc) { upload(g, g.rc, (const uint8_t*)rc_bytes.data(), rc_bytes.size()); upload(g, g.rc_offs, rc_offs.data(), rc_offs.size()); }
  init_tail(g, members, offs, C);
  return PZ_OK;
}

// ---- blockProcessing (service.go:238-363) ---------------------------------------------------
// Parsed on the calling thread, into one arena per call.  (On host threads, with a heap
// record per attestation, the parse itself was 2x slower -- the allocator shared by the
// threads -- and the walk that reads the records 10-20 % slower: records left in other cores'
// caches; profiles/r03/replay_threads_r3c.txt.)
// The call's arena: a copy of the input bytes (filled by whoever parses them), the records
// sized to the per-block counts (`first`, n + 1 entries), `npools` oblique pools.
static std::shared_ptr<CallArena> make_arena(const uint64_t* offs, uint64_t n, std::vector<uint64_t>&& first,
                                             size_t npools, PinBuf* pin = nullptr) {
  auto ar = std::make_shared<CallArena>();
  const uint64_t total = n ? offs[n] - offs[0] : 0;
  if (pin) {
    check(pin->reserve(total + 16));
    ar->bytes = pin->p;
  } else {
    ar->own.reset(new uint8_t[total + 16]);
    ar->bytes = ar->own.get();
  }
  std::memset(ar->bytes + total, 0, 16);
  ar->first = std::move(first);
  const uint64_t natt = ar->first.empty() ? 0 : ar->first.back();
  ar->atts.alloc(natt);
  ar->ptrs.resize(natt);
  ar->obl.resize(std::max<size_t>(npools, 1));
  return ar;
}

// Blocks [i0, i1): their record counts (field 8 of BeaconBlock, messages.pb.go:224-232) into
// cnt[i + 1]; returns the first block whose offsets are not monotone, or i1.
static uint64_t count_range(const uint8_t* data, const uint64_t* offs, uint64_t i0, uint64_t i1, uint64_t* cnt) {
  for (uint64_t i = i0; i < i1; ++i) {
    if (offs[i + 1] < offs[i]) return i;
    Reader r{data + offs[i], data + offs[i + 1]};
    uint64_t c = 0;
    while (r.more()) {
      const uint64_t key = r.varint();
      if ((key >> 3) == 8 && (key & 7) == 2) ++c;
      r.skip((uint32_t)(key & 7));
    }
    cnt[i + 1] = c;
  }
  return i1;
}

// Blocks [b0, b1): copied into the arena and parsed, their oblique hashes into pool `pl`
// (reserved here); returns the first malformed block or b1.
static uint64_t parse_range(const uint8_t* data, const uint64_t* offs, uint64_t b0, uint64_t b1, CallArena& ar,
                            std::vector<Block>& blocks, size_t pl) {
  const uint64_t o0 = offs[0];
  for (uint64_t i = b0; i < b1; ++i)
    if (offs[i + 1] < offs[i]) return i;
  if (b1 > b0) std::memcpy(ar.bytes + (offs[b0] - o0), data + offs[b0], offs[b1] - offs[b0]);
  CallArena::Pool& pool = ar.obl[pl];
  pool.reserve((offs[b1] - offs[b0]) / 2 + 1);
  const uint8_t* base = ar.bytes - o0;
  for (uint64_t i = b0; i < b1; ++i)
    if (!parse_block(base + offs[i], offs[i + 1] - offs[i], &blocks[i], &ar, i, pool)) return i;
  return b1;
}

// Threads for the parse of a call of `bytes` input bytes: at most pz_set_host_threads (the
// bench boxes' CPU share of one GPU is 16), one per 512 KB (10,000 blocks: 1.76 ms on 8,
// 1.22 ms on 16, profiles/r03/parse_probe_after_r3at.txt).
static int parse_threads(uint64_t bytes) {
  const uint64_t cap = host_threads();  // (pz_set_host_threads)
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(cap, bytes >> 19));
}

// The parse's worker threads, started once per process and kept (starting eight threads per
// call showed as 2 % of the replay's samples in pthread_create, profiles/r03/walk_sampler_r3av.txt).
// Never destroyed, like the pinned pool: idle workers wait on a condition variable.
struct WorkPool {
  std::mutex mu;
  std::condition_variable cv, done;
  std::vector<std::function<void()>> jobs;
  size_t next = 0, left = 0;
  int threads = 0;
  bool failed = false;
  std::mutex run_mu;  // one batch at a time (chains on other threads share the pool)
  // Runs fns[1..] on the workers and fns[0] here; returns when all are done.  Throws (PZ_EDEVICE
  // semantics: check's int) when a job threw.
  void run(std::vector<std::function<void()>>& fns) {
    std::lock_guard<std::mutex> one(run_mu);
    {
      std::unique_lock<std::mutex> lk(mu);
      while (threads < (int)fns.size() - 1) {
        std::thread([this] { work(); }).detach();
        ++threads;
      }
      jobs.assign(fns.begin() + 1, fns.end());
      next = 0;
      left = jobs.size();
      failed = false;
    }
    cv.notify_all();
    bool mine_failed = false;
    try {
      fns[0]();
    } catch (...) {
      mine_failed = true;
    }
    std::unique_lock<std::mutex> lk(mu);
    done.wait(lk, [this] { return left == 0; });
    jobs.clear();
    if (mine_failed || failed) throw (int)PZ_EDEVICE;
  }
  void work() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [this] { return next < jobs.size(); });
      // by pointer: the batch's vector is only cleared after every job has finished (run()), and a
      // copy here would sit outside the try (a throwing copy would end the process)
      std::function<void()>* f = &jobs[next++];
      lk.unlock();
      bool bad = false;
      try {
        (*f)();
      } catch (...) {
        bad = true;
      }
      lk.lock();
      if (bad) failed = true;
      if (--left == 0) done.notify_all();
    }
  }
};
// A forked child has none of the parent's workers (and maybe a locked mutex): it starts a pool
// of its own on first use.
static std::atomic<WorkPool*> g_work_pool{nullptr};
static void work_pool_after_fork() { g_work_pool.store(nullptr); }
static WorkPool& work_pool() {
  static const bool hooked = (pthread_atfork(nullptr, nullptr, work_pool_after_fork), true);
  (void)hooked;
  WorkPool* p = g_work_pool.load();
  if (!p) {
    static std::mutex mk;
    std::lock_guard<std::mutex> lk(mk);
    if (!(p = g_work_pool.load())) g_work_pool.store(p = new WorkPool());
  }
  return *p;
}

// Records per block as the prefix `first` (n + 1 entries); PZ_EINVAL when the offsets are not
// monotone.  The canonical-form checks are the parser's.  Large calls count on the worker pool
// (the count runs twice per call from Python, once to size the results: 0.3 ms each serially
// per 10,000 blocks).
static int count_per_block(const uint8_t* data, const uint64_t* offs, uint64_t n, std::vector<uint64_t>& first) {
  first.assign(n + 1, 0);
  const uint64_t bytes = n && offs[n] >= offs[0] ? offs[n] - offs[0] : 0;
  const uint64_t T = n >= 2048 ? std::min<uint64_t>((uint64_t)parse_threads(bytes), n / 1024) : 1;
  uint64_t bad = n;
  if (T <= 1) {
    bad = count_range(data, offs, 0, n, first.data());
  } else {
    std::vector<uint64_t> b(T, UINT64_MAX);
    std::vector<std::function<void()>> fns;
    for (uint64_t t = 0; t < T; ++t)
      fns.push_back([&, t] { b[t] = count_range(data, offs, n * t / T, n * (t + 1) / T, first.data()); });
    try {
      work_pool().run(fns);
      for (uint64_t t = 0; t < T; ++t)
        if (b[t] < n * (t + 1) / T) {
          bad = b[t];
          break;
        }
    } catch (const std::system_error&) {  // no thread to be had
      bad = count_range(data, offs, 0, n, first.data());
    } catch (int code) {  // a worker's job threw (WorkPool::run): both C-ABI callers return it
      return fail(code, "block count: a worker thread failed");
    }
  }
  if (bad < n) return fail(PZ_EINVAL, "offsets not monotone");
  for (uint64_t i = 0; i < n; ++i) first[i + 1] += first[i];
  return PZ_OK;
}

// Blocks [0, n) over ar.obl.size() threads (ranges of about equal bytes; records need no
// allocation, so the threads share nothing but the arena's disjoint ranges); returns the first
// malformed block or n.
static uint64_t parse_parallel(const uint8_t* data, const uint64_t* offs, uint64_t n, CallArena& ar,
                               std::vector<Block>& blocks) {
  const size_t T = ar.obl.size();
  if (T <= 1 || n < 2 * T) return parse_range(data, offs, 0, n, ar, blocks, 0);
  for (uint64_t i = 0; i < n; ++i)
    if (offs[i + 1] < offs[i]) return i;
  std::vector<uint64_t> cut(T + 1, n);
  cut[0] = 0;
  const uint64_t total = offs[n] - offs[0];
  for (size_t t = 1; t < T; ++t) {
    const uint64_t want = offs[0] + total / T * t;
    cut[t] = std::max<uint64_t>(cut[t - 1], std::lower_bound(offs, offs + n, want) - offs);
  }
  std::vector<uint64_t> bad(T, UINT64_MAX);
  std::vector<std::function<void()>> fns;
  for (size_t t = 0; t < T; ++t)
    fns.push_back([&, t] { bad[t] = parse_range(data, offs, cut[t], cut[t + 1], ar, blocks, t); });
  try {
    work_pool().run(fns);
  } catch (const std::system_error&) {  // no thread to be had: every range on this one
    for (size_t t = 0; t < T; ++t) bad[t] = parse_range(data, offs, cut[t], cut[t + 1], ar, blocks, t);
  }
  for (size_t t = 0; t < T; ++t)
    if (bad[t] < cut[t + 1]) return bad[t];
  return n;
}

// After a call: the records a live state still holds (the pending attestations of the
// chain's, the candidate's and the deferred epoch's states) move out of the call's arena --
// the Engine's pinned buffer, which the next call reuses -- into a small heap arena of their
// own; earlier such arenas stay while a live record points into them.
static void keep_arenas(Engine& g, CallArena* cur) {
  std::vector<std::vector<AttP>*> lists;
  if (g.A) lists.push_back(&g.A->pending);
  if (g.cand_A) lists.push_back(&g.cand_A->pending);
  if (g.deferred.live) lists.push_back(&g.deferred.pending);
  if (cur && !cur->atts.empty()) {
    const Att* lo = cur->atts.data();
    const Att* hi = lo + cur->atts.size();
    std::vector<AttP> mv;
    for (auto* l : lists)
      for (AttP p : *l)
        if (p >= lo && p < hi) mv.push_back(p);
    std::sort(mv.begin(), mv.end());
    mv.erase(std::unique(mv.begin(), mv.end()), mv.end());
    if (!mv.empty()) {
      auto na = std::make_shared<CallArena>();
      size_t bytes = 0, nobl = 0;
      for (AttP p : mv) {
        bytes += p->len;
        nobl += p->obl.n;
      }
      na->own.reset(new uint8_t[bytes + 16]);
      na->bytes = na->own.get();
      std::memset(na->bytes + bytes, 0, 16);
      na->atts.alloc(mv.size());
      na->obl.resize(1);
      na->obl[0].reserve(nobl + 1);
      size_t pos = 0, k = 0;
      for (AttP p : mv) {
        Att a = *p;
        std::memcpy(na->bytes + pos, p->base, p->len);
        a.base = na->bytes + pos;
        pos += p->len;
        a.obl_first = (uint32_t)na->obl[0].size();
        for (auto& o : p->obl) na->obl[0].push_back(o);
        a.obl.p = na->obl[0].data() + a.obl_first;  // (reserved: never reallocates)
        new (&na->atts[k++]) Att(a);
      }
      for (auto* l : lists)
        for (AttP& p : *l)
          if (p >= lo && p < hi) p = &na->atts[std::lower_bound(mv.begin(), mv.end(), p) - mv.begin()];
      g.arenas.push_back(na);
    }
  }
  std::vector<char> used(g.arenas.size(), 0);
  for (auto* l : lists)
    for (AttP p : *l)
      for (size_t k = 0; k < g.arenas.size(); ++k) {
        const AttStore& a = g.arenas[k]->atts;
        if (!a.empty() && p >= a.data() && p < a.data() + a.size()) {
          used[k] = 1;
          break;
        }
      }
  size_t j = 0;
  for (size_t k = 0; k < g.arenas.size(); ++k)
    if (used[k]) g.arenas[j++] = g.arenas[k];
  g.arenas.resize(j);
}

// Every block, on the calling thread, before anything else (the path that keeps a call
// all-or-nothing; pz_chain_process_blocks pipelines the parse otherwise).
static int parse_all(const uint8_t* data, const uint64_t* offs, uint64_t n, std::vector<Block>& blocks,
                     std::shared_ptr<CallArena>* keep, int threads, PinBuf* pin = nullptr) {
  std::vector<uint64_t> first;
  int rc = count_per_block(data, offs, n, first);
  if (rc) return rc;
  auto ar = make_arena(offs, n, std::move(first), (size_t)threads, pin);
  *keep = ar;  // the blocks' bytes live here for the whole call (records alias it beyond)
  blocks.resize(n);
  const uint64_t bad = parse_parallel(data, offs, n, *ar, blocks);
  if (bad < n) return fail(PZ_EINVAL, "block %llu is not a canonical BeaconBlock encoding", (unsigned long long)bad);
  return PZ_OK;
}

// Upload the hash-log entries appended since the last upload (the device copy grows,
// keeping its contents).
static void sync_hash_log(Engine& g) {
  const uint64_t n = g.hlog.size();
  if (n == g.d_hlog_n) return;
  if (n * 32 > g.d_hlog.n) {
    DevArr<uint8_t> nb;
    check(nb.alloc(std::max<uint64_t>(g.hlog.capacity() * 32, 2 * g.d_hlog.n)));  // (the call's reserve: once a call)
    if (g.d_hlog_n) hchk(hipMemcpyAsync(nb.p, g.d_hlog.p, g.d_hlog_n * 32, hipMemcpyDeviceToDevice, g.ms), "D2D");
    std::swap(g.d_hlog.p, nb.p);
    std::swap(g.d_hlog.n, nb.n);
    g.retired.keep(nb.p);  // (the queued copy reads it)
    nb.p = nullptr;
  }
  hchk(hipMemcpyAsync(g.d_hlog.p + g.d_hlog_n * 32, g.hlog[g.d_hlog_n].b, (n - g.d_hlog_n) * 32,
                      hipMemcpyHostToDevice, g.ms), "H2D hash log");
  g.d_hlog_n = n;
}

// The same for the recent-hash trail.
static void sync_trail(Engine& g) {
  const uint64_t n = g.trail.size();
  if (n == g.d_trail_n) return;
  if (n > g.d_trail.n) {
    DevArr<uint32_t> nb;
    check(nb.alloc(std::max<uint64_t>(g.trail.capacity(), 2 * g.d_trail.n)));
    if (g.d_trail_n) hchk(hipMemcpyAsync(nb.p, g.d_trail.p, g.d_trail_n * 4, hipMemcpyDeviceToDevice, g.ms), "D2D");
    std::swap(g.d_trail.p, nb.p);
    std::swap(g.d_trail.n, nb.n);
    g.retired.keep(nb.p);  // (the queued copy reads it)
    nb.p = nullptr;
  }
  hchk(hipMemcpyAsync(g.d_trail.p + g.d_trail_n, g.trail.data() + g.d_trail_n, (n - g.d_trail_n) * 4,
                      hipMemcpyHostToDevice, g.ms), "H2D trail");
  g.d_trail_n = n;
}

// Wait for the message batches in flight (their H2D copies read the pinned hash log, trail
// and records).
static void msg_drain(Engine& g) {
  if (!g.m_busy) return;
  hchk(hipStreamSynchronize(g.ms), "sync (message batch)");
  g.m_busy = false;
}

// processAttestation messages per batch sent while the walk goes on (PZ_MSG_BATCH; 0, the
// default: one batch at the end of the call).  The kernel is latency-bound (one lane runs a
// message's 17 compressions), ~0.13 ms for any batch up to 65,536 messages, so the last batch
// costs the same wait as one whole-call batch: 8,192 measured no better than 0 on the
// configs[4] replay (profiles/r03/msg_batch_ab_r3ap.txt), and costs six more sends.
static uint64_t msg_batch(const Engine& g) { return g.opt.msg_batch; }  // (pz_chain_options)

// Digest the messages the walk appended since the last batch, on stream ms: the new hash-log
// and trail entries, the records and var bytes H2D (pinned: no host staging), one
// pz_b2b_attmsg_kernel launch over the batch and the D2H of its digests into g.m_pin.  Nothing
// waits here; msg_drain / the end of the call does.
static void msg_send(Engine& g) {
  const uint64_t n = g.m_rec.n, k = n - g.m_sent;
  if (!k) return;
  PhaseTimer pt(g.prof[kProfMsgSend]);
  {
    PhaseTimer pl(g.prof[kProfMsgLog]);
    sync_hash_log(g);
    sync_trail(g);
  }
  if (g.m_var.n + 4 > g.d_mvar.n) {  // grow, keeping what earlier batches sent
    DevArr<uint8_t> nb;
    check(nb.alloc(std::max<uint64_t>(g.m_var.capacity() + 4, 2 * g.d_mvar.n)));  // (once a call, bar a regrowth)
    if (g.m_var_sent) hchk(hipMemcpyAsync(nb.p, g.d_mvar.p, g.m_var_sent, hipMemcpyDeviceToDevice, g.ms), "D2D");
    std::swap(g.d_mvar.p, nb.p);
    std::swap(g.d_mvar.n, nb.n);
    g.retired.keep(nb.p);  // (the queued copy reads it)
    nb.p = nullptr;
  }
  if (g.m_var.n > g.m_var_sent)
    hchk(hipMemcpyAsync(g.d_mvar.p + g.m_var_sent, g.m_var.data() + g.m_var_sent, g.m_var.n - g.m_var_sent,
                        hipMemcpyHostToDevice, g.ms), "H2D message ids / ShardBlockHash");
  hchk(hipMemcpyAsync(g.d_mrec.p + g.m_sent, g.m_rec.data() + g.m_sent, k * sizeof(AttMsg), hipMemcpyHostToDevice, g.ms),
       "H2D message records");
  hchk(launch_b2b_attmsg(g.d_hlog.p, g.d_trail.p, g.d_mrec.p + g.m_sent, g.d_mvar.p, k, g.d_mout.p + g.m_sent * 64, g.ms),
       "attestation message digests");
  hchk(hipMemcpyAsync(g.m_pin.p + g.m_sent * 64, g.d_mout.p + g.m_sent * 64, k * 64, hipMemcpyDeviceToHost, g.ms), "D2H");
  g.m_sent = n;
  g.m_var_sent = g.m_var.n;
  g.m_busy = true;
}

// Digest messages of blocks [b0, b1) and their na attestations (a0.. in call order), laid out
// [blocks][attestation encodings][Key() preimages] in pinned memory, then H2D, one CSR BLAKE2b
// launch and the D2H of the 32-byte digests, all on stream s.
// The host half: the messages into D's pinned buffers; returns their bytes (offsets in D.offs).
static uint64_t stage_host(const std::vector<Block>& blocks, uint64_t b0, uint64_t b1, uint64_t na, DigestBufs& D) {
  const uint64_t nb = b1 - b0, nmsg = nb + 2 * na;
  uint64_t total = 0;
  for (uint64_t bi = b0; bi < b1; ++bi) {
    total += blocks[bi].len;
    for (auto& a : blocks[bi].atts) total += a->len + 10 + a->sbh_len + 32 * a->obl.size();
  }
  check(D.msgs.reserve(total + 16));  // (the pipelined producer's buffers were reserved to fit)
  check(D.offs.reserve((nmsg + 1) * 8));
  check(D.dig.reserve(nmsg * 32 + 32));
  uint8_t* buf = D.msgs.p;
  uint64_t* ho = reinterpret_cast<uint64_t*>(D.offs.p);
  uint64_t pos = 0, k = 0, ka = nb + 1, kk = nb + na + 1;
  ho[0] = 0;
  for (uint64_t bi = b0; bi < b1; ++bi) ho[++k] = pos += blocks[bi].len;
  uint64_t pa = pos;
  for (uint64_t bi = b0; bi < b1; ++bi)
    for (auto& a : blocks[bi].atts) ho[ka++] = pa += a->len;
  uint64_t pk = pa;
  for (uint64_t bi = b0; bi < b1; ++bi)
    for (auto& a : blocks[bi].atts) ho[kk++] = pk += 10 + a->sbh_len + 32 * a->obl.size();
  uint64_t m = nb;
  for (uint64_t bi = b0; bi < b1; ++bi) {
    const Block& b = blocks[bi];
    std::memcpy(buf + ho[bi - b0], b.data, b.len);
    for (auto& ap : b.atts) {
      const Att& a = *ap;
      std::memcpy(buf + ho[m], a.base, a.len);
      // Key() preimage (types/attestation.go:61-77): a 10-byte buffer holding uvarint(slot)
      // overwritten by uvarint(shard), ShardBlockHash, each oblique hash copied into a [32]byte
      uint8_t* q = buf + ho[m + na];
      std::memset(q, 0, 10);
      uint8_t v[10];
      size_t vl = 0;
      for (uint64_t x = a.slot; ; x >>= 7) {
        v[vl++] = (uint8_t)(x >= 0x80 ? (x & 0x7F) | 0x80 : x);
        if (x < 0x80) break;
      }
      std::memcpy(q, v, vl);
      vl = 0;
      for (uint64_t x = a.shard; ; x >>= 7) {
        v[vl++] = (uint8_t)(x >= 0x80 ? (x & 0x7F) | 0x80 : x);
        if (x < 0x80) break;
      }
      std::memcpy(q, v, vl);
      std::memcpy(q + 10, a.at(a.sbh_off), a.sbh_len);
      uint64_t kl = 10 + a.sbh_len;
      for (auto& o : a.obl) {
        const H32 h = copy32(a.at(o.first), o.second);
        std::memcpy(q + kl, h.b, 32);
        kl += 32;
      }
      ++m;
    }
  }
  return pk;
}

// The device half: H2D, one CSR BLAKE2b launch, D2H of the 32-byte digests, on stream s.
static void stage_launch(uint64_t nmsg, uint64_t bytes, DigestBufs& D, hipStream_t s) {
  check(D.d_in.alloc(bytes + 16));
  check(D.d_out.alloc(nmsg * 32));
  check(D.d_offs.alloc(nmsg + 1));
  hchk(hipMemcpyAsync(D.d_offs.p, D.offs.p, (nmsg + 1) * 8, hipMemcpyHostToDevice, s), "H2D offsets");
  if (bytes) hchk(hipMemcpyAsync(D.d_in.p, D.msgs.p, bytes, hipMemcpyHostToDevice, s), "H2D msgs");
  hchk(launch_b2b_csr(D.d_in.p, D.d_offs.p, nmsg, D.d_out.p, 32, s), "blake2b csr");
  hchk(hipMemcpyAsync(D.dig.p, D.d_out.p, nmsg * 32, hipMemcpyDeviceToHost, s), "D2H digests");
}

// The batch path's digest batch, reading blocks and attestation encodings where they lie in
// the call's pinned arena (one H2D of the arena, no copy of them on the host); only the Key()
// preimages are built.  Digests [blocks][attestation Hash][Key], 32 B each, land in D.dig.
// Two launches on s: the nb block digests, D2H'd and then ev_blk; the attestations' Hash and
// Key behind them, then ev_att.  The host builds the Key() preimages while the arena and the
// block digests are on the way.
static void stage_digests_arena(const std::vector<Block>& blocks, uint64_t nb, uint64_t na, const CallArena& ar,
                                uint64_t abytes, DigestBufs& D, hipStream_t s, hipEvent_t ev_blk, hipEvent_t ev_att) {
  hchk(hipStreamSynchronize(s), "sync");  // (a failed call's attestation part may still read D)
  const uint64_t nmsg = nb + 2 * na, aal = (abytes + 15) & ~15ull;
  std::vector<uint64_t> kb(nb + 1, 0);  // per block, where its Key() preimages start
  for (uint64_t bi = 0; bi < nb; ++bi) {
    uint64_t k = 0;
    for (auto& a : blocks[bi].atts) k += 10 + a->sbh_len + 32 * a->obl.size();
    kb[bi + 1] = kb[bi] + k;
  }
  const uint64_t kbytes = kb[nb];
  check(D.msgs.reserve(kbytes + 16));
  check(D.offs.reserve(2 * nmsg * 8 + 8));
  check(D.dig.reserve(nmsg * 32 + 32));
  check(D.d_in.alloc(aal + kbytes + 16));
  check(D.d_out.alloc(nmsg * 32));
  check(D.d_offs.alloc(2 * nmsg + 1));
  // the arena's DMA first: it crosses PCIe while the spans and Key() preimages are built
  hchk(hipMemcpyAsync(D.d_in.p, ar.bytes, abytes + 16, hipMemcpyHostToDevice, s), "H2D arena");  // (+ its zero pad)
  uint64_t* beg = reinterpret_cast<uint64_t*>(D.offs.p);
  uint64_t* end = beg + nmsg;
  for (uint64_t bi = 0; bi < nb; ++bi) {
    beg[bi] = (uint64_t)(blocks[bi].data - ar.bytes);
    end[bi] = beg[bi] + blocks[bi].len;
  }
  hchk(hipMemcpyAsync(D.d_offs.p, beg, nb * 8, hipMemcpyHostToDevice, s), "H2D spans");
  hchk(hipMemcpyAsync(D.d_offs.p + nmsg, end, nb * 8, hipMemcpyHostToDevice, s), "H2D spans");
  hchk(launch_b2b_spans(D.d_in.p, D.d_offs.p, D.d_offs.p + nmsg, nb, D.d_out.p, 32, s), "blake2b spans (blocks)");
  hchk(hipMemcpyAsync(D.dig.p, D.d_out.p, nb * 32, hipMemcpyDeviceToHost, s), "D2H digests");
  hchk(hipEventRecord(ev_blk, s), "event");
  // the attestation spans and Key() preimages of blocks [b0, b1), on the parse's worker pool
  // (serial, this loop was ~3 % of the replay's samples, profiles/r03/walk_sampler_r3av.txt)
  auto fill = [&](uint64_t b0, uint64_t b1) {
    uint64_t ka = nb + ar.first[b0], kk = nb + na + ar.first[b0], kpos = kb[b0];
    for (uint64_t bi = b0; bi < b1; ++bi) {
      for (auto& ap : blocks[bi].atts) {
        const Att& a = *ap;
        beg[ka] = (uint64_t)(a.base - ar.bytes);
        end[ka] = beg[ka] + a.len;
        ++ka;
        // Key() preimage (types/attestation.go:61-77): a 10-byte buffer holding uvarint(slot)
        // overwritten by uvarint(shard), ShardBlockHash, each oblique hash copied into a [32]byte
        uint8_t* q = D.msgs.p + kpos;
        std::memset(q, 0, 10);
        put_uvarint(q, a.slot);
        put_uvarint(q, a.shard);
        std::memcpy(q + 10, a.at(a.sbh_off), a.sbh_len);
        uint64_t kl = 10 + a.sbh_len;
        for (auto& o : a.obl) {
          const H32 h = copy32(a.at(o.first), o.second);
          std::memcpy(q + kl, h.b, 32);
          kl += 32;
        }
        beg[kk] = aal + kpos;
        end[kk++] = aal + kpos + kl;
        kpos += kl;
      }
    }
  };
  const uint64_t T = std::min<uint64_t>((uint64_t)parse_threads(kbytes + 32 * na), nb / 64 + 1);
  if (T <= 1) {
    fill(0, nb);
  } else {
    std::vector<std::function<void()>> fns;
    for (uint64_t t = 0; t < T; ++t) fns.push_back([&, t] { fill(nb * t / T, nb * (t + 1) / T); });
    try {
      work_pool().run(fns);
    } catch (const std::system_error&) {  // no thread to be had
      fill(0, nb);
    }
  }
  if (na) {
    hchk(hipMemcpyAsync(D.d_offs.p + nb, beg + nb, 2 * na * 8, hipMemcpyHostToDevice, s), "H2D spans");
    hchk(hipMemcpyAsync(D.d_offs.p + nmsg + nb, end + nb, 2 * na * 8, hipMemcpyHostToDevice, s), "H2D spans");
    if (kbytes) hchk(hipMemcpyAsync(D.d_in.p + aal, D.msgs.p, kbytes, hipMemcpyHostToDevice, s), "H2D keys");
    hchk(hipMemsetAsync(D.d_in.p + aal + kbytes, 0, 16, s), "memset");
    hchk(launch_b2b_spans(D.d_in.p, D.d_offs.p + nb, D.d_offs.p + nmsg + nb, 2 * na, D.d_out.p + nb * 32, 32, s),
         "blake2b spans (attestations)");
    hchk(hipMemcpyAsync(D.dig.p + nb * 32, D.d_out.p + nb * 32, 2 * na * 32, hipMemcpyDeviceToHost, s), "D2H digests");
  }
  hchk(hipEventRecord(ev_att, s), "event");
}

static void stage_digests(const std::vector<Block>& blocks, uint64_t b0, uint64_t b1, uint64_t na, DigestBufs& D,
                          hipStream_t s) {
  const uint64_t bytes = stage_host(blocks, b0, b1, na, D);
  stage_launch((b1 - b0) + 2 * na, bytes, D, s);
}

// Where the walk finds its blocks and their digests (block / attestation Hash / Key, 32 B).
// Batch: everything parsed and hashed before the walk.  Pipelined: a producer thread parses
// chunks of kChunk blocks into the arena and enqueues each chunk's digest batch on its own
// stream while the walk consumes the previous chunks (SURVEY.md §8 a3/a4 hashing off the walk's
// critical path); it stays at most kRing chunks ahead.
struct Feeder {
  std::vector<Block>* blocks = nullptr;
  uint64_t n = 0, natt = 0;
  // batch
  const uint8_t* dg = nullptr;
  uint64_t dstride = 32;
  // pipelined
  bool piped = false;
  struct Slot {
    DigestBufs* d = nullptr;  // Engine::ring[j % kRing]
    hipEvent_t ev = nullptr;  // Engine::ring_ev[j % kRing]
    uint64_t b0 = 0, b1 = 0, a0 = 0, na = 0, bytes = 0;
    uint64_t launched = UINT64_MAX;  // the chunk whose digest batch was launched from this slot
  } slot[kRing];
  hipStream_t s2 = nullptr;
  std::atomic<uint64_t> ready{0};     // chunks parsed and their digests enqueued
  std::atomic<uint64_t> consumed{0};  // chunks the walk has finished
  std::atomic<uint64_t> bad{UINT64_MAX};  // first malformed block
  std::atomic<int> rc{0};
  std::atomic<bool> stop{false};
  uint64_t cur = UINT64_MAX;  // the chunk the walk is in
  hipEvent_t att_ev = nullptr;  // non-null: the attestations' Hash / Key land behind it (after the walk)
  double wait_s = 0;

  // false: block bi is not there (a malformed block at or before it ends the walk)
  bool ensure(uint64_t bi) {
    if (!piped) return true;
    const uint64_t j = bi / kChunk;
    if (j == cur) return bi < bad.load(std::memory_order_acquire);
    if (cur != UINT64_MAX) consumed.store(cur + 1, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    while (ready.load(std::memory_order_acquire) <= j && !rc.load() &&
           bad.load(std::memory_order_acquire) > bi)
      std::this_thread::yield();
    if (rc.load()) throw rc.load();
    if (bi >= bad.load(std::memory_order_acquire)) return false;
    launch(j);
    // the next chunk's batch goes out now, so it is done when the walk gets there
    if (ready.load(std::memory_order_acquire) > j + 1) launch(j + 1);
    Slot& S = slot[j % kRing];
    hchk(hipEventSynchronize(S.ev), "event sync (digests)");
    wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    cur = j;
    return true;
  }
  // Every HIP call of the pipeline is made here, on the walk's thread: HIP calls from the
  // producer thread (its own stream) made each of the walk's tally flushes ~4x slower (runtime
  // lock contention; profiles/r03/replay_pipeline_r3i.txt).
  void launch(uint64_t j) {
    Slot& S = slot[j % kRing];
    if (S.launched == j) return;
    S.launched = j;
    const uint64_t nmsg = (S.b1 - S.b0) + 2 * S.na;
    if (nmsg) stage_launch(nmsg, S.bytes, *S.d, s2);
    hchk(hipEventRecord(S.ev, s2), "event");
  }
  const uint8_t* blk(uint64_t bi) const {
    if (!piped) return dg + bi * dstride;
    const Slot& S = slot[(bi / kChunk) % kRing];
    return S.d->dig.p + (bi - S.b0) * 32;
  }
  const uint8_t* hash(uint64_t bi, uint64_t ga) const {
    if (!piped) return dg + (n + ga) * dstride;
    const Slot& S = slot[(bi / kChunk) % kRing];
    return S.d->dig.p + ((S.b1 - S.b0) + (ga - S.a0)) * 32;
  }
  const uint8_t* key(uint64_t bi, uint64_t ga) const {
    if (!piped) return dg + (n + natt + ga) * dstride;
    const Slot& S = slot[(bi / kChunk) % kRing];
    return S.d->dig.p + ((S.b1 - S.b0) + S.na + (ga - S.a0)) * 32;
  }
};

// The producer: chunk after chunk, parse into the arena and enqueue the digest batch.
static void feed(Engine& g, Feeder& F, const uint8_t* data, const uint64_t* offs, std::shared_ptr<CallArena> ar) {
  try {
    uint64_t a0 = 0;
    for (uint64_t j = 0, b0 = 0; b0 < F.n; ++j, b0 += kChunk) {
      while (F.consumed.load(std::memory_order_acquire) + kRing <= j) {
        if (F.stop.load()) return;
        std::this_thread::yield();
      }
      Feeder::Slot& S = F.slot[j % kRing];
      uint64_t b1 = std::min(F.n, b0 + kChunk);
      const uint64_t good = parse_range(data, offs, b0, b1, *ar, *F.blocks, (size_t)j);
      b1 = good;
      uint64_t na = 0;
      for (uint64_t bi = b0; bi < b1; ++bi) na += (*F.blocks)[bi].atts.size();
      S.b0 = b0;
      S.b1 = b1;
      S.a0 = a0;
      S.na = na;
      a0 += na;
      S.d = &g.ring[j % kRing];
      S.ev = g.ring_ev[j % kRing];
      S.bytes = b1 > b0 ? stage_host(*F.blocks, b0, b1, na, *S.d) : 0;
      if (good < std::min(F.n, b0 + kChunk)) F.bad.store(good, std::memory_order_release);
      F.ready.store(j + 1, std::memory_order_release);
      if (good < std::min(F.n, b0 + kChunk)) return;
    }
  } catch (int rc) {
    F.rc.store(rc ? rc : PZ_EDEVICE);
  }
}

static void process(Engine& g, Feeder& F, pz_block_result* br, pz_att_result* ar) {
  const uint64_t n = F.n, natt = F.natt;
  std::vector<Block>& blocks = *F.blocks;
  // the walk
  std::vector<uint64_t> msg_att;
  std::vector<AttLookup> look;  // per attestation of the current block
  std::vector<AttP> processed;
  std::vector<uint32_t> block_id(n);
  uint64_t ai = 0;
  msg_drain(g);  // (a failed call may have left a batch in flight)
  g.hlog.trim();
  g.trail.trim();
  g.m_rec.reset();
  g.m_var.reset();
  g.m_sent = g.m_var_sent = 0;
  g.m_rec.reserve(natt + 1);  // every message is an attestation of the call: no growth
  g.m_var.reserve(64 * natt + 4096);
  check(g.m_pin.reserve(natt * 64 + 64));
  check(g.d_mrec.alloc(natt + 1));
  check(g.d_mout.alloc(natt * 64 + 64));
  const uint64_t mbatch = msg_batch(g);
  read_knobs(g);
  // the tables grow once per call, not by doubling inside the walk
  g.slot_of.reserve(g.slot_of.size() + n);  // (plus any oblique hash shorter than 32 B: grows)
  g.hlog.reserve(g.hlog.size() + n + 2 * natt);
  g.id_slot.reserve(g.id_slot.size() + n + 2 * natt);
  g.trail.reserve(g.trail.size() + n + 2 * kCycle);
  // every block digest takes a vote-cache slot: one growth for the call, not a doubling (and
  // a stream sync) every few hundred blocks
  if (g.slot_hash.size() + n >= g.cap) grow_slots(g, std::max<uint64_t>(2 * g.cap, g.slot_hash.size() + n + 64));
  msg_att.reserve(natt);
  auto t_walk = std::chrono::steady_clock::now();
  uint64_t logged = 0;  // block digests are logged a chunk at a time, as they arrive
  for (uint64_t bi = 0; bi < n; ++bi) {
    if (!F.ensure(bi)) break;  // a malformed block: the call ends before it (EINVAL)
    if (bi == logged) {
      const uint64_t e = F.piped ? std::min(n, (bi / kChunk + 1) * kChunk) : n;
      for (; logged < e && (!F.piped || logged < F.bad.load()); ++logged) {
        H32 h;
        std::memcpy(h.b, F.blk(logged), 32);
        block_id[logged] = log_hash(g, h);
      }
    }
    const Block& b = blocks[bi];
    pz_block_result& r = br[bi];
    std::memcpy(r.hash, F.blk(bi), 32);
    r.status = PZ_BLOCK_PROCESSED;
    r.transition = 0;
    r.first_att = (uint32_t)ai;
    r.natt = (uint32_t)b.atts.size();
    const uint64_t a0 = ai;
    ai += b.atts.size();
    for (uint64_t j = 0; j < b.atts.size(); ++j) {
      pz_att_result& x = ar[a0 + j];
      std::memset(&x, 0, sizeof x);
      x.status = PZ_ATT_NOT_PROCESSED;
    }
    H32 h;
    std::memcpy(h.b, r.hash, 32);
    if (b.slot > 1 && !is_saved(g, b.parent)) {
      r.status = PZ_BLOCK_NO_PARENT;
      continue;
    }
    processed.clear();
    if (look.size() < b.atts.size()) look.resize(b.atts.size());
    bool can_atts = false;
    for (uint64_t j = 0; j < b.atts.size(); ++j) {
      pz_att_result& x = ar[a0 + j];
      try {
        FineTimer pt(g.prof[kProfCheck]);
        process_attestation(g, b.slot, *b.atts[j], look[j]);
      } catch (Rejected& e) {
        can_atts = false;
        x.status = e.code;
        continue;
      }
      can_atts = true;
      x.status = PZ_ATT_PROCESSED;
      if (!F.att_ev) {
        std::memcpy(x.hash, F.hash(bi, a0 + j), 32);
        std::memcpy(x.key, F.key(bi, a0 + j), 32);
      }
      x.msg_len = (uint32_t)(10 + 33 * kCycle + b.atts[j]->sbh_len);
      msg_att.push_back(a0 + j);
      processed.push_back(b.atts[j]);
    }
    if (!can_atts) {
      r.status = PZ_BLOCK_ATTS_REJECTED;
      continue;
    }
    bool cache_nil = true;  // the map returned by the last calculateBlockVoteCache call
    for (uint64_t j = 0; j < b.atts.size(); ++j) {
      try {
        FineTimer pt(g.prof[kProfQueue]);
        queue_vote_cache(g, b.slot, *b.atts[j], look[j]);
        cache_nil = g.A->cache_nil;
      } catch (Rejected&) {
        cache_nil = true;
      }
    }
    if (g.has_cand && b.slot > g.cand_slot && b.slot > 1) {  // updateHead (service.go:170-227)
      g.A = g.cand_A;
      g.C = g.cand_C;
      g.has_cand = false;
      g.cand_A.reset();
      g.cand_C.reset();
    }
    g.slot_saved[g.id_slot[block_id[bi]]] = 1;
    if (g.has_cand) {
      r.status = PZ_BLOCK_SAVED_NOT_CANDIDATE;
      continue;
    }
    AP A = g.A;
    CP C = g.C;
    if (b.slot >= C->lsr + kCycle) {  // IsCycleTransition (core.go:181-183)
      r.transition = 1;
      CP nc;
      AP na;
      state_recalc(g, C, A, b.slot, bi, &nc, &na);
      C = nc;
      A = na;
      if (mbatch && g.m_rec.n - g.m_sent >= mbatch) msg_send(g);  // (the walk just waited on the device)
    }
    // computeNewActiveState (core.go:223-237)
    A->cache_nil = cache_nil;
    A->pending.insert(A->pending.end(), processed.begin(), processed.end());
    push_recent(g, *A, block_id[bi]);
    A->recent_raw_empty = false;
    g.has_cand = true;
    g.cand_slot = b.slot;
    g.cand_A = A;
    g.cand_C = C;
  }
  g.prof[kProfWalk] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t_walk).count();
  flush_votes(g);
  epoch_collect(g);  // a panic of the last transition's epoch fails this call
  PhaseTimer pt(g.prof[kProfMsgHash]);
  const size_t nm = msg_att.size();
  if (g.m_rec.n != nm) throw fail(PZ_EDEVICE, "message batch out of step with the walk");
  msg_send(g);
  {
    PhaseTimer pw(g.prof[kProfMsgWait]);
    msg_drain(g);
  }
  const uint8_t* md = g.m_pin.p;
  const bool hk = F.att_ev != nullptr;  // the processed attestations' Hash and Key too (the batch path's second part)
  if (hk) hchk(hipEventSynchronize(F.att_ev), "event sync (attestation digests)");
  // 128 B per processed attestation into the caller's results: on the worker pool when large
  auto put = [&](size_t i0, size_t i1) {
    for (size_t i = i0; i < i1; ++i) {
      const uint64_t ga = msg_att[i];
      std::memcpy(ar[ga].msg_digest, &md[i * 64], 64);
      if (hk) {
        std::memcpy(ar[ga].hash, F.dg + (n + ga) * 32, 32);
        std::memcpy(ar[ga].key, F.dg + (n + natt + ga) * 32, 32);
      }
    }
  };
  const size_t T = std::min<size_t>((size_t)parse_threads((uint64_t)nm * 128), nm / 2048 + 1);
  if (T <= 1) {
    put(0, nm);
  } else {
    std::vector<std::function<void()>> fns;
    for (size_t t = 0; t < T; ++t) fns.push_back([&, t] { put(nm * t / T, nm * (t + 1) / T); });
    try {
      work_pool().run(fns);
    } catch (const std::system_error&) {  // no thread to be had
      put(0, nm);
    }
  }
}

}  // namespace chain
}  // namespace pz

using namespace pz;
using namespace pz::chain;

struct pz_chain {
  Engine g;
};

extern "C" {

// The chain's ranks: one on `device`, or one per local rank of `comm` (each on its device).
static void make_ranks(Engine& g, int device, pz_comm* comm) {
  g.comm = comm;
  g.world = comm ? comm->world : 1;
  const int L = comm ? comm->nlocal : 1;
  g.rk.resize(L);
  for (int i = 0; i < L; ++i) {
    RankDev& r = g.rk[i];
    r.dev = comm ? comm->dev[i] : device;
    r.grank = comm ? comm->rank0 + i : 0;
    check(pz_init(r.dev));
    hchk(hipSetDevice(r.dev), "hipSetDevice");
    hchk(hipStreamCreateWithFlags(&r.s, hipStreamNonBlocking), "hipStreamCreate");
  }
  g.device = g.rk[0].dev;
  g.s = g.rk[0].s;
  hchk(hipSetDevice(g.device), "hipSetDevice");
  hchk(hipStreamCreateWithFlags(&g.s2, hipStreamNonBlocking), "hipStreamCreate");
  hchk(hipStreamCreateWithFlags(&g.ms, hipStreamNonBlocking), "hipStreamCreate");
}

static void destroy_chain(pz_chain* c) {
  Engine& g = c->g;
  std::vector<std::pair<int, hipStream_t>> streams;
  for (RankDev& r : g.rk) {
    (void)hipSetDevice(r.dev);
    if (r.s) (void)hipStreamSynchronize(r.s);
    for (hipEvent_t e : {r.q_ev, r.vq_ev[0], r.vq_ev[1], r.ev_epoch, r.ev_t64})
      if (e) (void)hipEventDestroy(e);
    streams.push_back({r.dev, r.s});
  }
  for (hipEvent_t e : {g.ev_totals, g.ev_dblk, g.ev_datt})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : g.ring_ev)
    if (e) (void)hipEventDestroy(e);
  for (hipStream_t x : {g.s2, g.ms})
    if (x) {
      (void)hipSetDevice(g.device);
      (void)hipStreamSynchronize(x);
      streams.push_back({g.device, x});
    }
  delete c;
  for (auto& ds : streams)
    if (ds.second) {
      (void)hipSetDevice(ds.first);
      (void)hipStreamDestroy(ds.second);
    }
}

static int new_chain(uint64_t nval, int device, pz_comm* comm, pz_chain** out) {
  if (!out) return fail(PZ_EINVAL, "out is null");
  *out = nullptr;
  if (nval == 0 || nval > PZ_MAX_VALIDATORS) return fail(PZ_ETOOMANY, "validator count %llu out of range", (unsigned long long)nval);
  auto* c = new pz_chain();
  c->g.nval = nval;
  try {
    make_ranks(c->g, device, comm);
    check(genesis(c->g));
  } catch (int e) {
    destroy_chain(c);
    return e;
  }
  *out = c;
  return PZ_OK;
}

int pz_chain_new(uint64_t nval, int device, pz_chain** out) { return new_chain(nval, device, nullptr, out); }

int pz_chain_new_comm(uint64_t nval, pz_comm* comm, pz_chain** out) {
  if (!comm) return fail(PZ_EINVAL, "comm is null");
  return new_chain(nval, 0, comm, out);
}

int pz_chain_new_from_state(const uint8_t* cstate, uint64_t len, const uint8_t* saved_hashes, uint64_t nsaved,
                            int device, pz_chain** out) {
  if (!out) return fail(PZ_EINVAL, "out is null");
  *out = nullptr;
  if (!cstate || !len) return fail(PZ_EINVAL, "empty stored state");
  if (nsaved && !saved_hashes) return fail(PZ_EINVAL, "saved_hashes is null");
  auto* c = new pz_chain();
  try {
    make_ranks(c->g, device, nullptr);
    check(reload(c->g, cstate, len));
    for (uint64_t i = 0; i < nsaved; ++i) {
      H32 h;
      std::memcpy(h.b, saved_hashes + 32 * i, 32);
      c->g.saved.insert(h, 1);
    }
  } catch (int e) {
    destroy_chain(c);
    return e;
  }
  *out = c;
  return PZ_OK;
}

int pz_chain_set_options(pz_chain* c, const pz_chain_options* opts) {
  if (!c) return fail(PZ_EINVAL, "chain is null");
  Engine& g = c->g;
  std::lock_guard<std::mutex> lk(g.mu);
  const pz_chain_options o = opts ? *opts : pz_chain_options{};
  const bool bi = g.kmax <= kVoteInlineBits && !(o.tally_forms & PZ_TALLY_BITS_ROWS);
  const bool ir = (o.tally_forms & PZ_TALLY_ID_ROWS) != 0;
  // the tally forms shape the vote queue's records: a chain that has queued any under the old
  // form keeps it (its queue would be read against the other form at the next flush)
  if ((bi != g.bits_inline || ir != g.ids_rows || o.tally_forms != g.opt.tally_forms) && g.calls)
    return fail(PZ_EINVAL, "pz_chain_set_options: the tally forms are set before the first pz_chain_process_blocks call");
  g.opt = o;
  g.bits_inline = bi;
  g.ids_rows = ir;
  return PZ_OK;
}

void pz_chain_free(pz_chain* c) {
  if (!c) return;
  destroy_chain(c);
}

int pz_count_attestations(const uint8_t* blocks, const uint64_t* offsets, uint64_t n, uint64_t* count) {
  if (!count) return fail(PZ_EINVAL, "count is null");
  *count = 0;
  if (n && (!blocks || !offsets)) return fail(PZ_EINVAL, "null pointer");
  std::vector<uint64_t> first;
  const int rc = count_per_block(blocks, offsets, n, first);
  if (rc) return rc;
  *count = first[n];
  return PZ_OK;
}

int pz_chain_process_blocks(pz_chain* c, const uint8_t* blocks, const uint64_t* offsets, uint64_t n,
                            pz_block_result* block_out, pz_att_result* att_out, uint64_t att_cap) {
  if (!c) return fail(PZ_EINVAL, "chain is null");
  if (n == 0) return PZ_OK;
  if (!blocks || !offsets || !block_out) return fail(PZ_EINVAL, "null pointer");
  std::lock_guard<std::mutex> lk(c->g.mu);
  if (c->g.poisoned) return fail(PZ_EINDEX, "chain panicked earlier; create a new one");
  hipError_t e = hipSetDevice(c->g.device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  // the output capacity is checked before any state changes
  std::vector<uint64_t> first;
  int rc0;
  {
    PhaseTimer pt(c->g.prof[kProfCount]);
    rc0 = count_per_block(blocks, offsets, n, first);
  }
  if (rc0) return rc0;
  const uint64_t natt = first[n];
  if (natt > att_cap || (natt && !att_out)) return fail(PZ_EINVAL, "att_out holds %llu results, need %llu",
                                                        (unsigned long long)att_cap, (unsigned long long)natt);
  Engine& g = c->g;
  ++g.calls;
  std::vector<Block> parsed(n);
  Feeder F;
  F.blocks = &parsed;
  F.n = n;
  F.natt = natt;
  const uint64_t thr = serial_threshold();
  bool long_msg = false;
  for (uint64_t i = 0; i < n && !long_msg; ++i) long_msg = offsets[i + 1] >= offsets[i] && offsets[i + 1] - offsets[i] >= thr;
  std::shared_ptr<CallArena> arena;
  struct Keep {  // on every way out, the arenas the chain's states still point into stay
    Engine& g;
    std::shared_ptr<CallArena>& a;
    ~Keep() { keep_arenas(g, a.get()); }
  } keep{g, arena};
  std::vector<uint8_t> dg_slow;
  // The batch path (default): the whole call parsed, one digest batch, then the walk.  The
  // pipelined form (a producer thread parsing a chunk ahead, PZ_CHAIN_PIPELINE=1) measured
  // slower on the 10,000-block replay (177-183k vs 200-229k blocks/s; the producer slows the
  // walk's own host work, profiles/r03/replay_pipeline_r3*.txt), so it is an A/B knob.  Both
  // end the call at a malformed block with PZ_EINVAL, the blocks before it processed.
#ifdef PZ_AB_BUILD
  const char* pe = std::getenv("PZ_CHAIN_PIPELINE");
  F.piped = !long_msg && n >= 2 * kChunk && pe && pe[0] == '1';
#else
  F.piped = false;
#endif
  if (!F.piped) {
    try {
      PhaseTimer pt(g.prof[kProfParse]);
      arena = make_arena(offsets, n, std::move(first), (size_t)parse_threads(offsets[n] - offsets[0]), &g.arena_pin);
      const uint64_t good = parse_parallel(blocks, offsets, n, *arena, parsed);
      if (good < n) {  // the walk stops before the malformed block
        F.bad.store(good);
        F.n = good;
        F.natt = 0;
        for (uint64_t bi = 0; bi < good; ++bi) F.natt += parsed[bi].atts.size();
      }
    } catch (int rc) {
      return rc;
    }
    try {
      PhaseTimer pt(g.prof[kProfHash1]);
      if (!long_msg) {
        if (!g.ev_dblk) hchk(hipEventCreateWithFlags(&g.ev_dblk, hipEventDisableTiming), "event");
        if (!g.ev_datt) hchk(hipEventCreateWithFlags(&g.ev_datt, hipEventDisableTiming), "event");
        if (F.n) {
          stage_digests_arena(parsed, F.n, F.natt, *arena, offsets[n] - offsets[0], g.dbatch, g.s2, g.ev_dblk,
                              g.ev_datt);
          hchk(hipEventSynchronize(g.ev_dblk), "event sync (block digests)");
          F.att_ev = g.ev_datt;
        }
        F.dg = g.dbatch.dig.p;
        F.dstride = 32;
      } else {  // 64-byte digests; messages at or over the threshold on host threads
        std::string buf;
        std::vector<uint64_t> ho{0};
        const uint64_t ng = F.n;
        for (uint64_t bi = 0; bi < ng; ++bi) {
          buf.append((const char*)parsed[bi].data, parsed[bi].len);
          ho.push_back(buf.size());
        }
        for (uint64_t bi = 0; bi < ng; ++bi)
          for (auto& a : parsed[bi].atts) {
            buf.append((const char*)a->base, a->len);
            ho.push_back(buf.size());
          }
        for (uint64_t bi = 0; bi < ng; ++bi)
          for (auto& a : parsed[bi].atts) {  // Key() preimage (types/attestation.go:61-77)
            std::string k(10, '\0'), v;
            put_varint(v, a->slot);
            std::memcpy(&k[0], v.data(), v.size());
            v.clear();
            put_varint(v, a->shard);
            std::memcpy(&k[0], v.data(), v.size());
            k.append((const char*)a->at(a->sbh_off), a->sbh_len);
            for (auto& o : a->obl) {
              const H32 h = copy32(a->at(o.first), o.second);
              k.append((const char*)h.b, 32);
            }
            buf += k;
            ho.push_back(buf.size());
          }
        hash_many(g, buf, ho, dg_slow);
        F.dg = dg_slow.data();
        F.dstride = 64;
      }
    } catch (int rc) {
      return rc;
    }
  } else {
    // the parse and the digest batches run a chunk ahead of the walk on a producer thread
    try {
      arena = make_arena(offsets, n, std::move(first), (size_t)((n + kChunk - 1) / kChunk), &g.arena_pin);
    } catch (int rc) {
      return rc;
    }
  }
  std::thread producer;
  if (F.piped) {
    // the ring's pinned buffers and events, sized here for the largest chunk (the producer
    // makes no HIP call): the messages of a chunk are its blocks, their attestation encodings
    // (spans of the blocks) and Key() preimages of at most 10 + 16x the attestation's bytes
    uint64_t mx = 0;
    for (uint64_t b0 = 0; b0 < n; b0 += kChunk) mx = std::max(mx, offsets[std::min(n, b0 + kChunk)] - offsets[b0]);
    try {
      for (int k = 0; k < kRing; ++k) {
        check(g.ring[k].msgs.reserve(18 * mx + 10 * (mx / 8) + 16));
        check(g.ring[k].offs.reserve((kChunk + 2 * (mx / 8) + 2) * 8));
        check(g.ring[k].dig.reserve((kChunk + 2 * (mx / 8) + 2) * 32));
        if (!g.ring_ev[k]) hchk(hipEventCreateWithFlags(&g.ring_ev[k], hipEventDisableTiming), "event");
      }
    } catch (int rc) {
      return rc;
    }
    F.s2 = g.s2;
    producer = std::thread(feed, std::ref(g), std::ref(F), blocks, offsets, arena);
  }
  struct Join {  // the producer is stopped and joined on every way out (it reads F and parsed)
    Feeder& F;
    std::thread& t;
    ~Join() {
      F.stop.store(true);
      F.consumed.store(UINT64_MAX / 2);
      if (t.joinable()) t.join();
    }
  } join{F, producer};
  try {
    PhaseTimer pt(g.prof[kProfProcess]);
    process(g, F, block_out, att_out);
  } catch (Panic& p) {
    g.poisoned = true;
    return fail(PZ_EINDEX, "the reference panics here: %s", p.what.c_str());
  } catch (int rc) {
    g.poisoned = true;
    return rc;
  }
  g.prof[kProfHash1] += F.wait_s;
  if (!g.retired.p.empty()) {  // the call's grown-out buffers, once nothing queued reads them
    try {
      each_rank(g, [](RankDev& r) {
        hchk(hipSetDevice(r.dev), "hipSetDevice");
        hchk(hipStreamSynchronize(r.s), "sync");
      });
      hchk(hipSetDevice(g.device), "hipSetDevice");
      hchk(hipStreamSynchronize(g.s2), "sync");
      hchk(hipStreamSynchronize(g.ms), "sync");
    } catch (int rc) {
      return rc;
    }
    g.retired.release();
  }
  const uint64_t bad = F.bad.load();
  if (bad < n) return fail(PZ_EINVAL, "block %llu is not a canonical BeaconBlock encoding (blocks before it were "
                                      "processed)", (unsigned long long)bad);
  return PZ_OK;
}

int pz_chain_roots(pz_chain* c, uint8_t out[4 * 32], int* has_candidate) {
  if (!c || !out) return fail(PZ_EINVAL, "null pointer");
  std::lock_guard<std::mutex> lk(c->g.mu);
  Engine& g = c->g;
  try {
    hchk(hipSetDevice(g.device), "hipSetDevice");
    epoch_collect(g);
    std::string buf;
    std::vector<uint64_t> offs{0};
    buf += encode_active(g, *g.A);
    offs.push_back(buf.size());
    buf += encode_crystallized(g, *g.C);
    offs.push_back(buf.size());
    if (g.has_cand) {
      buf += encode_active(g, *g.cand_A);
      offs.push_back(buf.size());
      buf += encode_crystallized(g, *g.cand_C);
      offs.push_back(buf.size());
    }
    std::vector<uint8_t> d;
    hash_many(g, buf, offs, d);
    std::memset(out, 0, 4 * 32);
    for (size_t i = 0; i + 1 < offs.size(); ++i) std::memcpy(out + 32 * i, &d[64 * i], 32);
    if (has_candidate) *has_candidate = g.has_cand ? 1 : 0;
  } catch (Panic& p) {  // the last transition's epoch, collected here
    g.poisoned = true;
    return fail(PZ_EINDEX, "the reference panics here: %s", p.what.c_str());
  } catch (int rc) {
    return rc;
  }
  return PZ_OK;
}

int pz_chain_state_bytes(pz_chain* c, int which, uint8_t* out, uint64_t cap, uint64_t* len) {
  if (!c || !len) return fail(PZ_EINVAL, "null pointer");
  if (which < 0 || which > 3) return fail(PZ_EINVAL, "which must be 0..3");
  std::lock_guard<std::mutex> lk(c->g.mu);
  Engine& g = c->g;
  if (which >= 2 && !g.has_cand) return fail(PZ_EINVAL, "no candidate state");
  try {
    hchk(hipSetDevice(g.device), "hipSetDevice");
    epoch_collect(g);
    const std::string b = (which & 1) ? encode_crystallized(g, which >= 2 ? *g.cand_C : *g.C)
                                      : encode_active(g, which >= 2 ? *g.cand_A : *g.A);
    *len = b.size();
    if (out && cap >= b.size()) std::memcpy(out, b.data(), b.size());
  } catch (Panic& p) {
    g.poisoned = true;
    return fail(PZ_EINDEX, "the reference panics here: %s", p.what.c_str());
  } catch (int rc) {
    return rc;
  }
  return PZ_OK;
}

int pz_chain_vote_totals(pz_chain* c, uint8_t* hashes, uint64_t* totals, uint64_t cap, uint64_t* count) {
  if (!c || !count) return fail(PZ_EINVAL, "null pointer");
  std::lock_guard<std::mutex> lk(c->g.mu);
  Engine& g = c->g;
  const AState& A = g.has_cand ? *g.cand_A : *g.A;
  // the Go map holds the hashes some attestation signed (present), with their totals: the
  // sum of the ranks' partial VoteTotalDeposit (an all-reduce of a copy across processes)
  std::vector<uint8_t> pres;
  std::vector<uint64_t> tot;
  if (!A.cache_nil && !g.slot_hash.empty()) {
    const uint64_t ns = g.slot_hash.size();
    pres.resize(ns);
    tot.assign(ns, 0);
    try {
      RankDev& r0 = g.rk[0];
      hchk(hipSetDevice(r0.dev), "hipSetDevice");
      hchk(hipMemcpyAsync(pres.data(), r0.present.p, ns, hipMemcpyDeviceToHost, r0.s), "D2H");
      if (g.world == (int)g.rk.size()) {
        std::vector<uint64_t> part(ns);
        for (RankDev& r : g.rk) {
          hchk(hipSetDevice(r.dev), "hipSetDevice");
          hchk(hipMemcpyAsync(part.data(), r.totals.p, ns * 8, hipMemcpyDeviceToHost, r.s), "D2H");
          hchk(hipStreamSynchronize(r.s), "sync");
          for (uint64_t i = 0; i < ns; ++i) tot[i] += part[i];
        }
      } else {
        DevArr<uint64_t> cp;
        check(cp.alloc(ns));
        hchk(hipMemcpyAsync(cp.p, r0.totals.p, ns * 8, hipMemcpyDeviceToDevice, r0.s), "D2D");
        hipEvent_t ev;
        hchk(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
        uint64_t* b = cp.p;
        int rc = g.comm->allreduce_u64(&b, ns, &r0.s, &ev);
        if (!rc) {
          hchk(hipStreamWaitEvent(r0.s, ev, 0), "wait");
          hchk(hipMemcpyAsync(tot.data(), cp.p, ns * 8, hipMemcpyDeviceToHost, r0.s), "D2H");
          hchk(hipStreamSynchronize(r0.s), "sync");
        }
        (void)hipEventDestroy(ev);
        check(rc);
      }
      hchk(hipStreamSynchronize(r0.s), "sync");
    } catch (int rc) {
      return rc;
    }
  }
  uint64_t n = 0;
  for (uint8_t p : pres) n += p;
  *count = n;
  if (n > cap || !n) return PZ_OK;  // caller retries with a larger buffer
  if (!hashes || !totals) return fail(PZ_EINVAL, "null pointer");
  for (uint64_t i = 0, j = 0; i < pres.size(); ++i)
    if (pres[i]) {
      std::memcpy(hashes + 32 * j, g.slot_hash[i].b, 32);
      totals[j++] = tot[i];
    }
  return PZ_OK;
}

}  // extern "C"

// Observability (include/prysm_hip.h): cumulative wall seconds per phase of the block pipeline
// (parse, digest batch 1 (blocks/Hash/Key), attestation checks + message assembly, vote-cache
// queueing, vote tally flushes, stateRecalc (excluding its flush), message digests, ...).
extern "C" int pz_chain_phase_times(pz_chain* c, double* out, int n) {
  if (!c || !out) return PZ_EINVAL;
  for (int i = 0; i < n && i < pz::chain::kProfSlots; ++i) out[i] = c->g.prof[i];
  return pz::chain::kProfSlots;
}

#ifdef PZ_AB_BUILD
// Internal (tools/replay_timeline.py): up to n transitions' timestamps (4 u64 each, CLOCK_MONOTONIC
// ns: flush start, tally launch returned, epoch launches returned, totals seen); returns the
// count recorded since the chain was created (at most 65,536 are kept).
// Internal (tools/vote_trace.py): under PZ_VOTE_TRACE the first flushes' per-wave tally stamps
// (votes_dev.h PZ_VSTAMP: 8 wall-clock words per wave, kVoteTraceWaves waves per flush) into
// out[nflush][kVoteTraceWaves][8], each flush's wave count into waves[nflush]; returns the flushes.
extern "C" int pz_debug_vote_trace(pz_chain* c, uint64_t* out, uint64_t* waves, int nflush) {
  if (!c || !out || !waves) return PZ_EINVAL;
  auto& g = c->g;
  RankDev& r = g.rk[0];
  if (!r.v_trace.p) return 0;
  const int n = std::min<int>(nflush, (int)std::min<uint64_t>(g.vtrace_n, kVoteTraceFlushes));
  if (hipSetDevice(r.dev) != hipSuccess || hipStreamSynchronize(r.s) != hipSuccess) return PZ_EDEVICE;
  if (hipMemcpy(out, r.v_trace.p, (size_t)n * kVoteTraceWaves * 64, hipMemcpyDeviceToHost) != hipSuccess)
    return PZ_EDEVICE;
  for (int i = 0; i < n; ++i) waves[i] = g.vtrace_w[i];
  return n;
}

extern "C" int pz_debug_chain_timeline(pz_chain* c, uint64_t* out, int n) {
  if (!c || !out) return PZ_EINVAL;
  const auto& tl = c->g.tl;
  for (int i = 0; i < n && i < (int)tl.size(); ++i)
    for (int k = 0; k < 4; ++k) out[4 * i + k] = tl[i][k];
  return (int)tl.size();
}

// Internal (tests/, tools/: the A/B library; CPU-only: no device call): the block parser of
// pz_chain_process_blocks on its own with `threads` threads, `reps` times; returns the wall
// seconds of the fastest run and a checksum of what it parsed (every block's slot, parent and
// record count, every record's fields and oblique spans), so that thread counts can be
// compared.  A malformed block fails with PZ_EINVAL naming the first one.
extern "C" int pz_debug_parse(const uint8_t* data, const uint64_t* offs, uint64_t n, uint64_t threads, int reps,
                              double* seconds, uint64_t* checksum) {
  double best = 1e30;
  // PZ_DEBUG_PARSE_PIN=1: the arena in pooled pinned memory, as pz_chain_process_blocks has it
  // (a device call: GPU boxes only)
  const char* pe = std::getenv("PZ_DEBUG_PARSE_PIN");
  pz::chain::PinBuf pin;
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    {
      std::vector<pz::chain::Block> blocks;
      std::shared_ptr<pz::chain::CallArena> arena;
      const int rc = pz::chain::parse_all(data, offs, n, blocks, &arena, (int)std::max<uint64_t>(1, threads),
                                          pe && pe[0] == '1' ? &pin : nullptr);
      if (rc) return rc;
      best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      if (checksum && r == 0) {
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
        for (const auto& b : blocks) {
          mix(b.slot);
          mix(b.len);
          for (int k = 0; k < 32; ++k) mix(b.parent.b[k]);
          mix(b.atts.size());
          for (auto ap : b.atts) {
            const auto& a = *ap;
            mix((uint64_t)(a.base - b.data));
            mix(a.len); mix(a.slot); mix(a.shard); mix(a.jslot);
            mix(a.sbh_off); mix(a.sbh_len); mix(a.bf_off); mix(a.bf_len);
            for (auto& o : a.obl) { mix(o.first); mix(o.second); }
          }
        }
        *checksum = h;
      }
    }
  }
  if (seconds) *seconds = best;
  return PZ_OK;
}
#endif  // PZ_AB_BUILD
