// Host-side BLAKE2b-512 for LONG single messages (a serial compression chain).
//
// Placement decision (DESIGN.md §3 "H: long messages"): BLAKE2b is a Merkle-Damgard chain,
// so one message of C compressions is C dependent steps no matter how many lanes exist.
// On gfx950 one lane retires a compression in ~6 us (dependent VALU latency, measured:
// 83 ms for the 13,416-compression CrystallizedState at 65,536 validators); one host core
// does it in ~0.1 us.  The batch entry points therefore route a message whose length is at
// or above the serial threshold to host threads, concurrently with the GPU launch that
// hashes every other message of the batch.  This is not a fallback: the library still
// refuses to run without a gfx950 device, and everything batchable stays on the GPU.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

// Default small-batch threshold in compressions (measured crossover).
#define PZ_SMALL_BATCH_DEFAULT 256

namespace pz {

// Full BLAKE2b-512 (RFC 7693, unkeyed, 64-byte digest) of msg[0..len).
void host_blake2b512(const uint8_t* msg, size_t len, uint8_t out[64]);

// Hash messages `which[k]` (indices into a CSR batch with absolute byte offsets) on up to
// `threads` host threads; digest i (out_bytes of it) goes to out + i * out_bytes.
void host_blake2b512_many(const uint8_t* data, const uint64_t* offsets, const std::vector<uint64_t>& which,
                          uint8_t* out, uint32_t out_bytes, unsigned threads);

// Messages at least this long are hashed on the host (default 64 KiB = 512 compressions);
// UINT64_MAX keeps every message on the GPU.
uint64_t serial_threshold();
uint64_t set_serial_threshold(uint64_t bytes);

// Batches of at most this many compressions in all are hashed on the calling thread (the
// drop-in Hash() latency path); 0 sends every batch to the GPU.
uint64_t small_batch_threshold();
uint64_t set_small_batch_threshold(uint64_t compressions);

// Host threads the library uses for its own parallel host work (block parsing, digest
// staging, long messages): the CPUs this process may run on, at most 16 (the CPU share of
// one GPU on the bench hosts); PZ_HOST_THREADS overrides it.
unsigned host_threads();
unsigned set_host_threads(unsigned n);  // 0: back to the default; returns the previous setting

// Indices of the messages of a CSR batch that go to the host (length >= threshold).
std::vector<uint64_t> long_messages(const uint64_t* offsets, uint64_t n);

// The long messages of one batch, hashed on host threads while the caller drives the GPU.
// start() returns at once; join() waits (the destructor joins too).
class SerialHashJob {
 public:
  void start(const uint8_t* data, const uint64_t* offsets, std::vector<uint64_t> which, uint8_t* out,
             uint32_t out_bytes);
  void join();
  ~SerialHashJob() { join(); }

 private:
  std::vector<uint64_t> which_;
  void* thread_ = nullptr;  // std::thread*
};

}  // namespace pz
