// Host-staged collectives among the processes of one machine, through one POSIX shared-memory
// segment: the SHM backend of pz_comm (comm.h).
//
// Why it exists: RCCL refuses two ranks on one device ("Duplicate GPU"), so the one-process-per-
// GPU form of the sharded paths (pz_epoch_state, pz_chain_new_comm under torchrun) could only
// run on a node with a GPU per rank.  With this backend N processes sharing one GPU issue the
// same collective sequence the RCCL backend issues, so a one-GPU box runs that form end to end.
// It is a test / rehearsal backend: every collective is synchronous on the host.
//
// Protocol (one round per chunk of a collective; `seq` counts rounds, the same on every rank):
//   1. wait until every rank has consumed round seq-1 (so my slot is free);
//   2. copy my chunk into my slot, write my descriptor {op, a, b, chunk}, publish posted = seq;
//   3. wait until every rank has posted seq; every descriptor must equal mine -- otherwise the
//      ranks' collective sequences diverged (the hang an RCCL run would show), reported with
//      both ranks' calls and the group aborted;
//   4. combine the slots into my output, publish consumed = seq.
// A rank that does not arrive within the timeout fails the call (and aborts the group, so the
// others fail at once instead of timing out too).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace pz {

class ShmGroup {
 public:
  enum Op : uint32_t { kSumU64 = 1, kMinU32 = 2, kSumMin = 3, kAllGather = 4 };
  static constexpr int kMaxWorld = 64;

  // Every rank calls open with the same name, world and slot size; rank 0 creates the segment
  // (O_EXCL: a name in use fails), the others attach to it.  Returns when every rank has
  // attached; rank 0 then unlinks the name, so nothing is left in /dev/shm after the run.
  static int open(const char* name, int world, int rank, uint32_t timeout_ms, uint64_t slot_bytes, ShmGroup** out,
                  std::string* err);
  ~ShmGroup();

  int sum_u64(uint64_t* buf, size_t n, std::string* err);  // in place
  int min_u32(uint32_t* buf, size_t n, std::string* err);  // in place
  // one collective: the u64 sum over s and the u32 minimum over m (the RCCL backend's group)
  int sum_min(uint64_t* s, size_t ns, uint32_t* m, size_t nm, std::string* err);
  // recv receives every rank's `bytes` from send, rank-major
  int allgather(const void* send, void* recv, size_t bytes, std::string* err);

  int world() const { return world_; }
  int rank() const { return rank_; }
  uint64_t rounds() const { return seq_; }

 private:
  struct Desc {
    uint32_t op;
    uint64_t a, b, chunk;
  };
  template <typename F>
  int round(const void* mine, size_t bytes, const Desc& d, F&& combine, std::string* err);
  int wait_all(bool posted, uint64_t s, std::string* err);
  void abort_group();

  int world_ = 0, rank_ = 0;
  uint32_t timeout_ms_ = 0;
  uint64_t slot_bytes_ = 0;
  uint64_t seq_ = 0;
  void* base_ = nullptr;
  size_t map_bytes_ = 0;
};

}  // namespace pz
