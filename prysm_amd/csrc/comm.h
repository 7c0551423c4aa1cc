// Communicator behind pz_comm (include/prysm_hip.h): the ranks of one validator-range or
// message-batch partition and the collectives the sharded epoch needs (sum all-reduce of
// u64, all-gather of bytes).
//
// Two backends:
//   RCCL      over xGMI; one process per GPU (ncclCommInitRank) or one process driving
//             several GPUs (ncclCommInitAll, the Go node's shape).  librccl is resolved at
//             run time: the copy already mapped into the process (PyTorch-ROCm's, which
//             matches the HIP runtime this library binds to there) or /opt/rocm's.
//   LOOPBACK  every rank lives in this process on ONE device; collectives are device copies
//             and one summing kernel.  It exists so that the sharded code paths (the same
//             ones RCCL drives) run on a one-GPU box in the parity tests.
//   SHM       one process per rank, the ranks free to share a device: each collective is a
//             D2H of the rank's buffer, a round through a POSIX shared-memory group
//             (shm_group.h) and an H2D of the result, synchronous on the host.  It runs the
//             one-process-per-GPU form (the bench under torchrun) on a one-GPU box, and it checks
//             that every rank issued the same collective sequence (a divergence RCCL would turn
//             into a hang fails the call with both ranks' calls named).
//
// A collective is ordered after each local rank's compute stream (an event), runs on the
// rank's collective stream, and marks completion with a per-rank event the caller waits on
// before it reads the result -- so compute on other buffers overlaps it.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "shm_group.h"

#include <cstddef>
#include <cstdint>
#include <vector>

struct pz_comm;

namespace pz {

// RCCL entry points, resolved with dlsym (no link-time dependency on librccl).
struct RcclApi {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  const char* origin = nullptr;  // which librccl was bound
};
// Binds the API once per process; PZ_EDEVICE (with pz_last_error) when no librccl loads.
int rccl_api(const RcclApi** out);

}  // namespace pz

struct pz_comm {
  enum Kind { RCCL, LOOPBACK, SHM } kind = RCCL;
  int world = 1;      // ranks in the partition
  int nlocal = 1;     // ranks driven by this process
  int rank0 = 0;      // global rank of local rank 0 (local ranks are contiguous)
  std::vector<int> dev;               // device of each local rank
  std::vector<ncclComm_t> nccl;       // RCCL: one communicator per local rank
  std::vector<hipStream_t> cstream;   // collective stream of each local rank
  std::vector<hipEvent_t> ev_in;      // per local rank: compute stream -> collective stream
  const pz::RcclApi* api = nullptr;
  uint64_t** d_ptrs = nullptr;        // LOOPBACK: device array of the ranks' buffer pointers
  pz::ShmGroup* shm = nullptr;        // SHM: the process group
  std::vector<uint8_t> shm_stage;     // SHM: host copy of the rank's buffer

  // Collective timing (pz_comm_set_timing): an event pair on every local rank's collective
  // stream around each collective; pz_comm_collective_time sums the pairs (max over the local
  // ranks per collective) and recycles the events.
  bool timing = false;
  struct TimedOp {
    std::vector<hipEvent_t> t0, t1;
  };
  std::vector<TimedOp> timed;
  bool time_open = false;  // the last collective's start was recorded (its end is due)
  std::vector<hipEvent_t> ev_pool;
  hipStream_t cs(int i) const { return cstream[kind == LOOPBACK ? 0 : i]; }

  // Sum all-reduce of `count` u64 in place: bufs[i] is local rank i's buffer; the collective
  // starts after everything enqueued so far on compute[i]; done[i] is recorded when local
  // rank i's result is ready.
  int allreduce_u64(uint64_t* const* bufs, size_t count, const hipStream_t* compute, hipEvent_t* done);
  // One group of two all-reduces in place: a u64 sum over sbufs (scount) and a u32 minimum
  // over mbufs (mcount) -- one collective launch on RCCL.
  int allreduce_sum_min(uint64_t* const* sbufs, size_t scount, uint32_t* const* mbufs, size_t mcount,
                        const hipStream_t* compute, hipEvent_t* done);
  // All-gather: local rank i contributes `bytes` from send[i]; recv[i] receives all ranks'
  // contributions, rank-major (world * bytes).
  int allgather(const void* const* send, void* const* recv, size_t bytes, const hipStream_t* compute,
                hipEvent_t* done);
  ~pz_comm();
};
