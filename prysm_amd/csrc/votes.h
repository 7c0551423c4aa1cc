// Vote-cache tally kernel arguments and launcher (votes.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/prysm_hip.h"

namespace pz {
typedef pz_vote_batch VoteArgs;
hipError_t launch_vote_tally(const VoteArgs& a, hipStream_t s);
}  // namespace pz
