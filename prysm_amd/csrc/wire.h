// Device proto3 encoders (wire.hip): kernel arguments and launchers shared with chain.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/prysm_hip.h"

namespace pz {

struct WireValArgs {
  const uint64_t* col[5];  // public_key, withdrawal_shard, balance, start_dynasty, end_dynasty
  const uint64_t* ccol[5];  // the non-NULL columns of col, in field order (scalar-only kernel)
  uint32_t ctag[5];         // their proto3 tags
  uint32_t nc;              // how many
  const uint8_t* wa;       // withdrawal_address bytes (CSR wa_offs, n+1; NULL offs = all empty)
  const uint64_t* wa_offs;
  const uint8_t* rc;       // randao_commitment bytes
  const uint64_t* rc_offs;
  uint64_t n;
  uint32_t field;    // framing field number (11 in a CrystallizedState); 0 = bare records
  uint32_t tag_len;  // varint length of the framing tag
  uint8_t* out;
  uint64_t* offs;   // optional record offsets, n+1
  uint64_t* total;  // device u64
  uint64_t* status;  // per-tile look-back words (set by the launcher from the scratch)
  uint32_t* ticket;
  uint64_t* trace;   // tools/ only: per-tile phase timestamps (variant 32), else NULL
};

uint64_t wire_tiles(uint64_t n);
int wire_val_args(const pz_validator_cols* v, uint64_t n, uint32_t field_num, WireValArgs* a);
// scratch: (wire_tiles(n) + 1) u64, zeroed by the launcher
hipError_t launch_wire_validators(WireValArgs a, uint64_t* scratch, hipStream_t s);
#ifdef PZ_AB_BUILD
int set_wire_variant(int v);  // the A/B library only (pz_debug_set_wire_variant)
void set_wire_trace(uint64_t* dev);  // the A/B library only: variant 32's timestamp buffer [tiles][16]
#endif

}  // namespace pz
