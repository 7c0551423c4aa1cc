/*
 * prysm_hip.h — C ABI of the MI355X-native state-transition hot path.
 *
 * This is the drop-in boundary: the entry points a cgo shim inside the reference's Go
 * packages would bind.  Every function is `extern "C"`, takes plain
 * pointers and sizes, never retains a caller pointer after it returns, and is thread-safe
 * (per-device mutex; one library-owned HIP stream per device for the host-pointer API).
 *
 * Two flavours:
 *   pz_*      host pointers, synchronous (the Go-API drop-in; data is copied H2D/D2H);
 *   pz_dev_*  device pointers, enqueued on the caller's hipStream_t (passed as void*),
 *             asynchronous; used by the device-resident mirror and the benchmark.
 *
 * Paths below are relative to the reference tree (/root/reference).  All arithmetic is
 * integer and bit-exact with the Go reference (uint64 wrap-around, MSB-first bitfields).
 *
 * The library fails loudly: if no gfx950 device is usable every compute entry point
 * returns PZ_EDEVICE; there is no CPU fallback.
 */
#ifndef PRYSM_HIP_H
#define PRYSM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------ */
#define PZ_OK         0
#define PZ_ENIL      -1  /* nil message: Go returns a proto.ErrNil-wrapped error (types/block_test.go:37-43) */
#define PZ_EINDEX    -2  /* Go index-out-of-range panic (CheckBit / committee / record index) */
#define PZ_ETOOMANY  -3  /* > params.MaxValidators (utils/shuffle.go:15-17) */
#define PZ_EDEVICE   -4  /* HIP failure or no usable gfx950 device */
#define PZ_ENOTFOUND -5  /* committee lookup failed: Go error (blockchain/core.go:373) */
#define PZ_EINVAL    -6  /* malformed arguments (null pointer with n > 0, bad sizes) */
#define PZ_ERANGE    -7  /* slice bounds out of range (Go panic, blockchain/core.go:353) */

/* params/config.go:4-26 */
#define PZ_ATTESTER_REWARD      1ULL
#define PZ_CYCLE_LENGTH         64
#define PZ_SHARD_COUNT          1024
#define PZ_DEFAULT_BALANCE      32ULL
#define PZ_MAX_VALIDATORS       4194304ULL
#define PZ_MIN_COMMITTEE_SIZE   128
#define PZ_DEFAULT_END_DYNASTY  9999999999999999999ULL

/* ---- runtime ------------------------------------------------------------------------ */
int         pz_init(int device);          /* select/initialise a device for this thread */
int         pz_device_count(int* count);
const char* pz_last_error(void);          /* thread-local message for the last failure */
int         pz_version(void);             /* ABI version: 1 */
/* Releases every device context the library created (streams, staging buffers).  Call it
 * last, from one thread, after every pz_chain / pz_epoch_state / pz_comm has been freed;
 * afterwards any entry point re-initialises lazily.  (The reference has no teardown: the Go
 * process exits; a long-lived cgo host calls this on node shutdown, node/node.go:124-132.) */
void        pz_shutdown(void);

/* ---- H: BLAKE2b-512 of serialized messages ------------------------------------------
 * Replaces `h := blake2b.Sum512(data); copy(hash[:], h[:32])` at
 *   types/block.go:73-76          (*Block).Hash
 *   types/attestation.go:55-58    (*Attestation).Hash
 *   types/attestation.go:74-76    (*Attestation).Key
 *   types/state.go:145-148        (*ActiveState).Hash
 *   types/state.go:244-247        (*CrystallizedState).Hash
 *   blockchain/core.go:290        processAttestation message hash (keeps all 64 bytes)
 *   utils/shuffle.go:19           ShuffleIndices seed stream (keeps all 64 bytes)
 * Messages are CSR: message i is msgs[offsets[i] .. offsets[i+1]); offsets has n+1 entries.
 * out receives n * out_bytes bytes (out_bytes = 32: the hot path's truncated digest; 64: full).
 */
int pz_blake2b512_batch(const uint8_t* msgs, const uint64_t* offsets, uint64_t n,
                        uint8_t* out, uint32_t out_bytes);

/* Long single messages (a state root is one serial chain of up to 221,844 compressions at
 * 1M validators) cannot use more than one lane: the batch entry points above hash every
 * message of at least `bytes` bytes on host threads (AVX2), concurrently with the GPU launch
 * for the rest of the batch.  Default 65,536; UINT64_MAX keeps everything on
 * the GPU.  Returns the previous value.  The pz_dev_* forms never leave the device. */
uint64_t pz_set_serial_threshold(uint64_t bytes);
/* Host threads the library uses beside the GPU (the serial hashes of long messages, the chain
 * engine's parse and result copies): 0 (the default) min(16, the process's CPU affinity), else n
 * (at most 256).  Returns the previous setting.  A placement control, not a reference API. */
uint32_t pz_set_host_threads(uint32_t n);

/* A batch of at most `compressions` BLAKE2b compressions in all (a drop-in Hash() call: one
 * 100-600 B message is 1-5) is hashed on the calling thread: the GPU route's launch, PCIe
 * copies and stream sync cost tens of microseconds against ~1 us of host work (DESIGN.md §3,
 * the measured crossover).  0 sends every batch to the GPU.  Returns the previous value.
 * The library still refuses to run without a gfx950 device. */
uint64_t pz_set_small_batch_threshold(uint64_t compressions);

/* Device-resident forms (device pointers; caller's stream).  The CSR form requires 4
 * readable bytes past msgs[offsets[n]-1] (the library's own buffers are padded). */
int pz_dev_blake2b512_batch(const uint8_t* d_msgs, const uint64_t* d_offsets, uint64_t n,
                            uint8_t* d_out, uint32_t out_bytes, void* stream);
/* Fixed-length records: message i is d_msgs[i*stride .. i*stride+len); stride % 16 == 0,
 * d_msgs 16-byte aligned, stride >= len.  This is the batched-record fast path.  The kernels
 * load whole aligned chunks, so the buffer must be readable up to the end of the last
 * record's chunk: (n-1)*stride + 128*ceil(len/128) bytes when stride >= 128*ceil(len/128)
 * (the LDS-staged path), (n-1)*stride + 16*ceil(len/16) otherwise; a buffer of n*stride
 * bytes with stride a multiple of 128 always suffices.  Bytes past len never affect a digest. */
int pz_dev_blake2b512_fixed(const uint8_t* d_msgs, uint64_t stride, uint64_t len, uint64_t n,
                            uint8_t* d_out, uint32_t out_bytes, void* stream);

/* ---- a2 / §8f: proto3 encoding of ValidatorRecords on the device -------------------
 * Replaces the validators span of gogo proto.Marshal(CrystallizedState) at
 * types/state.go:141 (Marshal) and :240 (Hash); record layout messages.pb.go:803-809.
 * Columns are SoA; a NULL scalar column means 0 in every record (omitted, as proto3 omits
 * zero scalars); a bytes column is CSR (data + offsets[n+1]), NULL offsets = all empty.
 * field_num > 0 frames every record as that length-delimited field (11 = the
 * CrystallizedState's `validators`); 0 writes bare records (then offsets delimit them).
 * offsets (optional, n+1) receive each record's start in out; offsets[n] = total length. */
typedef struct pz_validator_cols {
  const uint64_t* public_key;              /* field 1 */
  const uint64_t* withdrawal_shard;        /* field 2 */
  const uint8_t*  withdrawal_address;      /* field 3 (bytes) */
  const uint64_t* withdrawal_address_offs;
  const uint8_t*  randao_commitment;       /* field 4 (bytes) */
  const uint64_t* randao_commitment_offs;
  const uint64_t* balance;                 /* field 5 */
  const uint64_t* start_dynasty;           /* field 6 */
  const uint64_t* end_dynasty;             /* field 7 */
} pz_validator_cols;
/* Upper bound of the encoded length (bytes_total = both bytes columns' total length). */
uint64_t pz_wire_validators_bound(uint64_t n, uint64_t bytes_total);
/* Device scratch the pz_dev_ form needs for n records. */
uint64_t pz_wire_scratch_bytes(uint64_t n);
/* Host pointers, synchronous.  PZ_ERANGE (nothing written) when the encoding exceeds cap;
 * *len always receives the encoded length. */
int pz_wire_validators(const pz_validator_cols* v, uint64_t n, uint32_t field_num, uint8_t* out,
                       uint64_t cap, uint64_t* offsets, uint64_t* len);
/* Device pointers (columns included), caller's stream.  d_out must hold
 * pz_wire_validators_bound(...) bytes; *d_total (device) receives the length. */
int pz_dev_wire_validators(const pz_validator_cols* v, uint64_t n, uint32_t field_num, uint8_t* d_out,
                           uint64_t* d_offsets, void* d_scratch, uint64_t* d_total, void* stream);

/* ---- a2 / §8f: proto3 encoding of AttestationRecords on the device -------------------
 * Replaces golang/protobuf proto.Marshal(AttestationRecord) at types/attestation.go:51,56
 * (and the records inside BeaconBlock field 8, block.go:69, and ActiveState field 1,
 * state.go:141); record layout messages.pb.go:889-896.  Scalars: NULL = 0 everywhere.
 * Bytes fields: CSR (data + offsets[n+1]; NULL offsets = empty).  oblique_parent_hashes: an
 * element CSR (data + oblique_offs[m+1]) and the element range of record i,
 * oblique_first[i] .. oblique_first[i+1] (NULL = none).  aggregate_sig: values and the range
 * of record i, aggregate_sig_first[i] .. [i+1] (NULL = none).  field_num frames each record
 * (8: BeaconBlock.attestations, 1: ActiveState.pending_attestations; 0: bare records, the
 * bytes Attestation.Hash() hashes).  offsets[i] = start of record i, offsets[n] = length. */
typedef struct pz_attestation_cols {
  const uint64_t* slot;                    /* field 1 */
  const uint64_t* shard_id;                /* field 2 */
  const uint64_t* justified_slot;          /* field 3 */
  const uint8_t*  justified_block_hash;    /* field 4 */
  const uint64_t* justified_block_hash_offs;
  const uint8_t*  shard_block_hash;        /* field 5 */
  const uint64_t* shard_block_hash_offs;
  const uint8_t*  attester_bitfield;       /* field 6 */
  const uint64_t* attester_bitfield_offs;
  const uint8_t*  oblique_parent_hashes;   /* field 7 */
  const uint64_t* oblique_offs;
  const uint64_t* oblique_first;
  const uint64_t* aggregate_sig;           /* field 8 */
  const uint64_t* aggregate_sig_first;
} pz_attestation_cols;
uint64_t pz_wire_attestations_bound(uint64_t n, uint64_t bytes_total, uint64_t n_oblique, uint64_t n_sig);
uint64_t pz_wire_attestations_scratch_bytes(uint64_t n);
/* Host pointers, synchronous; ranges must start at 0.  PZ_ERANGE when the encoding exceeds
 * cap (*len still receives its length). */
int pz_wire_attestations(const pz_attestation_cols* a, uint64_t n, uint32_t field_num, uint8_t* out,
                         uint64_t cap, uint64_t* offsets, uint64_t* len);
/* Device pointers, caller's stream; d_out holds pz_wire_attestations_bound(...) bytes,
 * d_offsets n+1 entries (required). */
int pz_dev_wire_attestations(const pz_attestation_cols* a, uint64_t n, uint32_t field_num, uint8_t* d_out,
                             uint64_t* d_offsets, void* d_scratch, void* stream);

/* ---- T/R: validator-set filters (casper/validator.go) ------------------------------- */
#define PZ_KIND_ACTIVE 0  /* start <= dyn < end        casper/validator.go:45-53 */
#define PZ_KIND_EXITED 1  /* start <  dyn && end <= dyn casper/validator.go:57-65 */
#define PZ_KIND_QUEUED 2  /* start >  dyn               casper/validator.go:69-77 */
/* out (capacity n) receives the ascending indices; *count their number (0 == Go nil). */
int pz_validator_indices(const uint64_t* start_dynasty, const uint64_t* end_dynasty, uint64_t n,
                         uint64_t dynasty, int kind, uint32_t* out, uint64_t* count);

/* casper/validator.go:93-102 GetAttestersTotalDeposit: popcount of every pending
 * attestation's bitfield bytes (concatenated) x DefaultBalance. */
int pz_attesters_total_deposit(const uint8_t* bits, uint64_t nbytes, uint64_t* out);

/* casper/incentives.go:14-32 CalculateRewards, in place on balance[n].
 * Pending attestations are CSR bitfields (bits, boffs[natt+1]); the reward bit for rank i
 * is CheckBit(last bitfield, active[i]) and the target is balance[i] (rank, not index).
 * Returns PZ_EINDEX (balances untouched) where Go would panic. *applied = 1 when the
 * 2/3 threshold held. */
int pz_calculate_rewards(uint64_t* balance, const uint64_t* start_dynasty,
                         const uint64_t* end_dynasty, uint64_t n, uint64_t dynasty,
                         uint64_t total_deposit, const uint8_t* bits, const uint64_t* boffs,
                         uint64_t natt, int* applied);

/* blockchain/core.go:515-545 processCrosslinks tallies: for attestation a with committee
 * c = att_committee[a] (members committee[coffs[c] .. coffs[c+1])):
 *   total[a] = sum balance[member], vote[a] = sum balance[member] * CheckBit(bits_a, pos). */
int pz_crosslink_tally(const uint32_t* committee, const uint64_t* coffs, uint64_t ncomm,
                       const uint32_t* att_committee, const uint8_t* bits, const uint64_t* boffs,
                       uint64_t natt, const uint64_t* balance, uint64_t nval,
                       uint64_t* vote_out, uint64_t* total_out);

/* blockchain/core.go:502-558 processCrosslinks, complete: tallies as above, then the in-order
 * winner rule — for each shard the FIRST attestation with 3*vote >= 2*total (uint64 wrap)
 * and dynasty > rec_dynasty[shard] wins.  winner[s] (capacity nrec) receives the winning
 * attestation index or UINT32_MAX; the caller rewrites records[s] = {dynasty, that
 * attestation's ShardBlockHash, slot}.  PZ_EINDEX where Go would panic. */
int pz_process_crosslinks(const uint32_t* committee, const uint64_t* coffs, uint64_t ncomm,
                          const uint32_t* att_committee, const uint32_t* att_shard,
                          const uint8_t* bits, const uint64_t* boffs, uint64_t natt,
                          const uint64_t* balance, uint64_t nval, const uint64_t* rec_dynasty,
                          uint64_t nrec, uint64_t dynasty, uint32_t* winner,
                          uint64_t* vote_out, uint64_t* total_out);

/* utils/shuffle.go:14-33 ShuffleIndices, in place.  Host-resident by design (a sequential
 * swap chain, north_star); the 64-byte seed stream blake2b.Sum512(seed) goes through the batch
 * hash API (one compression: the small-batch route).  While n - i > 255 every swap target is
 * i + a fixed byte offset, so the chain runs division-free in a 256-entry window. */
int pz_shuffle_indices(const uint8_t seed[32], uint32_t* list, uint64_t n);

/* casper/validator.go:17-41 RotateValidatorSet, in place on start/end: active validators
 * below DefaultBalance/2 exit (end = dynasty); then the first min(len(active)/30 + 1,
 * len(queued)) queued validators, by ascending index, start (start = dynasty).  The active
 * count, the exits and the queued list run on the device filter kernels. */
int pz_rotate_validator_set(const uint64_t* balance, uint64_t* start, uint64_t* end, uint64_t n,
                            uint64_t dynasty);

/* casper/sharding.go:11-53 ShuffleValidatorsToCommittees: active indices (device filter),
 * ShuffleIndices (host swap chain), then splitBySlotShard into CSR: slot s (0..63) holds
 * committees slot_offs[s] .. slot_offs[s+1]; committee c has shard shard_id[c] and members
 * members[coffs[c] .. coffs[c+1]].  members needs room for n, coffs for cap_comm+1 and shard_id
 * for cap_comm entries, slot_offs for 65; PZ_ERANGE (with *ncomm = the count needed) when
 * cap_comm is short, PZ_ETOOMANY above MaxValidators (utils/shuffle.go:15-17). */
int pz_shuffle_validators_to_committees(const uint8_t seed[32], const uint64_t* start, const uint64_t* end,
                                        uint64_t n, uint64_t dynasty, uint64_t crosslink_start_shard,
                                        uint32_t* members, uint64_t* coffs, uint64_t* shard_id,
                                        uint64_t* slot_offs, uint64_t cap_comm, uint64_t* ncomm);

/* ---- a device-resident mirror of the validator set (SURVEY.md §8b "Ownership") ----------
 * The Go APIs take []*pb.ValidatorRecord, so every host-pointer casper call above re-packs and
 * re-copies the whole set.  A pz_state keeps one CrystallizedState's validators (SoA balance /
 * start / end) in HBM, owned by the library; the shim syncs it explicitly (upload after the
 * set changes, download when Go needs the balances) and the casper drop-ins run on it:
 * only the attestation bitfields cross PCIe per call.  NULL columns in upload / download are
 * skipped.  Same results and error codes as the host-pointer forms. */
typedef struct pz_state pz_state;
int  pz_state_new(uint64_t n, int device, pz_state** out);
int  pz_state_upload(pz_state* st, const uint64_t* balance, const uint64_t* start_dynasty,
                     const uint64_t* end_dynasty);
int  pz_state_download(pz_state* st, uint64_t* balance, uint64_t* start_dynasty, uint64_t* end_dynasty);
/* casper/validator.go:45-77 (pz_validator_indices on the mirror) */
int  pz_state_validator_indices(pz_state* st, uint64_t dynasty, int kind, uint32_t* out, uint64_t* count);
/* casper/incentives.go:14-32 (pz_calculate_rewards on the mirror's balances, in place) */
int  pz_state_calculate_rewards(pz_state* st, uint64_t dynasty, uint64_t total_deposit, const uint8_t* bits,
                                const uint64_t* boffs, uint64_t natt, int* applied);
/* blockchain/core.go:459-464: sum of the active validators' balances (TotalDeposits) */
int  pz_state_active_balance(pz_state* st, uint64_t dynasty, uint64_t* total);
void pz_state_free(pz_state* st);

/* ---- device-resident batched epoch transition (throughput mode, multi-GPU shards) -----
 * B independent instances of the data-parallel part of stateRecalc (blockchain/core.go:
 * 433-464): crosslink tallies + winners, attester popcount, CalculateRewards and the
 * next-cycle total balance.  All pointers are device pointers.  Validators are
 * instance-major [B][nval]; this rank holds global indices [val_offset, val_offset+nval)
 * of nval_global.  `scal` must be zero before pass 1 (allocate it zeroed, then ping-pong
 * with `scal_next`, which the finish pass zeroes); pass 1 initialises `winner` itself.
 * Single GPU: pz_dev_epoch_count -> pz_dev_epoch_finish.  Multi-GPU: count ->
 * all-reduce(sum) over the contiguous block {scal, vote, total} -> [when not every
 * validator is active: all-gather act_mask -> pz_dev_epoch_gather_compact] -> finish ->
 * all-reduce(sum) of scal[.][PZ_SCAL_NEXT_BAL].  After a multi-rank all-reduce,
 * PZ_SCAL_MAXIDX1 holds the sum of the per-rank values (single rank: the value). */
#define PZ_SCAL_POP       0  /* attester bit count (deposit = 32 * this)               */
#define PZ_SCAL_NACT      1  /* validators matching `kind` (written by the finish pass)  */
#define PZ_SCAL_ERR_XL    2  /* != 0: processCrosslinks would panic                     */
#define PZ_SCAL_ERR_RWD   3  /* != 0: CalculateRewards would panic (if threshold holds)  */
#define PZ_SCAL_APPLIED   4  /* 1: threshold held, balances updated                     */
#define PZ_SCAL_NEXT_BAL  5  /* sum of post-reward balances of active validators         */
#define PZ_SCAL_MAXIDX1   6  /* 1 + max matching global index (0: none)                 */
#define PZ_SCAL_NOMATCH   7  /* pass 1: validators in range NOT matching `kind` (all-reduced
                                with the rest); pass 2 sets PZ_SCAL_NACT = nval_global - this */
#define PZ_SCAL_COUNT     8
/* PZ_SCAL_ERR_XL is the sum, over every (attestation, rank) that found one, of the
 * PZ_XLERR_* values below: != 0 is the panic; the bits name the cause when one raiser did. */
#define PZ_XLERR_MEMBER   1ULL
#define PZ_XLERR_BITFIELD 2ULL
#define PZ_XLERR_SHARD    4ULL
#define PZ_XLERR_LAYOUT   8ULL  /* committee-order layout used with a non-matching validator */

typedef struct pz_epoch_batch {
  uint32_t ninst;                 /* B */
  uint64_t nval;                  /* validators per instance on this rank */
  uint64_t val_offset;            /* global index of local validator 0 */
  uint64_t nval_global;           /* validators per instance over all ranks */
  int kind;                       /* PZ_KIND_* (epoch transition: PZ_KIND_ACTIVE) */
  uint64_t* balance;              /* [B][nval] in/out */
  const uint64_t* start;          /* [B][nval] */
  const uint64_t* end;            /* [B][nval] */
  const uint64_t* dynasty;        /* [B] CurrentDynasty */
  const uint64_t* total_deposit;  /* [B] TotalDeposits */
  uint32_t natt;                  /* pending attestations per instance */
  const uint8_t* bits;            /* CSR bitfield bytes over B*natt attestations */
  const uint64_t* boffs;          /* [B*natt + 1] */
  uint64_t max_inst_bytes;        /* max bitfield bytes of one instance */
  uint32_t pop_rank, pop_world;   /* popcount chunks split over ranks (0, 1 single GPU) */
  const uint32_t* committee;      /* committee members (global validator indices) */
  const uint64_t* coffs;          /* [ncomm + 1] */
  const uint32_t* att_comm;       /* [B*natt] committee id of each attestation */
  const uint32_t* att_shard;      /* [B*natt] shard id of each attestation */
  uint32_t nrec;                  /* crosslink records per instance */
  const uint64_t* rec_dynasty;    /* [B][nrec] */
  uint32_t* winner;               /* [B][nrec] out */
  uint64_t* vote;                 /* [B*natt] out */
  uint64_t* total;                /* [B*natt] out */
  uint64_t* scal;                 /* [B][PZ_SCAL_COUNT] out */
  uint64_t* act_mask;             /* [B][ceil(nval/64)] scratch (general rank path) */
  uint32_t* blk_cnt;              /* [B][ceil(nval/2048)] scratch */
  uint32_t* act_list;             /* [B][nval_global] scratch (general rank path) */
  uint64_t* scal_next;            /* optional [B][PZ_SCAL_COUNT]: zeroed by the finish pass so
                                     the NEXT step can accumulate into it (ping-pong; saves a
                                     memset launch per step) */
  const uint32_t* cpos;           /* optional, multi-rank: `committee`/`coffs` list only this
                                     rank's members (global indices in [val_offset,
                                     val_offset + nval), plus, on rank 0, any member >=
                                     nval_global so that its panic is raised) and cpos[k] is
                                     member k's position in its full committee (the bitfield
                                     bit); NULL: full committees, position = index in the row */
  const uint32_t* co_index;       /* optional "committee order": the validator arrays of every
                                     instance are stored in committee order -- committee c
                                     occupies storage positions [coffs[c], coffs[c+1]) of
                                     [0, nval_global), which the committees partition -- and
                                     co_index[p - val_offset] is the validator index stored at
                                     position p.  The crosslink tallies then stream contiguous
                                     balances (no member gathers; `committee`/`cpos` unused) and
                                     CalculateRewards reads bit co_index[p] of the last bitfield.
                                     Requires every validator to match `kind` (else
                                     PZ_XLERR_LAYOUT in scal[PZ_SCAL_ERR_XL]). */
} pz_epoch_batch;

/* ---- T: block vote-cache tally (blockchain/core.go:300-345 calculateBlockVoteCache) ----
 * Each signed parent hash h has a dense slot id (host-assigned; the host keeps the 32-byte
 * hash -> slot map exactly like the Go map key).  A work item (attestation a, slot s) adds
 * every committee member of a whose bit is set and who is not yet in s's voter set:
 * totals[s] += balance[v].  Slots own an nval-bit dedup bitmap (words_per_slot u32 words).
 * Items of many blocks may share a launch as long as no balance changes between them
 * (balances change only in stateRecalc).  *err != 0 where Go would panic. */
typedef struct pz_vote_batch {
  const uint32_t* committee;   /* committee members (validator indices) */
  const uint64_t* coffs;       /* [ncomm + 1] */
  const uint32_t* att_comm;    /* [natt] committee id of each attestation */
  const uint8_t* bits;         /* CSR bitfields of the attestations */
  const uint64_t* boffs;       /* [natt + 1] */
  const uint32_t* item_att;    /* [nitems] */
  const uint32_t* item_slot;   /* [nitems] */
  uint64_t nitems;
  const uint64_t* balance;     /* [nval] */
  uint64_t nval;
  uint32_t* bitmaps;           /* [nslots][words_per_slot] in/out */
  uint64_t words_per_slot;     /* >= ceil(nval / 32) */
  uint64_t* totals;            /* [nslots] in/out (VoteTotalDeposit) */
  uint64_t* err;               /* [1] in/out */
  uint64_t val_offset;         /* validator-range shard: this rank holds
                                  validators [val_offset, val_offset + nval) of nval_global;
                                  balance and the bitmaps index v - val_offset and the members
                                  outside the range are skipped (another rank adds them) */
  uint64_t nval_global;        /* 0: no shard (nval_global = nval, val_offset = 0) */
} pz_vote_batch;

int pz_dev_vote_tally(const pz_vote_batch* b, void* stream);

/* Host-pointer form: same inputs; bitmaps/totals are read and written back in place. */
int pz_vote_tally(const uint32_t* committee, const uint64_t* coffs, uint64_t ncomm,
                  const uint32_t* att_comm, const uint8_t* bits, const uint64_t* boffs,
                  uint64_t natt, const uint32_t* item_att, const uint32_t* item_slot,
                  uint64_t nitems, const uint64_t* balance, uint64_t nval, uint32_t* bitmaps,
                  uint64_t nslots, uint64_t words_per_slot, uint64_t* totals);

typedef struct pz_comm pz_comm;  /* the ranks of a multi-GPU partition ("multi-GPU" below) */
/* The same tally sharded by validator range over the ranks of `comm`:
 * every local rank tallies the items' committee members in its 64-aligned validator range
 * [lo, hi) into its slice of the bitmaps (words [lo/32, hi/32) of every slot), and one RCCL
 * all-reduce (u64 sum) of the per-slot partial totals gives every rank the totals
 * (stateRecalc reads them, core.go:413-418).  Dedup stays exact: a voter's bit lives on the
 * one rank that owns it.  Host arrays as in pz_vote_tally; `totals` receives the global
 * totals; only the bitmap words of this process's local ranks are written back (one process
 * per GPU: each process holds its own slice). */
int pz_comm_vote_tally(const pz_comm* comm, const uint32_t* committee, const uint64_t* coffs, uint64_t ncomm,
                       const uint32_t* att_comm, const uint8_t* bits, const uint64_t* boffs, uint64_t natt,
                       const uint32_t* item_att, const uint32_t* item_slot, uint64_t nitems,
                       const uint64_t* balance, uint64_t nval, uint32_t* bitmaps, uint64_t nslots,
                       uint64_t words_per_slot, uint64_t* totals);

/* Pass 1 (pre-reward balances): classify/count, attester popcount, crosslink tallies. */
int pz_dev_epoch_count(const pz_epoch_batch* b, void* stream);
/* Pass 2 (after any cross-rank all-reduce): winners, active-list compaction when needed,
 * rewards in place and the post-reward total. */
int pz_dev_epoch_finish(const pz_epoch_batch* b, void* stream);

/* Multi-rank general rank path (not every validator active): between count and finish,
 * all-gather every rank's act_mask into gathered_mask[world][B][shard_words] (rank r owns the
 * global validators [r*64*shard_words, (r+1)*64*shard_words)), then call this to rebuild the
 * global compacted active list act_list[B][nval_global] on every rank; CalculateRewards
 * (casper/incentives.go:22-28) reads it by global rank position.  gblk is scratch
 * [B][ceil(nval_global/2048)] u32.  Instances with every validator active are skipped. */
int pz_dev_epoch_gather_compact(const pz_epoch_batch* b, const uint64_t* gathered_mask, uint32_t world,
                                uint64_t shard_words, uint32_t* gblk, void* stream);

/* ---- multi-GPU: communicators (RCCL over xGMI) ------------------------------------------
 * The reference is one Go process (ChainService.blockProcessing is one goroutine,
 * blockchain/service.go:229); nothing in it is distributed.  North_star shards the epoch by
 * validator range over the GPUs of one node and combines the participation and total-balance
 * sums with RCCL all-reduce.  A pz_comm names the ranks of that partition:
 *   pz_init_devices       one process drives ndev GPUs (ncclCommInitAll): the Go node's shape;
 *   pz_comm_init_rank     one process per GPU (ncclCommInitRank), the id from rank 0's
 *                         pz_comm_unique_id passed to every rank by the launcher;
 *   pz_comm_init_loopback `world` ranks in this process on ONE device, collectives by device
 *                         copies and a sum kernel (no RCCL): the sharded code path on a
 *                         one-GPU machine (tests);
 *   pz_comm_init_shm      one process per rank, ranks free to share a device: collectives
 *                         staged through host memory and a POSIX shared-memory group named
 *                         `name` (rank 0 creates it, O_EXCL; unlinked once every rank attached),
 *                         synchronous.  The one-process-per-GPU call sequence on a one-GPU
 *                         machine (tests, the bench's gloo rehearsal).  Every collective checks
 *                         that all ranks issued the same one (kind and sizes): a divergence fails
 *                         with PZ_EINVAL naming both calls, a rank missing for timeout_ms (0:
 *                         60 s) with PZ_EDEVICE -- where RCCL would hang.
 * librccl is resolved at run time (the copy already mapped into the process, else /opt/rocm's). */
#define PZ_COMM_ID_BYTES 128
typedef struct pz_comm pz_comm;
int  pz_comm_unique_id(uint8_t id[PZ_COMM_ID_BYTES]);
int  pz_comm_init_rank(const uint8_t id[PZ_COMM_ID_BYTES], int world, int rank, int device, pz_comm** out);
int  pz_init_devices(int ndev, const int* devices /* NULL: 0..ndev-1 */, pz_comm** out);
int  pz_comm_init_loopback(int world, int device, pz_comm** out);
int  pz_comm_init_shm(const char* name, int world, int rank, int device, uint32_t timeout_ms, pz_comm** out);
/* Collective timing: with timing on, every collective is bracketed by a HIP event pair on the
 * communicator's stream of each local rank (after its wait for the compute stream: the
 * collective's own time, exposed or overlapped).  pz_comm_collective_time returns the sum over
 * the collectives since the last call (the max over local ranks for each) and their count, and
 * restarts the sum; it waits for the pending collectives.  Each timed collective holds two
 * events per local rank until it is collected: a caller that leaves timing on collects
 * regularly (the bench collects once per timed run). */
int  pz_comm_set_timing(pz_comm* comm, int on);
int  pz_comm_collective_time(pz_comm* comm, double* ms, uint64_t* count);
/* world = ranks in the partition, nlocal = ranks this process drives (global ranks
 * first_rank .. first_rank+nlocal-1). */
int  pz_comm_size(const pz_comm* comm, int* world, int* nlocal, int* first_rank);
int  pz_comm_device(const pz_comm* comm, int local, int* device);
void pz_comm_free(pz_comm* comm);

/* H over the communicator: message batches shard with no collective.  Local rank i hashes
 * messages [n*r/world, n*(r+1)/world) of the batch (r = first_rank + i), on its own device,
 * all local ranks concurrently; out receives those digests (out_bytes each, at the message's
 * index).  A single-process communicator (pz_init_devices) covers the whole batch, which is
 * the multi-GPU form of pz_blake2b512_batch. */
int pz_comm_blake2b512_batch(const pz_comm* comm, const uint8_t* msgs, const uint64_t* offsets, uint64_t n,
                             uint8_t* out, uint32_t out_bytes);

/* ---- multi-GPU: the device-resident, validator-range-sharded epoch ----------------------
 * B independent epoch instances (the data-parallel part of stateRecalc, blockchain/core.go:
 * 433-464), described by host arrays over ALL validators; each local rank of `comm` uploads
 * its 64-aligned validator range [lo, hi) of every instance into its GPU's HBM (SoA,
 * instance-major) and the committee members inside it.  comm == NULL: one device, world 1.
 * When every validator is active and the committees partition the set, the validators are
 * stored in committee order (pz_epoch_batch.co_index): the crosslink tallies stream contiguous
 * balances and each rank holds a range of committee positions.  A step enqueues (no host sync):
 *   count -> RCCL all-reduce {scal, vote, total} -> [some validator inactive: all-gather of
 *   the active masks -> global compaction] -> finish -> all-reduce of the next-cycle totals,
 * the instances split in two parts so one part's collectives overlap the other's kernels.
 * In committee order, unless some attestation names a shard >= nrec (that panic depends on
 * the tallies), the step is one pass over the validators instead:
 *   bit count -> one stream (classify, crosslink tallies on the pre-reward balances, reward,
 *   next-cycle sum) -> winners -> one grouped RCCL collective (u64 sum of scal, u32 minimum
 *   of the winners)
 * (32 B per validator-epoch instead of 40).  Its ranks hold committee-aligned ranges, so the
 * vote/total of an attestation are complete on the rank holding its committee;
 * pz_epoch_state_tallies completes them everywhere.
 * Results are those of pz_dev_epoch_count/finish (bit-exact with the reference; panics
 * reported in scal[PZ_SCAL_ERR_*] with the balances untouched). */
typedef struct pz_epoch_host {
  uint32_t ninst;                  /* B */
  uint64_t nval;                   /* N validators per instance */
  const uint64_t* balance;         /* [B][N] */
  const uint64_t* start;           /* [B][N] */
  const uint64_t* end;             /* [B][N] */
  const uint64_t* dynasty;         /* [B] */
  const uint64_t* total_deposit;   /* [B] */
  uint32_t natt;                   /* pending attestations per instance */
  const uint8_t* bits;             /* CSR bitfields over B*natt attestations */
  const uint64_t* boffs;           /* [B*natt + 1], boffs[0] == 0 */
  const uint32_t* committee;       /* committee members (global validator indices) */
  const uint64_t* coffs;           /* [ncomm + 1], coffs[0] == 0 */
  uint64_t ncomm;
  const uint32_t* att_comm;        /* [B*natt] */
  const uint32_t* att_shard;       /* [B*natt] */
  uint32_t nrec;                   /* crosslink records per instance */
  const uint64_t* rec_dynasty;     /* [B][nrec].  dynasty, rec_dynasty, the committees and the
                                      attestations are copied by pz_epoch_state_new and fixed for
                                      the state's lifetime (no call updates them; the one-pass
                                      step's plan tables are built from them once).  A caller
                                      whose records or dynasty change makes a new state. */
  uint32_t layout;                 /* PZ_LAYOUT_AUTO: committee order when every validator is
                                      active and the committees partition the set, else index
                                      order; PZ_LAYOUT_INDEX: always index order;
                                      PZ_LAYOUT_TWOPASS: AUTO's layout, two-pass step */
} pz_epoch_host;
#define PZ_LAYOUT_AUTO    0
#define PZ_LAYOUT_INDEX   1
#define PZ_LAYOUT_TWOPASS 2  /* committee order as AUTO, but the two-pass step (A/B, tests) */
typedef struct pz_epoch_state pz_epoch_state;
int  pz_epoch_state_new(pz_comm* comm, int device, const pz_epoch_host* h, pz_epoch_state** out);
/* The state's options (no reference counterpart: placement and test controls of this library;
 * NULL or pz_epoch_state_new: every field 0).  There are no environment switches. */
typedef struct pz_epoch_options {
  uint64_t rebase_period;  /* u32-offset balances: steps between re-bases of the offsets (0: 2^29,
                              the product; larger values are clamped to it) */
  int window_only;         /* 1: one instance on one rank also takes the window pass (the
                              multi-instance one-pass kernel) instead of pz_epoch_one_kernel */
} pz_epoch_options;
int  pz_epoch_state_new_opts(pz_comm* comm, int device, const pz_epoch_host* h, const pz_epoch_options* opts,
                             pz_epoch_state** out);
int  pz_epoch_state_step(pz_epoch_state* st);
int  pz_epoch_state_sync(pz_epoch_state* st);
/* Local rank `local`'s validator range, device and compute stream (for event timing). */
int  pz_epoch_state_shard(const pz_epoch_state* st, int local, uint64_t* lo, uint64_t* hi, int* device,
                          void** stream);
/* From now on local rank `local` enqueues its steps on the caller's hipStream_t `stream` (of
 * that rank's device; NULL: back to the state's own stream).  Work already enqueued is waited
 * for first.  Several states bound to one stream step in issue order (e.g. a caller rotating
 * over state sets larger than the caches, or ordering the step after its own kernels). */
int  pz_epoch_state_bind_stream(pz_epoch_state* st, int local, void* stream);
/* After a step (synchronises): the balances of the hi-lo validators local rank `local` holds
 * ([B][hi-lo], in its storage order: pz_epoch_state_validators names them), and the reduced
 * scal [B][PZ_SCAL_COUNT], vote / total [B][natt] and winners [B][nrec] (any may be NULL). */
int  pz_epoch_state_results(pz_epoch_state* st, int local, uint64_t* balance, uint64_t* scal, uint64_t* vote,
                            uint64_t* total, uint32_t* winner);
/* The validator index held at each of local rank `local`'s hi-lo storage positions: lo.. in
 * index order; the members of the committees, in committee order, in the committee-order
 * layout (pz_epoch_batch.co_index), which *committee_order reports. */
int  pz_epoch_state_validators(const pz_epoch_state* st, int local, uint32_t* index);
/* The sharded one-pass step leaves each attestation's vote/total complete only on the rank
 * holding its committee (its winners are exact everywhere: proposed by that rank, combined by
 * a minimum all-reduce); this collective (every rank calls it) completes them on every rank
 * for pz_epoch_state_results.  A no-op for the other steps, and for a step whose tallies it
 * has already completed (calling it twice never sums complete tallies again). */
int  pz_epoch_state_tallies(pz_epoch_state* st);
/* *committee_order: 0 index order, 1 committee order (two-pass step), 2 committee order with
 * the one-pass step. */
int  pz_epoch_state_layout(const pz_epoch_state* st, int* committee_order);
/* The widths the one-pass stream reads per validator-epoch (the roofline's bytes; no reference
 * counterpart -- the Go state holds *pb.ValidatorRecord, types/state.go, messages.pb.go:803-809):
 * *balance_bytes 4 when the balances are held as u32 offsets from a per-instance u64 base
 * (every instance's balances within 2^30 of each other; results are the u64 values, exact mod
 * 2^64; the state re-bases the offsets every 2^29 steps), else 8; *dynasty_bytes 4, 8 or 16 for
 * the {start, end} column (16-, 32-bit saturated, or the u64 columns).  The widest part wins. */
int  pz_epoch_state_columns(const pz_epoch_state* st, uint32_t* balance_bytes, uint32_t* dynasty_bytes);
void pz_epoch_state_free(pz_epoch_state* st);
/* Host only (no device call): the layout a pz_epoch_state would choose for h (as
 * pz_epoch_state_layout) and global rank `rank`'s storage positions [lo, hi) in a world of
 * `world` ranks.  Lets a launcher size each rank's memory before any device is opened. */
int  pz_epoch_plan(const pz_epoch_host* h, int world, int rank, uint64_t* lo, uint64_t* hi, int* committee_order);

/* ---- block pipeline: sync replay of serialized blocks ---------------------------------
 * A chain object runs blocks through the reference's ChainService.blockProcessing
 * (blockchain/service.go:229-363) and updateHead (:170-227) over BeaconChain (core.go),
 * starting from the genesis states of `nval` validators (types/state.go:44-112).  Blocks are
 * canonical proto3 BeaconBlock encodings (messages.proto:37-46), CSR (offsets[n+1]), as they
 * arrive from the sync service (sync/service.go:147-164); a block that is not the canonical
 * encoding of its own decoding is PZ_EINVAL (the reference hashes proto.Marshal of the decoded
 * block).  Results per block and per attestation are what the reference stores or logs:
 * block digest (Block.Hash), attestation Key/Hash (saveAttestation, Attestation.Hash) and the
 * 64-byte processAttestation message digest (core.go:277-290).  Where the reference panics
 * the call returns PZ_EINDEX and the chain is unusable afterwards.  Thread-safe per chain. */
#define PZ_BLOCK_PROCESSED            0  /* became the candidate (and maybe a cycle transition) */
#define PZ_BLOCK_NO_PARENT            1  /* parent never saved, slot > 1 (service.go:261-269)   */
#define PZ_BLOCK_ATTS_REJECTED        2  /* last attestation failed / none (service.go:304-306)  */
#define PZ_BLOCK_SAVED_NOT_CANDIDATE  3  /* saved, a candidate was already chosen (:331-333)     */
#define PZ_ATT_PROCESSED              0
#define PZ_ATT_NOT_PROCESSED          1  /* its block was dropped before processAttestation       */
#define PZ_ATT_SLOT_HIGH              2  /* core.go:244-248 */
#define PZ_ATT_SLOT_LOW               3  /* core.go:249-253 */
#define PZ_ATT_JUSTIFIED              4  /* core.go:255-259 */
#define PZ_ATT_NO_COMMITTEE           5  /* core.go:373     */
#define PZ_ATT_BITFIELD_LEN           6  /* core.go:379-382 */
#define PZ_ATT_TRAILING_BITS          7  /* core.go:385-392 */

/* ---- §8f: processAttestation's checks for a batch, one GPU lane per attestation --------
 * blockchain/core.go:240-297 with getSignedParentHashes (:348-360), getAttesterIndices
 * (:363-374) and validateAttesterBitfields (:377-394), in Go's order.  Attestation i was
 * carried by a block of slot block_slot[i]; the chain state is the one processAttestation
 * reads (CrystallizedState.LastJustifiedSlot / LastStateRecalc / ShardAndCommitteesForSlots,
 * len(ActiveState.RecentBlockHashes)).  status[i] receives PZ_ATT_PROCESSED or the first
 * check that failed (PZ_ATT_*), or PZ_ERANGE / PZ_EINDEX where Go panics (the slice bounds
 * of :353, the committee index of :367).  committee[i] (optional) receives the committee id
 * (UINT32_MAX if not reached) and parents_start[i] (optional) the first RecentBlockHashes
 * index the signed parent hashes start at. */
typedef struct pz_att_check_batch {
  uint64_t natt;
  const uint64_t* slot;            /* AttestationRecord.Slot */
  const uint64_t* justified_slot;  /* .JustifiedSlot */
  const uint64_t* shard_id;        /* .ShardId */
  const uint64_t* n_oblique;       /* len(.ObliqueParentHashes) */
  const uint8_t*  bits;            /* .AttesterBitfield, CSR */
  const uint64_t* boffs;           /* natt+1 */
  const uint64_t* block_slot;      /* SlotNumber of the carrying block */
  uint64_t last_justified_slot, last_state_recalc, n_recent;
  uint64_t narr;                   /* len(ShardAndCommitteesForSlots) */
  const uint64_t* arr_offs;        /* narr+1: array a = entries arr_offs[a] .. arr_offs[a+1] */
  const uint64_t* arr_shard;       /* entry -> ShardId */
  const uint32_t* arr_comm;        /* entry -> committee id */
  const uint64_t* coffs;           /* committee c has coffs[c+1] - coffs[c] members */
  int32_t*  status;
  uint32_t* committee;
  uint64_t* parents_start;
  const uint8_t* last_byte;        /* optional (NULL: read from bits): natt bytes, the last byte of
                                      each bitfield (bits[boffs[i+1]-1]; any value when empty), a
                                      caller-side column so the trailing-bits check streams 1 B per
                                      attestation instead of touching every bitfield line */
} pz_att_check_batch;
int pz_check_attestations(const pz_att_check_batch* b);                  /* host pointers */
int pz_dev_check_attestations(const pz_att_check_batch* b, void* stream); /* device pointers */

typedef struct pz_block_result {
  uint8_t hash[32];      /* Block.Hash() */
  int32_t status;        /* PZ_BLOCK_* */
  int32_t transition;    /* 1: stateRecalc ran for this block */
  uint32_t first_att;    /* index of its first attestation in att_out */
  uint32_t natt;
} pz_block_result;

typedef struct pz_att_result {
  int32_t status;        /* PZ_ATT_* */
  uint32_t msg_len;      /* processAttestation message length */
  uint8_t key[32];       /* Attestation.Key()  (types/attestation.go:61-77) */
  uint8_t hash[32];      /* Attestation.Hash() (types/attestation.go:49-59) */
  uint8_t msg_digest[64];/* blake2b.Sum512(msg) (core.go:290) */
} pz_att_result;

typedef struct pz_chain pz_chain;
int  pz_chain_new(uint64_t nval, int device, pz_chain** out);
/* NewBeaconChain over a database that holds a CrystallizedState (blockchain/core.go:86-95):
 * the chain resumes from the stored encoding `cstate` (the bytes pz_chain_state_bytes returns
 * for the chain's CrystallizedState, which updateHead persists, core.go:170-177) with the
 * genesis ActiveState, exactly as the reference reloads; `saved_hashes` (32 bytes each) are
 * the block hashes the database holds (hasBlock, core.go:591-601), so their children are
 * processed.  PZ_EINVAL when the bytes do not decode (proto.Unmarshal's error). */
int  pz_chain_new_from_state(const uint8_t* cstate, uint64_t len, const uint8_t* saved_hashes, uint64_t nsaved,
                             int device, pz_chain** out);
/* One chain over the ranks of `comm` (blockchain/core.go:300-345,
 * 398-497): each local rank holds the 64-aligned validator range [lo, hi) of the balances, its
 * columns of every vote-cache voter bitmap (so a voter's dedup bit lives on one rank) and its
 * partial VoteTotalDeposit sums; a stateRecalc all-reduces the 64 totals the justification
 * loop reads (65 words with the tally panic flag) and runs the epoch sharded like
 * pz_epoch_state (partial crosslink tallies, bit counts and next-cycle balances all-reduced,
 * rewards on each range).  The block walk, digests and messages run on local rank 0 of every
 * process (one process per GPU replays the same blocks; the device work is split).  Genesis
 * only: every validator stays active, so rank == index.  `comm` must outlive the chain. */
int  pz_chain_new_comm(uint64_t nval, pz_comm* comm, pz_chain** out);
void pz_chain_free(pz_chain* chain);
/* The engine's options (no reference counterpart: placement and test controls; every field 0
 * is the product's choice).  Set them before the chain's first pz_chain_process_blocks call:
 * afterwards a change of tally_forms fails with PZ_EINVAL (msg_batch may change at any time). */
typedef struct pz_chain_options {
  uint64_t msg_batch;    /* processAttestation messages digested in batches of at least this many,
                            sent while the walk goes on (0: one batch at the end of the call) */
  uint32_t tally_forms;  /* tests: the vote-cache tally's general forms forced (PZ_TALLY_*) */
} pz_chain_options;
#define PZ_TALLY_PER_ATTESTATION 1u  /* the per-attestation tally instead of the committee-grouped one */
#define PZ_TALLY_BITS_ROWS       2u  /* every bitfield in the row array, none inline in its record */
#define PZ_TALLY_ID_ROWS         4u  /* every attestation's parent ids as an explicit row, no run */
int  pz_chain_set_options(pz_chain* chain, const pz_chain_options* opts);
/* Number of attestations in a batch of serialized blocks (host only; sizes att_out). */
int  pz_count_attestations(const uint8_t* blocks, const uint64_t* offsets, uint64_t n, uint64_t* count);
/* att_out: capacity att_cap >= the total number of attestations in the batch.
 * A reference panic returns PZ_EINDEX and poisons the chain.  A stateRecalc's device epoch
 * (processCrosslinks, CalculateRewards) is collected at the next transition or at the end of
 * the call, so its panic is reported up to 63 blocks later: the message names the transition's
 * block index and slot, and the result rows of the blocks after that block are undefined (the
 * reference stops at it, blockchain/service.go:345-354). */
int  pz_chain_process_blocks(pz_chain* chain, const uint8_t* blocks, const uint64_t* offsets, uint64_t n,
                             pz_block_result* block_out, pz_att_result* att_out, uint64_t att_cap);
/* State roots (types/state.go:138-149, 237-248): out[0..31] chain ActiveState, [32..63] chain
 * CrystallizedState, [64..127] the candidate's (zero when *has_candidate == 0). */
int  pz_chain_roots(pz_chain* chain, uint8_t out[4 * 32], int* has_candidate);
/* Persistence format: the proto3 encoding the reference stores under activeStateLookupKey /
 * crystallizedStateLookupKey (PersistActiveState / PersistCrystallizedState,
 * blockchain/core.go:161-177, schema.go:17-27) — the bytes the state roots hash.
 * which: 0 chain ActiveState, 1 chain CrystallizedState, 2 / 3 the candidate's (PZ_EINVAL
 * when there is no candidate).  *len receives the size; bytes are written when cap >= *len. */
int  pz_chain_state_bytes(pz_chain* chain, int which, uint8_t* out, uint64_t cap, uint64_t* len);
/* The block vote cache: *count entries (0 when the map is nil); fills hashes[32*i] and
 * totals[i] (VoteTotalDeposit) when cap >= *count. */
int  pz_chain_vote_totals(pz_chain* chain, uint8_t* hashes, uint64_t* totals, uint64_t cap, uint64_t* count);
/* Observability (no reference counterpart; the Go node's pprof wall profile of the same
 * phases): the engine's cumulative wall seconds per phase of pz_chain_process_blocks since the
 * chain was created, out[0..n): parse, digest batch, attestation checks, vote queueing, tally
 * flushes, stateRecalc, message digests, the walk, the whole call, attestation counting, arena
 * waits, message sends / hash log / waits, the tally totals' wait, then two counts (tally-total
 * polls that fell back to the event wait; queued attestations with an explicit parent-id row).
 * The checks and vote queueing are clocked only by the A/B library (they read 0 here).
 * Returns the number of slots the library keeps. */
int  pz_chain_phase_times(pz_chain* chain, double* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* PRYSM_HIP_H */
