/* ORACLE (test infrastructure only) — C restatement of the reference's epoch T/R path in
 * the reference's own data layout: validators and attestations are heap records reached
 * through pointer arrays, like Go's []*pb.ValidatorRecord / []*pb.AttestationRecord, and
 * the loops are the Go loops (single goroutine).  Used as bench.py's epoch cpu_baseline
 * ("port") and cross-checked against oracle/epoch_np.py in tests.
 *   casper/validator.go:45-53 ActiveValidatorIndices     casper/validator.go:93-102 deposit
 *   casper/incentives.go:14-32 CalculateRewards          blockchain/core.go:502-558 crosslinks
 *   blockchain/core.go:459-464 next-cycle balance        utils/checkbit.go:4-23 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t public_key, withdrawal_shard;
  uint8_t* withdrawal_address; size_t withdrawal_address_len;
  uint8_t* randao_commitment; size_t randao_commitment_len;
  uint64_t balance, start_dynasty, end_dynasty;
} validator_record;

typedef struct {
  uint64_t slot, shard_id, justified_slot;
  uint8_t* attester_bitfield; size_t bitfield_len;
} attestation_record;

typedef struct { uint64_t dynasty; uint64_t slot; int64_t blockhash_from; } crosslink_record;

typedef struct { uint64_t shard_id; uint32_t* committee; size_t len; } shard_committee;
typedef struct { shard_committee* arr; size_t len; } shard_committee_array;

typedef struct {
  validator_record** validators; size_t nval;
  attestation_record** pending; size_t natt;
  shard_committee_array* committees; size_t nslots;
  crosslink_record* records; size_t nrec;
  uint64_t dynasty, total_deposits, last_state_recalc;
  /* outputs */
  int applied; uint64_t next_balance; int panicked;
} epoch_ctx;

static int check_bit(const uint8_t* bf, size_t len, long index, int* panic) {
  long chunk = (index + 1) / 8, loc = (index + 1) % 8;
  if (loc == 0) loc = 8; else chunk++;
  if (chunk - 1 < 0 || (size_t)(chunk - 1) >= len) { *panic = 1; return 0; }
  return (bf[chunk - 1] >> (8 - loc)) % 2 != 0;
}

static uint8_t bit_set_count(uint8_t v) {
  v = (v & 0x55) + ((v >> 1) & 0x55);
  v = (v & 0x33) + ((v >> 2) & 0x33);
  return (v + (v >> 4)) & 0xF;
}

static uint32_t* active_indices(epoch_ctx* e, size_t* n) {
  uint32_t* out = NULL; size_t cap = 0, k = 0;
  for (size_t i = 0; i < e->nval; ++i) {
    validator_record* v = e->validators[i];
    if (v->start_dynasty <= e->dynasty && e->dynasty < v->end_dynasty) {
      if (k == cap) { cap = cap ? cap * 2 : 16; out = realloc(out, cap * sizeof *out); }
      out[k++] = (uint32_t)i;
    }
  }
  *n = k;
  return out;
}

static uint64_t attesters_total_deposit(epoch_ctx* e) {
  long bits = 0;
  for (size_t a = 0; a < e->natt; ++a)
    for (size_t j = 0; j < e->pending[a]->bitfield_len; ++j) bits += bit_set_count(e->pending[a]->attester_bitfield[j]);
  return (uint64_t)bits * 32u;
}

static shard_committee* attester_indices(epoch_ctx* e, attestation_record* a) {
  uint64_t idx = a->slot - e->last_state_recalc;
  if (idx >= e->nslots) return NULL;
  shard_committee_array* arr = &e->committees[idx];
  for (size_t i = 0; i < arr->len; ++i) if (arr->arr[i].shard_id == a->shard_id) return &arr->arr[i];
  return NULL;
}

static void process_crosslinks(epoch_ctx* e, uint64_t slot) {
  for (size_t k = 0; k < e->natt; ++k) {
    attestation_record* a = e->pending[k];
    shard_committee* sc = attester_indices(e, a);
    if (!sc) { e->panicked = 1; return; }
    uint64_t total = 0, vote = 0;
    for (size_t i = 0; i < sc->len; ++i) total += e->validators[sc->committee[i]]->balance;
    for (size_t i = 0; i < sc->len; ++i)
      if (check_bit(a->attester_bitfield, a->bitfield_len, (long)i, &e->panicked))
        vote += e->validators[sc->committee[i]]->balance;
    if (e->panicked) return;
    if (3 * vote < 2 * total) continue;  /* Go's && short-circuits before the record index */
    if (a->shard_id >= e->nrec) { e->panicked = 1; return; }
    if (e->dynasty > e->records[a->shard_id].dynasty) {
      e->records[a->shard_id].dynasty = e->dynasty;
      e->records[a->shard_id].slot = slot;
      e->records[a->shard_id].blockhash_from = (int64_t)k;
    }
  }
}

static void calculate_rewards(epoch_ctx* e) {
  size_t na;
  uint32_t* act = active_indices(e, &na);
  uint64_t dep = attesters_total_deposit(e);
  e->applied = 0;
  if (dep * 3 >= e->total_deposits * 2) {
    e->applied = 1;
    for (size_t i = 0; i < na; ++i) {
      attestation_record* last = e->pending[e->natt - 1];
      int voted = check_bit(last->attester_bitfield, last->bitfield_len, (long)act[i], &e->panicked);
      if (e->panicked) break;
      if (voted) e->validators[i]->balance += 1; else e->validators[i]->balance -= 1;
    }
  }
  free(act);
}

/* The data-parallel part of stateRecalc (core.go:433-464) on one instance. */
void oracle_epoch_run(epoch_ctx* e, uint64_t slot) {
  e->panicked = 0;
  process_crosslinks(e, slot);
  if (e->panicked) return;
  calculate_rewards(e);
  if (e->panicked) return;
  size_t na;
  uint32_t* act = active_indices(e, &na);
  uint64_t s = 0;
  for (size_t i = 0; i < na; ++i) s += e->validators[act[i]]->balance;
  free(act);
  e->next_balance = s;
}

/* Build the AoS/pointer layout from SoA arrays (not timed). */
epoch_ctx* oracle_epoch_build(const uint64_t* start, const uint64_t* end, const uint64_t* balance, size_t nval,
                              const uint8_t* bits, const uint64_t* boffs, const uint64_t* att_slot,
                              const uint32_t* att_shard, size_t natt, const uint32_t* committee,
                              const uint64_t* coffs, const uint32_t* comm_slot, const uint32_t* comm_shard,
                              size_t ncomm, const uint64_t* rec_dynasty, size_t nrec, uint64_t dynasty,
                              uint64_t total_deposits) {
  epoch_ctx* e = calloc(1, sizeof *e);
  e->nval = nval;
  e->validators = malloc(nval * sizeof(validator_record*));
  for (size_t i = 0; i < nval; ++i) {
    validator_record* v = calloc(1, sizeof *v);
    v->start_dynasty = start[i]; v->end_dynasty = end[i]; v->balance = balance[i];
    e->validators[i] = v;
  }
  e->natt = natt;
  e->pending = malloc((natt ? natt : 1) * sizeof(attestation_record*));
  for (size_t a = 0; a < natt; ++a) {
    attestation_record* r = calloc(1, sizeof *r);
    r->slot = att_slot[a]; r->shard_id = att_shard[a];
    r->bitfield_len = boffs[a + 1] - boffs[a];
    r->attester_bitfield = malloc(r->bitfield_len ? r->bitfield_len : 1);
    memcpy(r->attester_bitfield, bits + boffs[a], r->bitfield_len);
    e->pending[a] = r;
  }
  e->nslots = 64;
  e->committees = calloc(64, sizeof(shard_committee_array));
  for (size_t c = 0; c < ncomm; ++c) {
    shard_committee_array* arr = &e->committees[comm_slot[c]];
    arr->arr = realloc(arr->arr, (arr->len + 1) * sizeof(shard_committee));
    shard_committee* sc = &arr->arr[arr->len++];
    sc->shard_id = comm_shard[c];
    sc->len = coffs[c + 1] - coffs[c];
    sc->committee = malloc((sc->len ? sc->len : 1) * sizeof(uint32_t));
    memcpy(sc->committee, committee + coffs[c], sc->len * sizeof(uint32_t));
  }
  e->nrec = nrec;
  e->records = calloc(nrec, sizeof(crosslink_record));
  for (size_t s = 0; s < nrec; ++s) { e->records[s].dynasty = rec_dynasty[s]; e->records[s].blockhash_from = -1; }
  e->dynasty = dynasty;
  e->total_deposits = total_deposits;
  return e;
}

void oracle_epoch_results(const epoch_ctx* e, uint64_t* balance, int64_t* winner, int* applied,
                          uint64_t* next_balance, int* panicked) {
  for (size_t i = 0; i < e->nval; ++i) balance[i] = e->validators[i]->balance;
  for (size_t s = 0; s < e->nrec; ++s) winner[s] = e->records[s].blockhash_from;
  *applied = e->applied; *next_balance = e->next_balance; *panicked = e->panicked;
}

void oracle_epoch_free(epoch_ctx* e) {
  for (size_t i = 0; i < e->nval; ++i) free(e->validators[i]);
  free(e->validators);
  for (size_t a = 0; a < e->natt; ++a) { free(e->pending[a]->attester_bitfield); free(e->pending[a]); }
  free(e->pending);
  for (size_t s = 0; s < e->nslots; ++s) {
    for (size_t i = 0; i < e->committees[s].len; ++i) free(e->committees[s].arr[i].committee);
    free(e->committees[s].arr);
  }
  free(e->committees);
  free(e->records);
  free(e);
}
