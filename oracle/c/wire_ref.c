/* ORACLE (test infrastructure only) — C restatement of the proto3 encoding of
 * CrystallizedState.validators (repeated ValidatorRecord = 11), in the reference's own data
 * layout: records are heap structs reached through a pointer array, like Go's
 * []*pb.ValidatorRecord.  The control flow follows the generated marshaller behind gogo
 * proto.Marshal (types/state.go:141,240): a Size() pass over every record to allocate,
 * then a MarshalTo() pass writing fields in ascending number, skipping zero scalars and
 * empty bytes (messages.pb.go:803-809 struct tags).  Used as bench.py's wire
 * cpu_baseline ("port") and pinned against Google's protobuf runtime in tests. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t public_key, withdrawal_shard;
  uint8_t* withdrawal_address; size_t withdrawal_address_len;
  uint8_t* randao_commitment; size_t randao_commitment_len;
  uint64_t balance, start_dynasty, end_dynasty;
} wire_validator;

typedef struct { wire_validator** v; size_t n; } wire_set;

static size_t sov(uint64_t x) { size_t n = 1; while (x >= 0x80) { x >>= 7; ++n; } return n; }

static uint8_t* enc_varint(uint8_t* p, uint64_t x) {
  while (x >= 0x80) { *p++ = (uint8_t)(x | 0x80); x >>= 7; }
  *p++ = (uint8_t)x;
  return p;
}

static size_t rec_size(const wire_validator* m) {
  size_t n = 0;
  if (m->public_key) n += 1 + sov(m->public_key);
  if (m->withdrawal_shard) n += 1 + sov(m->withdrawal_shard);
  if (m->withdrawal_address_len) n += 1 + sov(m->withdrawal_address_len) + m->withdrawal_address_len;
  if (m->randao_commitment_len) n += 1 + sov(m->randao_commitment_len) + m->randao_commitment_len;
  if (m->balance) n += 1 + sov(m->balance);
  if (m->start_dynasty) n += 1 + sov(m->start_dynasty);
  if (m->end_dynasty) n += 1 + sov(m->end_dynasty);
  return n;
}

static uint8_t* rec_write(const wire_validator* m, uint8_t* p) {
  if (m->public_key) { *p++ = 0x08; p = enc_varint(p, m->public_key); }
  if (m->withdrawal_shard) { *p++ = 0x10; p = enc_varint(p, m->withdrawal_shard); }
  if (m->withdrawal_address_len) {
    *p++ = 0x1a; p = enc_varint(p, m->withdrawal_address_len);
    memcpy(p, m->withdrawal_address, m->withdrawal_address_len); p += m->withdrawal_address_len;
  }
  if (m->randao_commitment_len) {
    *p++ = 0x22; p = enc_varint(p, m->randao_commitment_len);
    memcpy(p, m->randao_commitment, m->randao_commitment_len); p += m->randao_commitment_len;
  }
  if (m->balance) { *p++ = 0x28; p = enc_varint(p, m->balance); }
  if (m->start_dynasty) { *p++ = 0x30; p = enc_varint(p, m->start_dynasty); }
  if (m->end_dynasty) { *p++ = 0x38; p = enc_varint(p, m->end_dynasty); }
  return p;
}

/* SoA columns (NULL = zero / empty) -> heap records behind a pointer array. */
void* oracle_wire_build(const uint64_t* pk, const uint64_t* shard, const uint8_t* wa, const uint64_t* wa_offs,
                        const uint8_t* rc, const uint64_t* rc_offs, const uint64_t* bal, const uint64_t* start,
                        const uint64_t* end, size_t n) {
  wire_set* s = calloc(1, sizeof *s);
  s->n = n;
  s->v = calloc(n ? n : 1, sizeof *s->v);
  for (size_t i = 0; i < n; ++i) {
    wire_validator* m = calloc(1, sizeof *m);
    m->public_key = pk ? pk[i] : 0;
    m->withdrawal_shard = shard ? shard[i] : 0;
    m->balance = bal ? bal[i] : 0;
    m->start_dynasty = start ? start[i] : 0;
    m->end_dynasty = end ? end[i] : 0;
    if (wa_offs && wa_offs[i + 1] > wa_offs[i]) {
      m->withdrawal_address_len = wa_offs[i + 1] - wa_offs[i];
      m->withdrawal_address = malloc(m->withdrawal_address_len);
      memcpy(m->withdrawal_address, wa + wa_offs[i], m->withdrawal_address_len);
    }
    if (rc_offs && rc_offs[i + 1] > rc_offs[i]) {
      m->randao_commitment_len = rc_offs[i + 1] - rc_offs[i];
      m->randao_commitment = malloc(m->randao_commitment_len);
      memcpy(m->randao_commitment, rc + rc_offs[i], m->randao_commitment_len);
    }
    s->v[i] = m;
  }
  return s;
}

void oracle_wire_free(void* h) {
  wire_set* s = h;
  for (size_t i = 0; i < s->n; ++i) {
    free(s->v[i]->withdrawal_address);
    free(s->v[i]->randao_commitment);
    free(s->v[i]);
  }
  free(s->v);
  free(s);
}

/* Encode every record framed as field `field` (single-byte tag, field <= 15).  Returns the
 * encoded length; writes nothing when it exceeds cap (out may be NULL to query). */
uint64_t oracle_wire_validators(void* h, uint32_t field, uint8_t* out, uint64_t cap) {
  const wire_set* s = h;
  uint64_t total = 0;
  for (size_t i = 0; i < s->n; ++i) {
    const size_t r = rec_size(s->v[i]);
    total += 1 + sov(r) + r;
  }
  if (!out || total > cap) return total;
  uint8_t* p = out;
  for (size_t i = 0; i < s->n; ++i) {
    *p++ = (uint8_t)((field << 3) | 2);
    p = enc_varint(p, rec_size(s->v[i]));
    p = rec_write(s->v[i], p);
  }
  return total;
}
