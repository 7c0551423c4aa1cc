/* ORACLE (test infrastructure only) — C restatement of the proto3 encoding of
 * CrystallizedState.validators (repeated ValidatorRecord = 11), in the reference's own data
 * layout: records are heap structs reached through a pointer array, like Go's
 * []*pb.ValidatorRecord.  The control flow follows the generated marshaller behind gogo
 * proto.Marshal (types/state.go:141,240): a Size() pass over every record to allocate,
 * then a MarshalTo() pass writing fields in ascending number, skipping zero scalars and
 * empty bytes (messages.pb.go:803-809 struct tags).  The second half restates
 * golang/protobuf's marshal of AttestationRecord (types/attestation.go:51; messages.pb.go:
 * 889-896) the same way.  Used as bench.py's wire / wire_att cpu_baselines ("port") and
 * pinned against Google's protobuf runtime in tests. */
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

/* ---- AttestationRecord (messages.pb.go:889-896), the record Attestation.Hash() marshals -- */
typedef struct {
  uint64_t slot, shard_id, justified_slot;
  uint8_t* jbh; size_t jbh_len;
  uint8_t* sbh; size_t sbh_len;
  uint8_t* bitfield; size_t bitfield_len;
  uint8_t** oblique; size_t* oblique_len; size_t n_oblique;
  uint64_t* sig; size_t n_sig;
} wire_att;

typedef struct { wire_att** a; size_t n; } wire_att_set;

static uint8_t* dup_bytes(const uint8_t* src, size_t len) {
  uint8_t* p = malloc(len ? len : 1);
  if (len) memcpy(p, src, len);
  return p;
}

void* oracle_wire_att_build(const uint64_t* slot, const uint64_t* shard, const uint64_t* js, const uint8_t* jbh,
                            const uint64_t* jbh_offs, const uint8_t* sbh, const uint64_t* sbh_offs, const uint8_t* bf,
                            const uint64_t* bf_offs, const uint8_t* obl, const uint64_t* obl_offs,
                            const uint64_t* obl_first, const uint64_t* sig, const uint64_t* sig_first, size_t n) {
  wire_att_set* s = calloc(1, sizeof *s);
  s->n = n;
  s->a = calloc(n ? n : 1, sizeof *s->a);
  for (size_t i = 0; i < n; ++i) {
    wire_att* m = calloc(1, sizeof *m);
    m->slot = slot[i];
    m->shard_id = shard[i];
    m->justified_slot = js[i];
    m->jbh_len = jbh_offs[i + 1] - jbh_offs[i];
    m->jbh = dup_bytes(jbh + jbh_offs[i], m->jbh_len);
    m->sbh_len = sbh_offs[i + 1] - sbh_offs[i];
    m->sbh = dup_bytes(sbh + sbh_offs[i], m->sbh_len);
    m->bitfield_len = bf_offs[i + 1] - bf_offs[i];
    m->bitfield = dup_bytes(bf + bf_offs[i], m->bitfield_len);
    m->n_oblique = obl_first[i + 1] - obl_first[i];
    m->oblique = calloc(m->n_oblique ? m->n_oblique : 1, sizeof *m->oblique);
    m->oblique_len = calloc(m->n_oblique ? m->n_oblique : 1, sizeof *m->oblique_len);
    for (size_t e = 0; e < m->n_oblique; ++e) {
      const uint64_t k = obl_first[i] + e;
      m->oblique_len[e] = obl_offs[k + 1] - obl_offs[k];
      m->oblique[e] = dup_bytes(obl + obl_offs[k], m->oblique_len[e]);
    }
    m->n_sig = sig_first[i + 1] - sig_first[i];
    m->sig = (uint64_t*)dup_bytes((const uint8_t*)(sig + sig_first[i]), m->n_sig * 8);
    s->a[i] = m;
  }
  return s;
}

void oracle_wire_att_free(void* h) {
  wire_att_set* s = h;
  for (size_t i = 0; i < s->n; ++i) {
    wire_att* m = s->a[i];
    free(m->jbh); free(m->sbh); free(m->bitfield); free(m->sig);
    for (size_t e = 0; e < m->n_oblique; ++e) free(m->oblique[e]);
    free(m->oblique); free(m->oblique_len); free(m);
  }
  free(s->a);
  free(s);
}

static size_t att_size(const wire_att* m, size_t* sigb) {
  size_t n = 0, sb = 0;
  if (m->slot) n += 1 + sov(m->slot);
  if (m->shard_id) n += 1 + sov(m->shard_id);
  if (m->justified_slot) n += 1 + sov(m->justified_slot);
  if (m->jbh_len) n += 1 + sov(m->jbh_len) + m->jbh_len;
  if (m->sbh_len) n += 1 + sov(m->sbh_len) + m->sbh_len;
  if (m->bitfield_len) n += 1 + sov(m->bitfield_len) + m->bitfield_len;
  for (size_t e = 0; e < m->n_oblique; ++e) n += 1 + sov(m->oblique_len[e]) + m->oblique_len[e];
  for (size_t e = 0; e < m->n_sig; ++e) sb += sov(m->sig[e]);
  if (sb) n += 1 + sov(sb) + sb;
  *sigb = sb;
  return n;
}

static uint8_t* put_bytes_field(uint8_t* p, uint8_t tag, const uint8_t* b, size_t len) {
  *p++ = tag;
  p = enc_varint(p, len);
  memcpy(p, b, len);
  return p + len;
}

/* Marshal every record bare, back to back (offs[n+1] receives the record starts): a Size()
 * pass then a MarshalTo() pass per record, like proto.Marshal.  Returns the total length. */
uint64_t oracle_wire_attestations(void* h, uint8_t* out, uint64_t cap, uint64_t* offs) {
  const wire_att_set* s = h;
  uint64_t total = 0;
  for (size_t i = 0; i < s->n; ++i) {
    size_t sb;
    total += att_size(s->a[i], &sb);
  }
  if (!out || total > cap) return total;
  uint8_t* p = out;
  for (size_t i = 0; i < s->n; ++i) {
    const wire_att* m = s->a[i];
    size_t sb;
    (void)att_size(m, &sb);
    if (offs) offs[i] = (uint64_t)(p - out);
    if (m->slot) { *p++ = 0x08; p = enc_varint(p, m->slot); }
    if (m->shard_id) { *p++ = 0x10; p = enc_varint(p, m->shard_id); }
    if (m->justified_slot) { *p++ = 0x18; p = enc_varint(p, m->justified_slot); }
    if (m->jbh_len) p = put_bytes_field(p, 0x22, m->jbh, m->jbh_len);
    if (m->sbh_len) p = put_bytes_field(p, 0x2a, m->sbh, m->sbh_len);
    if (m->bitfield_len) p = put_bytes_field(p, 0x32, m->bitfield, m->bitfield_len);
    for (size_t e = 0; e < m->n_oblique; ++e) p = put_bytes_field(p, 0x3a, m->oblique[e], m->oblique_len[e]);
    if (sb) {
      *p++ = 0x42;
      p = enc_varint(p, sb);
      for (size_t e = 0; e < m->n_sig; ++e) p = enc_varint(p, m->sig[e]);
    }
  }
  if (offs) offs[s->n] = total;
  return total;
}
