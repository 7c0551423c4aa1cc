/* ORACLE (test infrastructure only) — C restatement of processAttestation's checks
 * (blockchain/core.go:240-297 with getSignedParentHashes :348-360, getAttesterIndices
 * :363-374, validateAttesterBitfields :377-394) over attestations reached through a pointer
 * array, like Go's []*pb.AttestationRecord, one at a time (the reference's loop,
 * blockchain/service.go:282-296).  Used as bench.py's attcheck cpu_baseline ("port") and
 * checked against the scalar oracle (oracle/ref.py) in tests.  Status codes are
 * include/prysm_hip.h's PZ_ATT_* (PZ_ERANGE / PZ_EINDEX where Go panics). */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t slot, justified_slot, shard_id, n_oblique, block_slot;
  uint8_t* bitfield; size_t bitfield_len;
} att_rec;

typedef struct { att_rec** a; size_t n; } att_set;

void* oracle_att_build(const uint64_t* slot, const uint64_t* js, const uint64_t* shard, const uint64_t* nob,
                       const uint8_t* bits, const uint64_t* boffs, const uint64_t* bslot, size_t n) {
  att_set* s = calloc(1, sizeof *s);
  s->n = n;
  s->a = calloc(n ? n : 1, sizeof *s->a);
  for (size_t i = 0; i < n; ++i) {
    att_rec* r = calloc(1, sizeof *r);
    r->slot = slot[i];
    r->justified_slot = js[i];
    r->shard_id = shard[i];
    r->n_oblique = nob[i];
    r->block_slot = bslot[i];
    r->bitfield_len = boffs[i + 1] - boffs[i];
    r->bitfield = malloc(r->bitfield_len ? r->bitfield_len : 1);
    memcpy(r->bitfield, bits + boffs[i], r->bitfield_len);
    s->a[i] = r;
  }
  return s;
}

void oracle_att_free(void* h) {
  att_set* s = h;
  for (size_t i = 0; i < s->n; ++i) {
    free(s->a[i]->bitfield);
    free(s->a[i]);
  }
  free(s->a);
  free(s);
}

/* Committee table: array a has entries arr_offs[a]..arr_offs[a+1] of (shard, committee id);
 * committee c has coffs[c+1]-coffs[c] members. */
void oracle_att_check(void* h, uint64_t ljs, uint64_t lsr, uint64_t n_recent, uint64_t narr, const uint64_t* arr_offs,
                      const uint64_t* arr_shard, const uint32_t* arr_comm, const uint64_t* coffs, int32_t* status) {
  const att_set* s = h;
  for (size_t i = 0; i < s->n; ++i) {
    const att_rec* a = s->a[i];
    int32_t st = 0;
    if ((int64_t)a->slot > (int64_t)a->block_slot) {
      st = 2;
    } else if ((int64_t)a->slot < (int64_t)a->block_slot - 64) {
      st = 3;
    } else if (a->justified_slot != ljs) {
      st = 4;
    } else {
      const uint64_t start = a->block_slot - a->slot, end = a->block_slot - a->slot - a->n_oblique + 64;
      const uint64_t idx = a->slot - lsr;
      if (start > end || end > n_recent) {
        st = -7;
      } else if (idx >= narr) {
        st = -2;
      } else {
        int64_t c = -1;
        for (uint64_t e = arr_offs[idx]; e < arr_offs[idx + 1]; ++e)
          if (arr_shard[e] == a->shard_id) { c = arr_comm[e]; break; }
        if (c < 0) {
          st = 5;
        } else {
          const uint64_t k = coffs[c + 1] - coffs[c];
          if ((k + 7) / 8 != a->bitfield_len) st = 6;
          else if (k % 8 && (a->bitfield[a->bitfield_len - 1] & (0xFFu >> (k % 8)))) st = 7;
        }
      }
    }
    status[i] = st;
  }
}
