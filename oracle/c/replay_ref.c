/* ORACLE (test infrastructure only) — C restatement of the reference's block pipeline, the
 * one-core CPU baseline of the sync-replay leg (BASELINE configs[4]) and a checker of the
 * GPU engine over whole chains.
 *
 * It follows oracle/replay.py (itself pinned by tests/golden/replay_n1024.json) and the Go it
 * cites, keeping the reference's data layout and algorithms rather than the GPU engine's:
 *   - blocks arrive serialized and are decoded into heap records (sync/service.go:147-164);
 *   - ChainService.blockProcessing (blockchain/service.go:238-363) and updateHead (:170-227,
 *     minus its DB writes, logging and the fork-choice shuffle whose result is only logged);
 *   - Block.Hash / Attestation.Hash re-marshal the decoded message (types/block.go:67-77,
 *     attestation.go:49-59); Attestation.Key (attestation.go:61-77);
 *   - processAttestation (core.go:240-297) with getSignedParentHashes (:348-360), which
 *     rebuilds the BytesToHash view of RecentBlockHashes on every call (state.go:189-195);
 *   - calculateBlockVoteCache (core.go:300-345) with Go's linear scan of VoterIndices for
 *     duplicates (O(k^2) per hash) over a map keyed by the 32-byte hash;
 *   - stateRecalc (core.go:398-497): justification over 64 slots, processCrosslinks in order
 *     (:502-558), CalculateRewards over []*ValidatorRecord (casper/incentives.go:14-32), the
 *     next-cycle total (:459-464), the new states sharing the validator and crosslink slices;
 *   - state roots: proto3 Marshal of ActiveState / CrystallizedState + BLAKE2b (state.go).
 * Go panics return ORACLE_PANIC.  uint64 arithmetic wraps like Go's. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void oracle_blake2b512(const uint8_t* msg, uint64_t len, uint8_t out[64]);
int oracle_shuffle_indices(const uint8_t seed[32], uint32_t* list, uint64_t n);

#define ORACLE_PANIC (-2)
#define ORACLE_EINVAL (-6)
#define CYCLE 64
#define SHARDS 1024
#define DEF_BAL 32ull
#define DEF_END 9999999999999999999ull
#define MIN_COMM 128

/* ---- arena (the replay's objects live until oracle_replay_free, like Go's GC'd heap) ---- */
typedef struct arena_blk { struct arena_blk* next; size_t used, cap; } arena_blk;
typedef struct { arena_blk* head; } arena;
static void* aalloc(arena* a, size_t n) {
  n = (n + 15) & ~(size_t)15;
  if (!a->head || a->head->used + n > a->head->cap) {
    size_t cap = n > (1u << 20) ? n : (1u << 20);
    arena_blk* b = (arena_blk*)malloc(sizeof(arena_blk) + cap);
    b->next = a->head; b->used = 0; b->cap = cap; a->head = b;
  }
  void* p = (char*)(a->head + 1) + a->head->used;
  a->head->used += n;
  return p;
}
static void afree(arena* a) {
  while (a->head) { arena_blk* n = a->head->next; free(a->head); a->head = n; }
}

typedef struct { const uint8_t* p; uint64_t n; } bytes_t;

typedef struct {
  uint64_t slot, shard_id, justified_slot;
  bytes_t jbh, sbh, bitfield;
  bytes_t* oblique; uint64_t n_oblique;
  uint64_t* sig; uint64_t n_sig;
} att_rec;

typedef struct {
  bytes_t parent_hash, randao, pow, ash, csh;
  uint64_t slot;
  int has_ts; int64_t ts_sec; int32_t ts_nanos;
  att_rec** atts; uint64_t natt;
} block_rec;

typedef struct { uint64_t balance, start_dynasty, end_dynasty; } validator_rec;  /* genesis fields */
typedef struct { uint64_t shard_id; uint32_t* committee; uint64_t n; } shard_committee;
typedef struct { shard_committee** arr; uint64_t n; } sc_array;
typedef struct { uint64_t dynasty, slot; bytes_t blockhash; } crosslink_rec;

typedef struct {
  uint64_t last_state_recalc, justified_streak, last_justified_slot, last_finalized_slot, current_dynasty,
      crosslinking_start_shard, total_deposits, dynasty_seed_last_reset;
  bytes_t dynasty_seed;
  crosslink_rec** records; uint64_t nrec;    /* shared between old and new states, like Go */
  validator_rec** validators; uint64_t nval;  /* shared */
  sc_array** sacfs; uint64_t nsacfs;          /* shared */
} cstate_t;

/* ---- the block vote cache: map[[32]byte]*VoteCache (types/state.go:28-31) ---- */
typedef struct {
  uint8_t key[32]; int used; uint32_t* voters; uint64_t nv, capv; uint64_t total;
  uint64_t* seen;  /* checker mode only: voter bitmap (same set as the VoterIndices scan) */
} vc_entry;
typedef struct { vc_entry* tab; uint64_t cap, count; } vote_cache;

static uint64_t vc_slot(const uint8_t k[32], uint64_t cap) {
  uint64_t h; memcpy(&h, k, 8); h ^= h >> 29; h *= 0x9E3779B97F4A7C15ull;
  return h & (cap - 1);
}
static vc_entry* vc_find(vote_cache* c, const uint8_t k[32]) {
  if (!c->cap) return NULL;
  for (uint64_t i = vc_slot(k, c->cap);; i = (i + 1) & (c->cap - 1)) {
    if (!c->tab[i].used) return NULL;
    if (!memcmp(c->tab[i].key, k, 32)) return &c->tab[i];
  }
}
static vc_entry* vc_insert(vote_cache* c, const uint8_t k[32]) {
  if ((c->count + 1) * 2 > c->cap) {
    uint64_t ncap = c->cap ? c->cap * 2 : 256;
    vc_entry* nt = (vc_entry*)calloc(ncap, sizeof(vc_entry));
    for (uint64_t i = 0; i < c->cap; ++i)
      if (c->tab[i].used) {
        uint64_t j = vc_slot(c->tab[i].key, ncap);
        while (nt[j].used) j = (j + 1) & (ncap - 1);
        nt[j] = c->tab[i];
      }
    free(c->tab); c->tab = nt; c->cap = ncap;
  }
  uint64_t i = vc_slot(k, c->cap);
  while (c->tab[i].used) i = (i + 1) & (c->cap - 1);
  vc_entry* e = &c->tab[i];
  memset(e, 0, sizeof *e);
  memcpy(e->key, k, 32);
  e->used = 1;
  c->count++;
  return e;
}
static void vc_free(vote_cache* c) {
  for (uint64_t i = 0; i < c->cap; ++i) { free(c->tab[i].voters); free(c->tab[i].seen); }
  free(c->tab); c->tab = NULL; c->cap = c->count = 0;
}

typedef struct {
  att_rec** pending; uint64_t npending, cap_pending;
  bytes_t* recent; uint64_t nrecent;          /* RecentBlockHashes as stored (raw bytes) */
  vote_cache* cache;                          /* shared map; NULL = nil map */
} astate_t;

typedef struct { uint8_t h[32]; } hash32;

typedef struct {
  arena ar;
  cstate_t* C;
  astate_t* A;
  vote_cache cache;                  /* the one map every ActiveState shares */
  int has_cand;
  uint64_t cand_slot;
  astate_t* candA; cstate_t* candC;
  hash32* saved; uint64_t nsaved, capsaved;  /* hasBlock: block hashes saved (sorted set) */
  int bitmap_dedup;  /* 0: Go's linear scan of VoterIndices (the baseline); 1: a bitmap per
                        hash with the same answer (the checker over long chains) */
} chain_t;

/* ---- proto3 encoding (golang/protobuf v1.1 semantics; messages.pb.go struct tags) ---- */
typedef struct { uint8_t* p; uint64_t n, cap; } buf_t;
static void bput(buf_t* b, const void* s, uint64_t n) {
  if (b->n + n > b->cap) { b->cap = (b->n + n) * 2 + 64; b->p = (uint8_t*)realloc(b->p, b->cap); }
  memcpy(b->p + b->n, s, n); b->n += n;
}
static void bvar(buf_t* b, uint64_t x) {
  uint8_t t[10]; int k = 0;
  while (x >= 0x80) { t[k++] = (uint8_t)(x | 0x80); x >>= 7; }
  t[k++] = (uint8_t)x;
  bput(b, t, k);
}
static uint64_t svar(uint64_t x) { uint64_t n = 1; while (x >= 0x80) { x >>= 7; ++n; } return n; }
static void f_u64(buf_t* b, int f, uint64_t v) { if (v) { bvar(b, (uint64_t)f << 3); bvar(b, v); } }
static void f_bytes(buf_t* b, int f, bytes_t v) { if (v.n) { bvar(b, ((uint64_t)f << 3) | 2); bvar(b, v.n); bput(b, v.p, v.n); } }
static void f_bytes_rep(buf_t* b, int f, bytes_t v) { bvar(b, ((uint64_t)f << 3) | 2); bvar(b, v.n); bput(b, v.p, v.n); }

static void enc_att(buf_t* b, const att_rec* a) {
  f_u64(b, 1, a->slot);
  f_u64(b, 2, a->shard_id);
  f_u64(b, 3, a->justified_slot);
  f_bytes(b, 4, a->jbh);
  f_bytes(b, 5, a->sbh);
  f_bytes(b, 6, a->bitfield);
  for (uint64_t i = 0; i < a->n_oblique; ++i) f_bytes_rep(b, 7, a->oblique[i]);
  if (a->n_sig) {  /* packed */
    uint64_t len = 0;
    for (uint64_t i = 0; i < a->n_sig; ++i) len += svar(a->sig[i]);
    bvar(b, (8 << 3) | 2); bvar(b, len);
    for (uint64_t i = 0; i < a->n_sig; ++i) bvar(b, a->sig[i]);
  }
}
static void enc_sub(buf_t* b, int f, void (*enc)(buf_t*, const void*), const void* m) {
  buf_t t = {0, 0, 0};
  enc(&t, m);
  bvar(b, ((uint64_t)f << 3) | 2); bvar(b, t.n); if (t.n) bput(b, t.p, t.n);
  free(t.p);
}
static void enc_att_v(buf_t* b, const void* m) { enc_att(b, (const att_rec*)m); }
static void enc_block(buf_t* b, const block_rec* k) {
  f_bytes(b, 1, k->parent_hash);
  f_u64(b, 2, k->slot);
  f_bytes(b, 3, k->randao);
  f_bytes(b, 4, k->pow);
  f_bytes(b, 5, k->ash);
  f_bytes(b, 6, k->csh);
  if (k->has_ts) {
    buf_t t = {0, 0, 0};
    f_u64(&t, 1, (uint64_t)k->ts_sec);
    f_u64(&t, 2, (uint64_t)(int64_t)k->ts_nanos);  /* int32 varint: sign-extended */
    bvar(b, (7 << 3) | 2); bvar(b, t.n); if (t.n) bput(b, t.p, t.n);
    free(t.p);
  }
  for (uint64_t i = 0; i < k->natt; ++i) enc_sub(b, 8, enc_att_v, k->atts[i]);
}
static void enc_validator(buf_t* b, const void* m) {
  const validator_rec* v = (const validator_rec*)m;
  f_u64(b, 5, v->balance);
  f_u64(b, 6, v->start_dynasty);
  f_u64(b, 7, v->end_dynasty);
}
static void enc_crosslink(buf_t* b, const void* m) {
  const crosslink_rec* r = (const crosslink_rec*)m;
  f_u64(b, 1, r->dynasty);
  f_bytes(b, 2, r->blockhash);
  f_u64(b, 3, r->slot);
}
static void enc_sc(buf_t* b, const void* m) {
  const shard_committee* s = (const shard_committee*)m;
  f_u64(b, 1, s->shard_id);
  if (s->n) {
    uint64_t len = 0;
    for (uint64_t i = 0; i < s->n; ++i) len += svar(s->committee[i]);
    bvar(b, (2 << 3) | 2); bvar(b, len);
    for (uint64_t i = 0; i < s->n; ++i) bvar(b, s->committee[i]);
  }
}
static void enc_sca(buf_t* b, const void* m) {
  const sc_array* a = (const sc_array*)m;
  for (uint64_t i = 0; i < a->n; ++i) enc_sub(b, 1, enc_sc, a->arr[i]);
}
static void enc_cstate(buf_t* b, const cstate_t* c) {
  f_u64(b, 1, c->last_state_recalc);
  f_u64(b, 2, c->justified_streak);
  f_u64(b, 3, c->last_justified_slot);
  f_u64(b, 4, c->last_finalized_slot);
  f_u64(b, 5, c->current_dynasty);
  f_u64(b, 6, c->crosslinking_start_shard);
  f_u64(b, 7, c->total_deposits);
  f_bytes(b, 8, c->dynasty_seed);
  f_u64(b, 9, c->dynasty_seed_last_reset);
  for (uint64_t i = 0; i < c->nrec; ++i) enc_sub(b, 10, enc_crosslink, c->records[i]);
  for (uint64_t i = 0; i < c->nval; ++i) enc_sub(b, 11, enc_validator, c->validators[i]);
  for (uint64_t i = 0; i < c->nsacfs; ++i) enc_sub(b, 12, enc_sca, c->sacfs[i]);
}
static void enc_astate(buf_t* b, const astate_t* a) {
  for (uint64_t i = 0; i < a->npending; ++i) enc_sub(b, 1, enc_att_v, a->pending[i]);
  for (uint64_t i = 0; i < a->nrecent; ++i) f_bytes_rep(b, 2, a->recent[i]);
}
static void hash32_of(const buf_t* b, uint8_t out[32]) {
  uint8_t d[64];
  oracle_blake2b512(b->p, b->n, d);
  memcpy(out, d, 32);
}

/* ---- proto3 decoding of the incoming BeaconBlock ---- */
typedef struct { const uint8_t* p; const uint8_t* e; int bad; } rd_t;
static uint64_t rvar(rd_t* r) {
  uint64_t x = 0; int s = 0;
  while (r->p < r->e && s < 64) { uint8_t c = *r->p++; x |= (uint64_t)(c & 0x7F) << s; if (!(c & 0x80)) return x; s += 7; }
  r->bad = 1; return 0;
}
static bytes_t rbytes(rd_t* r) {
  bytes_t v = {0, 0};
  uint64_t n = rvar(r);
  if (r->bad || (uint64_t)(r->e - r->p) < n) { r->bad = 1; return v; }
  v.p = r->p; v.n = n; r->p += n;
  return v;
}
static void rskip(rd_t* r, int wt) {
  if (wt == 0) rvar(r);
  else if (wt == 2) rbytes(r);
  else if (wt == 1) { if (r->e - r->p < 8) r->bad = 1; else r->p += 8; }
  else if (wt == 5) { if (r->e - r->p < 4) r->bad = 1; else r->p += 4; }
  else r->bad = 1;
}
static att_rec* dec_att(arena* ar, const uint8_t* p, uint64_t n, int* bad) {
  att_rec* a = (att_rec*)aalloc(ar, sizeof *a);
  memset(a, 0, sizeof *a);
  rd_t r = {p, p + n, 0};
  /* two passes: count the repeated fields, then fill */
  uint64_t no = 0, ns = 0;
  while (r.p < r.e && !r.bad) {
    uint64_t k = rvar(&r); int f = (int)(k >> 3), wt = (int)(k & 7);
    if (f == 7 && wt == 2) { rbytes(&r); ++no; }
    else if (f == 8 && wt == 2) { bytes_t v = rbytes(&r); rd_t q = {v.p, v.p + v.n, 0}; while (q.p < q.e && !q.bad) { rvar(&q); ++ns; } }
    else if (f == 8 && wt == 0) { rvar(&r); ++ns; }
    else rskip(&r, wt);
  }
  a->oblique = (bytes_t*)aalloc(ar, (no + 1) * sizeof(bytes_t));
  a->sig = (uint64_t*)aalloc(ar, (ns + 1) * sizeof(uint64_t));
  r.p = p;
  while (r.p < r.e && !r.bad) {
    uint64_t k = rvar(&r); int f = (int)(k >> 3), wt = (int)(k & 7);
    if (f == 1 && wt == 0) a->slot = rvar(&r);
    else if (f == 2 && wt == 0) a->shard_id = rvar(&r);
    else if (f == 3 && wt == 0) a->justified_slot = rvar(&r);
    else if (f == 4 && wt == 2) a->jbh = rbytes(&r);
    else if (f == 5 && wt == 2) a->sbh = rbytes(&r);
    else if (f == 6 && wt == 2) a->bitfield = rbytes(&r);
    else if (f == 7 && wt == 2) a->oblique[a->n_oblique++] = rbytes(&r);
    else if (f == 8 && wt == 2) { bytes_t v = rbytes(&r); rd_t q = {v.p, v.p + v.n, 0}; while (q.p < q.e && !q.bad) a->sig[a->n_sig++] = rvar(&q); }
    else if (f == 8 && wt == 0) a->sig[a->n_sig++] = rvar(&r);
    else rskip(&r, wt);
  }
  *bad |= r.bad;
  return a;
}
static block_rec* dec_block(arena* ar, const uint8_t* p, uint64_t n, int* bad) {
  block_rec* k = (block_rec*)aalloc(ar, sizeof *k);
  memset(k, 0, sizeof *k);
  rd_t r = {p, p + n, 0};
  uint64_t na = 0;
  while (r.p < r.e && !r.bad) {
    uint64_t key = rvar(&r); int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 8 && wt == 2) { rbytes(&r); ++na; } else rskip(&r, wt);
  }
  k->atts = (att_rec**)aalloc(ar, (na + 1) * sizeof(att_rec*));
  r.p = p;
  while (r.p < r.e && !r.bad) {
    uint64_t key = rvar(&r); int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 1 && wt == 2) k->parent_hash = rbytes(&r);
    else if (f == 2 && wt == 0) k->slot = rvar(&r);
    else if (f == 3 && wt == 2) k->randao = rbytes(&r);
    else if (f == 4 && wt == 2) k->pow = rbytes(&r);
    else if (f == 5 && wt == 2) k->ash = rbytes(&r);
    else if (f == 6 && wt == 2) k->csh = rbytes(&r);
    else if (f == 7 && wt == 2) {
      bytes_t v = rbytes(&r); rd_t q = {v.p, v.p + v.n, 0};
      k->has_ts = 1;
      while (q.p < q.e && !q.bad) {
        uint64_t kk = rvar(&q); int ff = (int)(kk >> 3), ww = (int)(kk & 7);
        if (ff == 1 && ww == 0) k->ts_sec = (int64_t)rvar(&q);
        else if (ff == 2 && ww == 0) k->ts_nanos = (int32_t)rvar(&q);
        else rskip(&q, ww);
      }
      r.bad |= q.bad;
    } else if (f == 8 && wt == 2) { bytes_t v = rbytes(&r); k->atts[k->natt++] = dec_att(ar, v.p, v.n, &r.bad); }
    else rskip(&r, wt);
  }
  *bad |= r.bad;
  return k;
}

/* ---- helpers (go-ethereum common, utils/checkbit.go) ---- */
static void bytes_to_hash(bytes_t b, uint8_t out[32]) {  /* common.BytesToHash: right-align */
  memset(out, 0, 32);
  if (b.n >= 32) memcpy(out, b.p + b.n - 32, 32);
  else memcpy(out + 32 - b.n, b.p, b.n);
}
static int check_bit(bytes_t bf, uint64_t i, int* panic) {
  if ((i >> 3) >= bf.n) { *panic = 1; return 0; }
  return (bf.p[i >> 3] >> (7 - (i & 7))) & 1;
}
static uint64_t put_uvarint(uint8_t* b, uint64_t x) {
  uint64_t i = 0;
  while (x >= 0x80) { b[i++] = (uint8_t)(x | 0x80); x >>= 7; }
  b[i] = (uint8_t)x;
  return i + 1;
}

/* ---- casper / sharding (genesis committees) ---- */
static sc_array** split_by_slot_shard(arena* ar, const uint32_t* sh, uint64_t n, uint64_t start_shard) {
  uint64_t cps = 1, spc = 1;
  if (n >= (uint64_t)CYCLE * MIN_COMM) cps = n / (CYCLE * MIN_COMM * 2) + 1;
  else while (n * spc < (uint64_t)MIN_COMM * CYCLE && spc < CYCLE) spc *= 2;
  sc_array** out = (sc_array**)aalloc(ar, CYCLE * sizeof(sc_array*));
  for (uint64_t i = 0; i < CYCLE; ++i) {
    const uint64_t s0 = n * i / CYCLE, s1 = n * (i + 1) / CYCLE, len = s1 - s0;
    sc_array* a = (sc_array*)aalloc(ar, sizeof *a);
    a->n = cps;
    a->arr = (shard_committee**)aalloc(ar, cps * sizeof(shard_committee*));
    const uint64_t ss = start_shard + i * cps / spc;
    for (uint64_t j = 0; j < cps; ++j) {
      const uint64_t c0 = s0 + len * j / cps, c1 = s0 + len * (j + 1) / cps;
      shard_committee* sc = (shard_committee*)aalloc(ar, sizeof *sc);
      sc->shard_id = (ss + j) % SHARDS;
      sc->n = c1 - c0;
      sc->committee = (uint32_t*)aalloc(ar, (sc->n + 1) * 4);
      memcpy(sc->committee, sh + c0, sc->n * 4);
      a->arr[j] = sc;
    }
    out[i] = a;
  }
  return out;
}

static chain_t* genesis(uint64_t nval) {
  chain_t* g = (chain_t*)calloc(1, sizeof *g);
  arena* ar = &g->ar;
  cstate_t* c = (cstate_t*)aalloc(ar, sizeof *c);
  memset(c, 0, sizeof *c);
  c->nval = nval;
  c->validators = (validator_rec**)aalloc(ar, (nval + 1) * sizeof(validator_rec*));
  for (uint64_t i = 0; i < nval; ++i) {
    validator_rec* v = (validator_rec*)malloc(sizeof *v);  /* one heap record each, like Go */
    v->balance = DEF_BAL; v->start_dynasty = 0; v->end_dynasty = DEF_END;
    c->validators[i] = v;
  }
  uint32_t* idx = (uint32_t*)malloc((nval + 1) * 4);
  uint64_t na = 0;
  for (uint64_t i = 0; i < nval; ++i)
    if (c->validators[i]->start_dynasty <= 1 && 1 < c->validators[i]->end_dynasty) idx[na++] = (uint32_t)i;
  uint8_t seed[32] = {0};  /* common.BytesToHash([]byte{}) (types/state.go:70) */
  oracle_shuffle_indices(seed, idx, na);
  sc_array** com = split_by_slot_shard(ar, idx, na, 0);
  free(idx);
  c->nsacfs = 4 * CYCLE;  /* committees appended twice, then the loop over append(c, c...) */
  c->sacfs = (sc_array**)aalloc(ar, c->nsacfs * sizeof(sc_array*));
  for (uint64_t i = 0; i < c->nsacfs; ++i) c->sacfs[i] = com[i % CYCLE];
  c->nrec = SHARDS;
  c->records = (crosslink_rec**)aalloc(ar, SHARDS * sizeof(crosslink_rec*));
  for (uint64_t i = 0; i < SHARDS; ++i) {
    crosslink_rec* r = (crosslink_rec*)aalloc(ar, sizeof *r);
    memset(r, 0, sizeof *r);
    c->records[i] = r;
  }
  c->current_dynasty = 1;
  c->total_deposits = nval * DEF_BAL;
  astate_t* a = (astate_t*)aalloc(ar, sizeof *a);
  memset(a, 0, sizeof *a);
  a->nrecent = 2 * CYCLE;
  a->recent = (bytes_t*)aalloc(ar, a->nrecent * sizeof(bytes_t));
  memset(a->recent, 0, a->nrecent * sizeof(bytes_t));
  a->cache = &g->cache;
  g->C = c;
  g->A = a;
  return g;
}

/* ---- the hasBlock set ---- */
static int saved_has(chain_t* g, const uint8_t h[32]) {
  uint64_t lo = 0, hi = g->nsaved;
  while (lo < hi) { uint64_t m = (lo + hi) / 2; int c = memcmp(g->saved[m].h, h, 32); if (!c) return 1; if (c < 0) lo = m + 1; else hi = m; }
  return 0;
}
static void saved_add(chain_t* g, const uint8_t h[32]) {
  if (saved_has(g, h)) return;
  if (g->nsaved == g->capsaved) { g->capsaved = g->capsaved ? 2 * g->capsaved : 1024; g->saved = (hash32*)realloc(g->saved, g->capsaved * sizeof(hash32)); }
  uint64_t lo = 0, hi = g->nsaved;
  while (lo < hi) { uint64_t m = (lo + hi) / 2; if (memcmp(g->saved[m].h, h, 32) < 0) lo = m + 1; else hi = m; }
  memmove(g->saved + lo + 1, g->saved + lo, (g->nsaved - lo) * sizeof(hash32));
  memcpy(g->saved[lo].h, h, 32);
  g->nsaved++;
}

/* ---- blockchain/core.go ---- */
/* RecentBlockHashes() (types/state.go:189-195): a fresh BytesToHash copy on every call */
static hash32* recent_hashes(const astate_t* a) {
  hash32* r = (hash32*)malloc((a->nrecent + 1) * sizeof(hash32));
  for (uint64_t i = 0; i < a->nrecent; ++i) bytes_to_hash(a->recent[i], r[i].h);
  return r;
}

/* getAttesterIndices (core.go:363-374): 0 ok, 1 Go error (not found), ORACLE_PANIC */
static int attester_indices(const cstate_t* c, const att_rec* a, const shard_committee** out) {
  const uint64_t i = a->slot - c->last_state_recalc;
  if (i >= c->nsacfs) return ORACLE_PANIC;
  const sc_array* arr = c->sacfs[i];
  for (uint64_t k = 0; k < arr->n; ++k)
    if (arr->arr[k]->shard_id == a->shard_id) { *out = arr->arr[k]; return 0; }
  return 1;
}

/* getSignedParentHashes (core.go:348-360): malloc'd list of *n hashes, or NULL on a panic */
static hash32* signed_parents(const astate_t* A, uint64_t block_slot, const att_rec* a, uint64_t* n) {
  const uint64_t start = block_slot - a->slot;
  const uint64_t end = block_slot - a->slot - a->n_oblique + CYCLE;
  if (start > end || end > A->nrecent) return NULL;  /* slice bounds out of range */
  hash32* rec = recent_hashes(A);
  *n = end - start + a->n_oblique;
  hash32* out = (hash32*)malloc((*n + 1) * sizeof(hash32));
  memcpy(out, rec + start, (end - start) * sizeof(hash32));
  for (uint64_t k = 0; k < a->n_oblique; ++k) bytes_to_hash(a->oblique[k], out[end - start + k].h);
  free(rec);
  return out;
}

/* processAttestation (core.go:240-297): 0 processed, 1 rejected (Go error), ORACLE_PANIC */
static int process_attestation(chain_t* g, uint64_t block_slot, const att_rec* a, uint8_t msg_digest[64],
                               uint32_t* msg_len) {
  const cstate_t* c = g->C;
  if ((int64_t)a->slot > (int64_t)block_slot) return 1;              /* int(...) comparisons */
  if ((int64_t)a->slot < (int64_t)block_slot - CYCLE) return 1;
  if (a->justified_slot != c->last_justified_slot) return 1;
  uint64_t np = 0;
  hash32* parents = signed_parents(g->A, block_slot, a, &np);
  if (!parents) return ORACLE_PANIC;
  const shard_committee* sc;
  int rc = attester_indices(c, a, &sc);
  if (rc) { free(parents); return rc; }
  /* validateAttesterBitfields (core.go:377-394) */
  if ((sc->n + 7) / 8 != a->bitfield.n) { free(parents); return 1; }
  if (sc->n % 8) {
    int panic = 0;
    for (uint64_t i = 0; i < 8 - sc->n % 8; ++i)
      if (check_bit(a->bitfield, sc->n + i, &panic)) { free(parents); return 1; }
    if (panic) { free(parents); return ORACLE_PANIC; }
  }
  /* the message (core.go:277-290): both varints at offset 0 */
  const uint64_t len = 10 + 33 * np + a->sbh.n;
  uint8_t* m = (uint8_t*)calloc(len + 1, 1);
  put_uvarint(m, a->slot % CYCLE);
  for (uint64_t k = 0; k < np; ++k) { memcpy(m + 10 + 33 * k, parents[k].h, 32); m[10 + 33 * k + 32] = ' '; }
  put_uvarint(m, a->shard_id);
  memcpy(m + 10 + 33 * np, a->sbh.p, a->sbh.n);
  oracle_blake2b512(m, len, msg_digest);
  *msg_len = (uint32_t)len;
  free(m);
  free(parents);
  return 0;
}

/* calculateBlockVoteCache (core.go:300-345): 0 ok, 1 Go error, ORACLE_PANIC */
static int vote_cache_update(chain_t* g, uint64_t block_slot, const att_rec* a) {
  vote_cache* vc = g->A->cache;
  uint64_t np = 0;
  hash32* parents = signed_parents(g->A, block_slot, a, &np);
  if (!parents) return ORACLE_PANIC;
  const shard_committee* sc;
  int rc = attester_indices(g->C, a, &sc);
  if (rc) { free(parents); return rc; }
  if (!vc) { free(parents); return ORACLE_PANIC; }  /* assignment to entry in nil map */
  for (uint64_t k = 0; k < np; ++k) {
    int skip = 0;
    for (uint64_t o = 0; o < a->n_oblique; ++o)
      if (a->oblique[o].n == 32 && !memcmp(parents[k].h, a->oblique[o].p, 32)) skip = 1;
    if (skip) continue;
    vc_entry* e = vc_find(vc, parents[k].h);
    if (!e) e = vc_insert(vc, parents[k].h);
    for (uint64_t i = 0; i < sc->n; ++i) {
      int panic = 0;
      if (!check_bit(a->bitfield, i, &panic)) {
        if (panic) { free(parents); return ORACLE_PANIC; }
        continue;
      }
      const uint32_t v = sc->committee[i];
      int existing = 0;
      if (g->bitmap_dedup && v < g->C->nval) {
        if (!e->seen) e->seen = (uint64_t*)calloc((g->C->nval + 63) / 64, 8);
        existing = (int)((e->seen[v >> 6] >> (v & 63)) & 1);
        e->seen[v >> 6] |= 1ull << (v & 63);
      } else {
        for (uint64_t j = 0; j < e->nv; ++j)  /* Go's linear scan of VoterIndices */
          if (e->voters[j] == v) existing = 1;
      }
      if (!existing) {
        if (v >= g->C->nval) { free(parents); return ORACLE_PANIC; }
        if (e->nv == e->capv) { e->capv = e->capv ? 2 * e->capv : 16; e->voters = (uint32_t*)realloc(e->voters, e->capv * 4); }
        e->voters[e->nv++] = v;
        e->total += g->C->validators[v]->balance;
      }
    }
  }
  free(parents);
  return 0;
}

/* stateRecalc (core.go:398-497) -> the new states (in the arena); ORACLE_PANIC on a panic */
static int state_recalc(chain_t* g, cstate_t* c, astate_t* a, uint64_t block_slot, cstate_t** nc_out,
                        astate_t** na_out) {
  arena* ar = &g->ar;
  uint64_t streak = c->justified_streak, justified = c->last_justified_slot, finalized = c->last_finalized_slot;
  const uint64_t lsr = c->last_state_recalc;
  hash32* recent = recent_hashes(a);
  for (uint64_t i = 0; i < CYCLE; ++i) {
    const uint64_t slot = lsr - CYCLE + i;
    vc_entry* e = a->cache ? vc_find(a->cache, recent[i].h) : NULL;
    const uint64_t bal = e ? e->total : 0;
    if (3 * bal >= 2 * c->total_deposits) {
      if (slot > justified) justified = slot;
      streak++;
    } else {
      streak = 0;
    }
    if (streak >= CYCLE + 1 && slot - CYCLE > finalized) finalized = slot - CYCLE;
  }
  /* processCrosslinks (core.go:502-558), in order, records replaced in place */
  for (uint64_t k = 0; k < a->npending; ++k) {
    const att_rec* at = a->pending[k];
    const shard_committee* sc;
    int rc = attester_indices(c, at, &sc);
    if (rc) { free(recent); return rc == 1 ? 1 : ORACLE_PANIC; }
    uint64_t total = 0, vote = 0;
    for (uint64_t i = 0; i < sc->n; ++i) {
      if (sc->committee[i] >= c->nval) { free(recent); return ORACLE_PANIC; }
      total += c->validators[sc->committee[i]]->balance;
    }
    for (uint64_t i = 0; i < sc->n; ++i) {
      int panic = 0;
      if (check_bit(at->bitfield, i, &panic)) vote += c->validators[sc->committee[i]]->balance;
      if (panic) { free(recent); return ORACLE_PANIC; }
    }
    if (3 * vote >= 2 * total) {
      if (at->shard_id >= c->nrec) { free(recent); return ORACLE_PANIC; }
      if (c->current_dynasty > c->records[at->shard_id]->dynasty) {
        crosslink_rec* r = (crosslink_rec*)aalloc(ar, sizeof *r);
        r->dynasty = c->current_dynasty; r->blockhash = at->sbh; r->slot = block_slot;
        c->records[at->shard_id] = r;
      }
    }
  }
  /* the pending attestations that survive (core.go:445-450) */
  astate_t* na = (astate_t*)aalloc(ar, sizeof *na);
  memset(na, 0, sizeof *na);
  na->pending = (att_rec**)aalloc(ar, (a->npending + 1) * sizeof(att_rec*));
  for (uint64_t k = 0; k < a->npending; ++k)
    if (a->pending[k]->slot > lsr) na->pending[na->npending++] = a->pending[k];
  na->cap_pending = a->npending + 1;
  /* CalculateRewards (casper/incentives.go:14-32): rank-targeted */
  uint64_t pop = 0;
  for (uint64_t k = 0; k < a->npending; ++k)
    for (uint64_t i = 0; i < a->pending[k]->bitfield.n; ++i) pop += (uint64_t)__builtin_popcount(a->pending[k]->bitfield.p[i]);
  const uint64_t dep = pop * DEF_BAL;
  const uint64_t d = c->current_dynasty;
  if (3 * dep >= 2 * c->total_deposits) {
    uint64_t rank = 0;
    for (uint64_t i = 0; i < c->nval; ++i) {
      const validator_rec* v = c->validators[i];
      if (!(v->start_dynasty <= d && d < v->end_dynasty)) continue;
      if (!a->npending) { free(recent); return ORACLE_PANIC; }
      int panic = 0;
      const int voted = check_bit(a->pending[a->npending - 1]->bitfield, i, &panic);
      if (panic) { free(recent); return ORACLE_PANIC; }
      validator_rec* t = c->validators[rank++];
      t->balance = voted ? t->balance + 1 : t->balance - 1;
    }
  }
  uint64_t nxt = 0;
  for (uint64_t i = 0; i < c->nval; ++i) {
    const validator_rec* v = c->validators[i];
    if (v->start_dynasty <= d && d < v->end_dynasty) nxt += v->balance;
  }
  cstate_t* nc = (cstate_t*)aalloc(ar, sizeof *nc);
  memset(nc, 0, sizeof *nc);
  nc->validators = c->validators; nc->nval = c->nval;       /* shared slices, like Go */
  nc->last_state_recalc = lsr + CYCLE;
  nc->sacfs = c->sacfs; nc->nsacfs = c->nsacfs;
  nc->last_justified_slot = justified;
  nc->justified_streak = streak;
  nc->last_finalized_slot = finalized;
  nc->crosslinking_start_shard = 0;
  nc->records = c->records; nc->nrec = c->nrec;
  nc->dynasty_seed_last_reset = c->dynasty_seed_last_reset;
  nc->total_deposits = nxt;
  /* RecentBlockHashes normalised to 32 bytes, the last 128 kept (core.go:480-488) */
  const uint64_t keep = a->nrecent > 2 * CYCLE ? 2 * CYCLE : a->nrecent;
  na->nrecent = keep;
  na->recent = (bytes_t*)aalloc(ar, (keep + 1) * sizeof(bytes_t));
  for (uint64_t i = 0; i < keep; ++i) {
    uint8_t* h = (uint8_t*)aalloc(ar, 32);
    memcpy(h, recent[a->nrecent - keep + i].h, 32);
    na->recent[i].p = h; na->recent[i].n = 32;
  }
  na->cache = a->cache;
  free(recent);
  *nc_out = nc;
  *na_out = na;
  return 0;
}

/* computeNewActiveState (core.go:223-237), in place */
static void compute_new_active_state(chain_t* g, astate_t* a, att_rec** atts, uint64_t n, const uint8_t h[32]) {
  arena* ar = &g->ar;
  if (a->npending + n > a->cap_pending) {
    uint64_t cap = (a->npending + n) * 2 + 8;
    att_rec** p = (att_rec**)aalloc(ar, cap * sizeof(att_rec*));
    memcpy(p, a->pending, a->npending * sizeof(att_rec*));
    a->pending = p; a->cap_pending = cap;
  }
  memcpy(a->pending + a->npending, atts, n * sizeof(att_rec*));
  a->npending += n;
  hash32* rec = recent_hashes(a);
  const uint64_t total = a->nrecent + 1;
  const uint64_t keep = total > 2 * CYCLE ? 2 * CYCLE : total;
  bytes_t* nr = (bytes_t*)aalloc(ar, (keep + 1) * sizeof(bytes_t));
  for (uint64_t i = 0; i < keep; ++i) {
    const uint64_t src = total - keep + i;
    uint8_t* p = (uint8_t*)aalloc(ar, 32);
    if (src < a->nrecent) memcpy(p, rec[src].h, 32); else memcpy(p, h, 32);
    nr[i].p = p; nr[i].n = 32;
  }
  a->recent = nr; a->nrecent = keep;
  free(rec);
}

/* statuses: the product's PZ_BLOCK_* / PZ_ATT_* classes (errors collapse to one code) */
enum { B_PROCESSED = 0, B_NO_PARENT = 1, B_ATTS_REJECTED = 2, B_SAVED_NOT_CANDIDATE = 3 };
enum { A_PROCESSED = 0, A_NOT_PROCESSED = 1, A_REJECTED = 2 };

/* One block through blockProcessing (service.go:238-363). */
static int process_block(chain_t* g, const block_rec* b, uint8_t bhash[32], int32_t* bstatus, int32_t* btrans,
                         uint8_t* akey, uint8_t* ahash, uint8_t* amsg, uint32_t* amsg_len, int32_t* astatus) {
  buf_t buf = {0, 0, 0};
  enc_block(&buf, b);
  hash32_of(&buf, bhash);
  *btrans = 0;
  for (uint64_t k = 0; k < b->natt; ++k) astatus[k] = A_NOT_PROCESSED;
  uint8_t ph[32] = {0};
  memcpy(ph, b->parent_hash.p, b->parent_hash.n < 32 ? b->parent_hash.n : 32);  /* copy(h[:], ...) */
  if (!saved_has(g, ph) && b->slot > 1) { *bstatus = B_NO_PARENT; free(buf.p); return 0; }
  att_rec** processed = (att_rec**)malloc((b->natt + 1) * sizeof(att_rec*));
  uint64_t nproc = 0;
  int can = 0;
  for (uint64_t k = 0; k < b->natt; ++k) {
    const att_rec* a = b->atts[k];
    int rc = process_attestation(g, b->slot, a, amsg + 64 * k, &amsg_len[k]);
    if (rc == ORACLE_PANIC) { free(processed); free(buf.p); return ORACLE_PANIC; }
    if (rc) { can = 0; astatus[k] = A_REJECTED; continue; }
    can = 1;
    astatus[k] = A_PROCESSED;
    /* Attestation.Key (attestation.go:61-77) and Hash (:49-59) */
    buf.n = 0;
    uint8_t z[10] = {0};
    bput(&buf, z, 10);
    put_uvarint(buf.p, a->slot);
    put_uvarint(buf.p, a->shard_id);
    bput(&buf, a->sbh.p, a->sbh.n);
    for (uint64_t o = 0; o < a->n_oblique; ++o) {
      uint8_t h[32] = {0};
      memcpy(h, a->oblique[o].p, a->oblique[o].n < 32 ? a->oblique[o].n : 32);
      bput(&buf, h, 32);
    }
    hash32_of(&buf, akey + 32 * k);
    buf.n = 0;
    enc_att(&buf, a);
    hash32_of(&buf, ahash + 32 * k);
    processed[nproc++] = (att_rec*)a;
  }
  free(buf.p);
  if (!can) { *bstatus = B_ATTS_REJECTED; free(processed); return 0; }
  vote_cache* vcache = NULL;
  for (uint64_t k = 0; k < b->natt; ++k) {
    int rc = vote_cache_update(g, b->slot, b->atts[k]);
    if (rc == ORACLE_PANIC) { free(processed); return ORACLE_PANIC; }
    vcache = rc ? NULL : g->A->cache;
  }
  if (g->has_cand && b->slot > g->cand_slot && b->slot > 1) {  /* updateHead */
    g->A = g->candA; g->C = g->candC; g->has_cand = 0;
  }
  saved_add(g, bhash);
  if (g->has_cand) { *bstatus = B_SAVED_NOT_CANDIDATE; free(processed); return 0; }
  astate_t* A = g->A;
  cstate_t* C = g->C;
  if (b->slot >= C->last_state_recalc + CYCLE) {
    *btrans = 1;
    cstate_t* nc; astate_t* na;
    int rc = state_recalc(g, C, A, b->slot, &nc, &na);
    if (rc) { free(processed); return ORACLE_PANIC; }
    C = nc; A = na;
  }
  A->cache = vcache;
  compute_new_active_state(g, A, processed, nproc, bhash);
  free(processed);
  g->has_cand = 1; g->cand_slot = b->slot; g->candA = A; g->candC = C;
  *bstatus = B_PROCESSED;
  return 0;
}

/* ---- the C ABI of the checker ---- */
void* oracle_replay_new(uint64_t nval, int bitmap_dedup) {
  chain_t* g = genesis(nval);
  g->bitmap_dedup = bitmap_dedup;
  return g;
}

/* Decode and process n serialized blocks (CSR).  Per block: hash, status, transition; per
 * attestation (in block order, att_cap entries): status, key, hash, 64-B message digest and
 * its length.  Returns 0, ORACLE_EINVAL (undecodable input / att_cap short) or ORACLE_PANIC
 * (*at_block = the block whose processing panicked). */
int oracle_replay_blocks(void* h, const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t* bhash,
                         int32_t* bstatus, int32_t* btrans, int32_t* astatus, uint8_t* akey, uint8_t* ahash,
                         uint8_t* amsg, uint32_t* amsg_len, uint64_t att_cap, uint64_t* at_block) {
  chain_t* g = (chain_t*)h;
  uint64_t ai = 0;
  for (uint64_t i = 0; i < n; ++i) {
    int bad = 0;
    block_rec* b = dec_block(&g->ar, data + offs[i], offs[i + 1] - offs[i], &bad);
    if (bad || ai + b->natt > att_cap) return ORACLE_EINVAL;
    int rc = process_block(g, b, bhash + 32 * i, &bstatus[i], &btrans[i], akey + 32 * ai, ahash + 32 * ai,
                           amsg + 64 * ai, amsg_len + ai, astatus + ai);
    if (rc) { if (at_block) *at_block = i; return rc; }
    ai += b->natt;
  }
  return 0;
}

/* roots: [chain active, chain crystallized, candidate active, candidate crystallized] */
void oracle_replay_roots(void* h, uint8_t out[128], int* has_cand) {
  chain_t* g = (chain_t*)h;
  buf_t b = {0, 0, 0};
  enc_astate(&b, g->A); hash32_of(&b, out); b.n = 0;
  enc_cstate(&b, g->C); hash32_of(&b, out + 32); b.n = 0;
  memset(out + 64, 0, 64);
  *has_cand = g->has_cand;
  if (g->has_cand) {
    enc_astate(&b, g->candA); hash32_of(&b, out + 64); b.n = 0;
    enc_cstate(&b, g->candC); hash32_of(&b, out + 96);
  }
  free(b.p);
}

/* The vote cache of the candidate's (else the chain's) ActiveState: count, and when cap
 * allows, every 32-byte key and VoteTotalDeposit (unordered). */
uint64_t oracle_replay_vote_totals(void* h, uint8_t* hashes, uint64_t* totals, uint64_t cap) {
  chain_t* g = (chain_t*)h;
  vote_cache* c = g->has_cand ? g->candA->cache : g->A->cache;
  if (!c) return 0;
  if (cap >= c->count) {
    uint64_t k = 0;
    for (uint64_t i = 0; i < c->cap; ++i)
      if (c->tab[i].used) { memcpy(hashes + 32 * k, c->tab[i].key, 32); totals[k++] = c->tab[i].total; }
  }
  return c->count;
}

void oracle_replay_free(void* h) {
  chain_t* g = (chain_t*)h;
  if (!g) return;
  /* validators are individual heap records; the first state's slice owns them */
  cstate_t* c = g->C;
  for (uint64_t i = 0; i < c->nval; ++i) free(c->validators[i]);
  vc_free(&g->cache);
  free(g->saved);
  afree(&g->ar);
  free(g);
}
