/*
 * replay_sets.c — bench tool (not product, not an oracle): the cost of the Go-side callback sink.
 *
 * In GoWorld every AOI pair event fires two callbacks (mover first), and each callback runs
 * Entity.interest / uninterest (/root/reference/engine/entity/Entity.go:227-246):
 *     OnEnterAOI(other): e.InterestedIn.Add(other); other.InterestedBy.Add(e)
 *     OnLeaveAOI(other): e.InterestedIn.Del(other); other.InterestedBy.Del(e)
 * i.e. four hash-set operations per pair event on map[*Entity]struct{} sets (entity_map.go:164-187).
 * This file stands in for those sets with one open-addressing hash set of 64-bit keys
 * (set | entity << 1 | other << 32), populated with the current relation, so bench.py can time the
 * replay of a tick's events (`replay_ms`) next to the GPU tick. Single-threaded, like the game loop.
 * The sharded variant (rs_sharded_*) is the same sink split by owning entity over worker threads (a Go
 * sink could do the same with one goroutine per shard: every set operation belongs to exactly one
 * entity's set, so the shards never touch each other's state): `replay_ms_sharded`.
 * Built by __graft_entry__.build() into tools/_bin/libreplay.so.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t* t;
  uint64_t mask;
  uint64_t used;   /* live + tombstones */
  uint64_t live;
} rs_set;

static const uint64_t kEmpty = 0, kTomb = ~0ull;

static inline uint64_t mix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

/* key of "b in set X of a" (X: 0 = InterestedIn, 1 = InterestedBy); never 0 or ~0 */
static inline uint64_t key(uint32_t a, uint32_t b, uint32_t x) { return ((uint64_t)b << 32 | (uint64_t)a << 1 | x) + 1; }

rs_set* rs_create(uint64_t expect) {
  rs_set* s = (rs_set*)calloc(1, sizeof *s);
  if (!s) return NULL;
  uint64_t cap = 1024;
  while (cap < 2 * expect + 1024) cap <<= 1;
  s->t = (uint64_t*)calloc(cap, sizeof(uint64_t));
  if (!s->t) {
    free(s);
    return NULL;
  }
  s->mask = cap - 1;
  return s;
}

void rs_destroy(rs_set* s) {
  if (!s) return;
  free(s->t);
  free(s);
}

static int rs_insert(rs_set* s, uint64_t k);

static void rs_rehash(rs_set* s) {
  const uint64_t old = s->mask + 1;
  uint64_t* ot = s->t;
  uint64_t cap = old;
  if (s->live * 2 > old / 2) cap <<= 1;
  s->t = (uint64_t*)calloc(cap, sizeof(uint64_t));
  s->mask = cap - 1;
  s->used = s->live = 0;
  for (uint64_t i = 0; i < old; ++i)
    if (ot[i] != kEmpty && ot[i] != kTomb) rs_insert(s, ot[i]);
  free(ot);
}

/* 1 if inserted, 0 if it was present */
static int rs_insert(rs_set* s, uint64_t k) {
  if ((s->used + 1) * 4 > (s->mask + 1) * 3) rs_rehash(s);
  uint64_t i = mix(k) & s->mask, tomb = ~0ull;
  for (;; i = (i + 1) & s->mask) {
    const uint64_t v = s->t[i];
    if (v == k) return 0;
    if (v == kTomb) {
      if (tomb == ~0ull) tomb = i;
    } else if (v == kEmpty) {
      if (tomb != ~0ull) {
        i = tomb;
      } else {
        ++s->used;
      }
      s->t[i] = k;
      ++s->live;
      return 1;
    }
  }
}

/* 1 if erased, 0 if it was absent */
static int rs_erase(rs_set* s, uint64_t k) {
  for (uint64_t i = mix(k) & s->mask;; i = (i + 1) & s->mask) {
    const uint64_t v = s->t[i];
    if (v == k) {
      s->t[i] = kTomb;
      --s->live;
      return 1;
    }
    if (v == kEmpty) return 0;
  }
}

/* The sets of the current relation: row s = neighbours of s (CSR over slots). */
void rs_load_relation(rs_set* s, const uint32_t* row_ptr, const uint32_t* cols, uint32_t nrows) {
  for (uint32_t a = 0; a < nrows; ++a)
    for (uint32_t p = row_ptr[a]; p < row_ptr[a + 1]; ++p) {
      rs_insert(s, key(a, cols[p], 0));
      rs_insert(s, key(a, cols[p], 1));
    }
}

/* Replay pair events {mover, other | 0x80000000 for ENTER}: mover's callback, then other's.
 * Returns the number of set operations that found an inconsistent state (0 when the events are
 * exactly the relation's changes). */
uint64_t rs_replay(rs_set* s, const uint32_t* ev, uint64_t count) {
  uint64_t bad = 0;
  for (uint64_t i = 0; i < count; ++i) {
    const uint32_t m = ev[2 * i], o = ev[2 * i + 1] & 0x7fffffffu;
    if (ev[2 * i + 1] & 0x80000000u) {
      bad += !rs_insert(s, key(m, o, 0)); /* m.InterestedIn.Add(o) */
      bad += !rs_insert(s, key(o, m, 1)); /* o.InterestedBy.Add(m) */
      bad += !rs_insert(s, key(o, m, 0)); /* o.InterestedIn.Add(m) */
      bad += !rs_insert(s, key(m, o, 1)); /* m.InterestedBy.Add(o) */
    } else {
      bad += !rs_erase(s, key(m, o, 0));
      bad += !rs_erase(s, key(o, m, 1));
      bad += !rs_erase(s, key(o, m, 0));
      bad += !rs_erase(s, key(m, o, 1));
    }
  }
  return bad;
}

uint64_t rs_size(const rs_set* s) { return s->live; }

/* ---- sharded sink: shard k holds the set entries of the entities a with a % nshards == k ---- */
typedef struct {
  uint32_t n;
  rs_set** sh;
} rs_sharded;

rs_sharded* rs_sharded_create(uint64_t expect, uint32_t nshards) {
  rs_sharded* r = (rs_sharded*)calloc(1, sizeof *r);
  if (!r) return NULL;
  r->n = nshards ? nshards : 1;
  r->sh = (rs_set**)calloc(r->n, sizeof(rs_set*));
  if (!r->sh) {
    free(r);
    return NULL;
  }
  for (uint32_t k = 0; k < r->n; ++k)
    if (!(r->sh[k] = rs_create(expect / r->n + 1024))) {
      for (uint32_t j = 0; j < k; ++j) rs_destroy(r->sh[j]);
      free(r->sh);
      free(r);
      return NULL;
    }
  return r;
}

void rs_sharded_destroy(rs_sharded* r) {
  if (!r) return;
  for (uint32_t k = 0; k < r->n; ++k) rs_destroy(r->sh[k]);
  free(r->sh);
  free(r);
}

void rs_sharded_load_relation(rs_sharded* r, const uint32_t* row_ptr, const uint32_t* cols, uint32_t nrows) {
  for (uint32_t a = 0; a < nrows; ++a) {
    rs_set* s = r->sh[a % r->n];
    for (uint32_t p = row_ptr[a]; p < row_ptr[a + 1]; ++p) {
      rs_insert(s, key(a, cols[p], 0));
      rs_insert(s, key(a, cols[p], 1));
    }
  }
}

typedef struct {
  rs_sharded* r;
  uint32_t k;
  const uint32_t* ev;
  uint64_t count;
  uint64_t bad;
} rs_job;

/* every event, only the set operations of this shard's entities (same order per set as rs_replay) */
static void* rs_shard_run(void* p) {
  rs_job* j = (rs_job*)p;
  rs_set* s = j->r->sh[j->k];
  const uint32_t n = j->r->n, k = j->k;
  uint64_t bad = 0;
  for (uint64_t i = 0; i < j->count; ++i) {
    const uint32_t m = j->ev[2 * i], o = j->ev[2 * i + 1] & 0x7fffffffu;
    const int mine_m = m % n == k, mine_o = o % n == k;
    if (!mine_m && !mine_o) continue;
    if (j->ev[2 * i + 1] & 0x80000000u) {
      if (mine_m) bad += !rs_insert(s, key(m, o, 0)) + !rs_insert(s, key(m, o, 1));
      if (mine_o) bad += !rs_insert(s, key(o, m, 1)) + !rs_insert(s, key(o, m, 0));
    } else {
      if (mine_m) bad += !rs_erase(s, key(m, o, 0)) + !rs_erase(s, key(m, o, 1));
      if (mine_o) bad += !rs_erase(s, key(o, m, 1)) + !rs_erase(s, key(o, m, 0));
    }
  }
  j->bad = bad;
  return NULL;
}

/* one worker thread per shard; returns the inconsistent set operations (as rs_replay) */
uint64_t rs_sharded_replay(rs_sharded* r, const uint32_t* ev, uint64_t count) {
  pthread_t* th = (pthread_t*)calloc(r->n, sizeof(pthread_t));
  rs_job* jb = (rs_job*)calloc(r->n, sizeof(rs_job));
  uint64_t bad = 0;
  if (!th || !jb) {
    free(th);
    free(jb);
    return ~0ull;
  }
  for (uint32_t k = 0; k < r->n; ++k) {
    jb[k] = (rs_job){r, k, ev, count, 0};
    if (pthread_create(&th[k], NULL, rs_shard_run, &jb[k])) rs_shard_run(&jb[k]), th[k] = 0;
  }
  for (uint32_t k = 0; k < r->n; ++k) {
    if (th[k]) pthread_join(th[k], NULL);
    bad += jb[k].bad;
  }
  free(th);
  free(jb);
  return bad;
}

uint64_t rs_sharded_size(const rs_sharded* r) {
  uint64_t n = 0;
  for (uint32_t k = 0; k < r->n; ++k) n += r->sh[k]->live;
  return n;
}
