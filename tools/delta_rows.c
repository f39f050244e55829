/*
 * delta_rows.c — bench tool: the relation consumer by delta (Go `Sets`): every
 * entity's neighbour set kept as a sorted array per slot (InterestedIn == InterestedBy under the XZ
 * manager, Entity.go:53-54), patched with gwaoi_export_relation_delta's entries {row, col | ENTER}: an
 * ENTER inserts col into row (binary search + shift), a LEAVE removes it. Host cost per entry is a
 * search and a shift inside one short row, instead of a hash-set operation per event and direction.
 * Counts inconsistent entries (insert of a present col, removal of an absent one): 0 when the delta is
 * exactly the relation's change.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint32_t nrows;
  uint32_t* len;
  uint32_t* cap;
  uint32_t** row;
} dr_sets;

void dr_destroy(dr_sets* s);

dr_sets* dr_create(const uint32_t* row_ptr, const uint32_t* cols, uint32_t nrows) {
  dr_sets* s = calloc(1, sizeof *s);
  if (!s) return NULL;
  s->nrows = nrows;
  s->len = calloc(nrows, sizeof *s->len);
  s->cap = calloc(nrows, sizeof *s->cap);
  s->row = calloc(nrows, sizeof *s->row); /* zeroed: dr_destroy frees only the rows built */
  if (!s->len || !s->cap || !s->row) {
    dr_destroy(s);
    return NULL;
  }
  for (uint32_t r = 0; r < nrows; ++r) {
    const uint32_t n = row_ptr[r + 1] - row_ptr[r];
    s->cap[r] = n + 8;
    s->row[r] = malloc(s->cap[r] * sizeof(uint32_t));
    if (!s->row[r]) {
      dr_destroy(s);
      return NULL;
    }
    memcpy(s->row[r], cols + row_ptr[r], n * sizeof(uint32_t));
    s->len[r] = n;
  }
  return s;
}

void dr_destroy(dr_sets* s) {
  if (!s) return;
  if (s->row)
    for (uint32_t r = 0; r < s->nrows; ++r) free(s->row[r]);
  free(s->row);
  free(s->cap);
  free(s->len);
  free(s);
}

static uint32_t lower(const uint32_t* a, uint32_t n, uint32_t v) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

/* entries: n x {row, col | 0x80000000 (joined) or col (left)} */
uint64_t dr_apply(dr_sets* s, const uint32_t* d, uint64_t n) {
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t r = d[2 * i], c = d[2 * i + 1] & 0x7FFFFFFFu, add = d[2 * i + 1] >> 31;
    if (r >= s->nrows) {
      ++bad;
      continue;
    }
    uint32_t* a = s->row[r];
    const uint32_t len = s->len[r], p = lower(a, len, c);
    const int present = p < len && a[p] == c;
    if (add) {
      if (present) {
        ++bad;
        continue;
      }
      if (len == s->cap[r]) {
        const uint32_t nc = s->cap[r] * 2 + 8;
        uint32_t* b = realloc(a, nc * sizeof(uint32_t));
        if (!b) return ~0ull;
        s->row[r] = a = b;
        s->cap[r] = nc;
      }
      memmove(a + p + 1, a + p, (len - p) * sizeof(uint32_t));
      a[p] = c;
      s->len[r] = len + 1;
    } else {
      if (!present) {
        ++bad;
        continue;
      }
      memmove(a + p, a + p + 1, (len - p - 1) * sizeof(uint32_t));
      s->len[r] = len - 1;
    }
  }
  return bad;
}

/* dr_apply over worker threads: thread k applies the entries of rows r with r % nthreads == k, in entry
 * order (every row belongs to one thread, so the per-row result equals dr_apply's) */
typedef struct {
  dr_sets* s;
  const uint32_t* d;
  uint64_t n;
  uint32_t k, nt;
  uint64_t bad;
} dr_job;

static void* dr_run(void* p) {
  dr_job* j = (dr_job*)p;
  dr_sets* s = j->s;
  uint64_t bad = 0;
  for (uint64_t i = 0; i < j->n; ++i) {
    const uint32_t r = j->d[2 * i];
    if (r % j->nt != j->k) continue;
    const uint64_t b = dr_apply(s, j->d + 2 * i, 1);
    if (b == ~0ull) {
      j->bad = ~0ull;
      return NULL;
    }
    bad += b;
  }
  j->bad = bad;
  return NULL;
}

uint64_t dr_apply_mt(dr_sets* s, const uint32_t* d, uint64_t n, uint32_t nthreads) {
  if (nthreads < 2) return dr_apply(s, d, n);
  pthread_t* th = calloc(nthreads, sizeof(pthread_t));
  dr_job* jb = calloc(nthreads, sizeof(dr_job));
  uint64_t bad = 0;
  if (!th || !jb) {
    free(th);
    free(jb);
    return ~0ull;
  }
  for (uint32_t k = 0; k < nthreads; ++k) {
    jb[k] = (dr_job){s, d, n, k, nthreads, 0};
    if (pthread_create(&th[k], NULL, dr_run, &jb[k])) dr_run(&jb[k]), th[k] = 0;
  }
  for (uint32_t k = 0; k < nthreads; ++k) {
    if (th[k]) pthread_join(th[k], NULL);
    bad = (bad == ~0ull || jb[k].bad == ~0ull) ? ~0ull : bad + jb[k].bad;
  }
  free(th);
  free(jb);
  return bad;
}

/* rows that differ from the CSR (row_ptr, cols) */
uint64_t dr_diff(const dr_sets* s, const uint32_t* row_ptr, const uint32_t* cols) {
  uint64_t bad = 0;
  for (uint32_t r = 0; r < s->nrows; ++r) {
    const uint32_t n = row_ptr[r + 1] - row_ptr[r];
    if (n != s->len[r] || memcmp(s->row[r], cols + row_ptr[r], n * sizeof(uint32_t))) ++bad;
  }
  return bad;
}
