/*
 * TEST INFRASTRUCTURE ONLY — never linked into or called by the product (libgwaoi).
 *
 * oracle (ii): the AOI semantics of SURVEY.md §8a-R restated as a STATEFUL sequential model, with a
 * uniform grid only to find candidates. It shares no code and no algorithm with the GPU pipeline
 * (which is tick-batched and stateless); it is cross-checked against oracle (i) (xzlist_aoi.c, the
 * go-aoi list restatement) in tests/, and is the checker used at full size (1M entities), where the
 * list restatement costs O(N^1.5) per tick.
 *
 * Semantics (go-aoi v0.2.0 XZListAOIManager, rev 5e9d879, Gopkg.lock:155-159 [UPSTREAM-RECALLED];
 * call sites engine/entity/Space.go:211,221,243,259):
 *   in(m, o) := fl32(m.x-D) <= o.x <= fl32(m.x+D) && fl32(m.z-D) <= o.z <= fl32(m.z+D)
 *   Enter(m):  ENTER(m,o) for every present o != m with in(m,o)
 *   Leave(m):  LEAVE(m,o) for every o in N(m)
 *   Moved(m):  LEAVE(m,o) for o in N(m) with !in(m_new,o); ENTER(m,o) for o not in N(m) with in(m_new,o)
 * where N is the explicit symmetric neighbour relation, updated as events fire.
 * PARITY UNPINNED (see xzlist_aoi.c header).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define GR_EV_ENTER 0x80000000u

typedef struct {
  uint32_t mover;
  uint32_t other;
} gr_event;

typedef struct {
  uint32_t* v;
  uint32_t n, cap;
} gr_vec;

typedef struct {
  float dist;
  uint32_t cap;
  double x0, z0, cs;
  int64_t ncx, ncz;
  float* x;
  float* z;
  uint8_t* present;
  uint32_t* cell_of;
  gr_vec* cells;
  gr_vec* nb;
  uint32_t* stampA;
  uint32_t* stampN;
  uint32_t opid;
  gr_event* ev;
  uint64_t nev, evcap;
  int record;
} gr_mgr;

static void vpush(gr_vec* a, uint32_t s) {
  if (a->n == a->cap) {
    a->cap = a->cap ? a->cap * 2 : 8;
    a->v = (uint32_t*)realloc(a->v, a->cap * sizeof(uint32_t));
  }
  a->v[a->n++] = s;
}

static void vdel(gr_vec* a, uint32_t s) {
  for (uint32_t i = 0; i < a->n; ++i) {
    if (a->v[i] == s) {
      a->v[i] = a->v[--a->n];
      return;
    }
  }
}

static void gemit(gr_mgr* m, uint32_t mover, uint32_t other, int enter) {
  if (!m->record) return;
  if (m->nev == m->evcap) {
    m->evcap = m->evcap ? m->evcap * 2 : 1024;
    m->ev = (gr_event*)realloc(m->ev, m->evcap * sizeof(gr_event));
  }
  m->ev[m->nev].mover = mover;
  m->ev[m->nev].other = other | (enter ? GR_EV_ENTER : 0u);
  m->nev++;
}

static int64_t cellc(double v, double o, double cs, int64_t n) {
  double f = floor((v - o) / cs);
  if (!(f >= 0)) return 0;
  if (f >= (double)n) return n - 1;
  return (int64_t)f;
}

/* bounds: the grid covers [minx,maxx]x[minz,maxz]; positions outside are clamped into edge cells. */
gr_mgr* gr_create(float dist, uint32_t cap, float minx, float minz, float maxx, float maxz) {
  gr_mgr* m = (gr_mgr*)calloc(1, sizeof(gr_mgr));
  m->dist = dist;
  m->cap = cap;
  m->cs = (double)dist;
  if (!(maxx > minx)) maxx = minx + dist;
  if (!(maxz > minz)) maxz = minz + dist;
  m->x0 = minx;
  m->z0 = minz;
  m->ncx = (int64_t)(((double)maxx - minx) / m->cs) + 1;
  m->ncz = (int64_t)(((double)maxz - minz) / m->cs) + 1;
  while (m->ncx * m->ncz > 4 * (int64_t)cap + 64) {
    m->cs *= 2;
    m->ncx = (int64_t)(((double)maxx - minx) / m->cs) + 1;
    m->ncz = (int64_t)(((double)maxz - minz) / m->cs) + 1;
  }
  uint32_t c1 = cap ? cap : 1;
  m->x = (float*)calloc(c1, sizeof(float));
  m->z = (float*)calloc(c1, sizeof(float));
  m->present = (uint8_t*)calloc(c1, 1);
  m->cell_of = (uint32_t*)calloc(c1, sizeof(uint32_t));
  m->cells = (gr_vec*)calloc((size_t)(m->ncx * m->ncz), sizeof(gr_vec));
  m->nb = (gr_vec*)calloc(c1, sizeof(gr_vec));
  m->stampA = (uint32_t*)calloc(c1, sizeof(uint32_t));
  m->stampN = (uint32_t*)calloc(c1, sizeof(uint32_t));
  m->record = 1;
  return m;
}

void gr_destroy(gr_mgr* m) {
  if (!m) return;
  for (int64_t c = 0; c < m->ncx * m->ncz; ++c) free(m->cells[c].v);
  for (uint32_t s = 0; s < m->cap; ++s) free(m->nb[s].v);
  free(m->cells);
  free(m->nb);
  free(m->x);
  free(m->z);
  free(m->present);
  free(m->cell_of);
  free(m->stampA);
  free(m->stampN);
  free(m->ev);
  free(m);
}

void gr_set_record(gr_mgr* m, int r) { m->record = r; }
uint64_t gr_event_count(const gr_mgr* m) { return m->nev; }
const gr_event* gr_events(const gr_mgr* m) { return m->ev; }
void gr_clear_events(gr_mgr* m) { m->nev = 0; }

static uint32_t cell_index(gr_mgr* m, float x, float z) {
  return (uint32_t)(cellc(x, m->x0, m->cs, m->ncx) + m->ncx * cellc(z, m->z0, m->cs, m->ncz));
}

static int inbox(float cx, float cz, float d, float px, float pz) {
  float lx = cx - d, hx = cx + d, lz = cz - d, hz = cz + d;
  return px >= lx && px <= hx && pz >= lz && pz <= hz;
}

/* stamp every present o != s with in(s at (x,z), o) into stampA with the current opid */
static void query(gr_mgr* m, uint32_t s, float x, float z, gr_vec* out) {
  float d = m->dist;
  int64_t cx0 = cellc((double)x - d, m->x0, m->cs, m->ncx) - 1, cx1 = cellc((double)x + d, m->x0, m->cs, m->ncx) + 1;
  int64_t cz0 = cellc((double)z - d, m->z0, m->cs, m->ncz) - 1, cz1 = cellc((double)z + d, m->z0, m->cs, m->ncz) + 1;
  if (cx0 < 0) cx0 = 0;
  if (cz0 < 0) cz0 = 0;
  if (cx1 >= m->ncx) cx1 = m->ncx - 1;
  if (cz1 >= m->ncz) cz1 = m->ncz - 1;
  out->n = 0;
  for (int64_t cz = cz0; cz <= cz1; ++cz) {
    for (int64_t cx = cx0; cx <= cx1; ++cx) {
      gr_vec* c = &m->cells[cz * m->ncx + cx];
      for (uint32_t i = 0; i < c->n; ++i) {
        uint32_t o = c->v[i];
        if (o == s) continue;
        if (inbox(x, z, d, m->x[o], m->z[o])) {
          m->stampA[o] = m->opid;
          vpush(out, o);
        }
      }
    }
  }
}

static gr_vec g_scratch;

int gr_enter(gr_mgr* m, uint32_t s, float x, float z) {
  if (s >= m->cap || m->present[s]) return -2;
  m->opid++;
  m->x[s] = x;
  m->z[s] = z;
  query(m, s, x, z, &g_scratch);
  for (uint32_t i = 0; i < g_scratch.n; ++i) {
    uint32_t o = g_scratch.v[i];
    vpush(&m->nb[s], o);
    vpush(&m->nb[o], s);
    gemit(m, s, o, 1);
  }
  m->present[s] = 1;
  m->cell_of[s] = cell_index(m, x, z);
  vpush(&m->cells[m->cell_of[s]], s);
  return 0;
}

int gr_leave(gr_mgr* m, uint32_t s) {
  if (s >= m->cap || !m->present[s]) return -2;
  gr_vec* nb = &m->nb[s];
  for (uint32_t i = 0; i < nb->n; ++i) {
    gemit(m, s, nb->v[i], 0);
    vdel(&m->nb[nb->v[i]], s);
  }
  nb->n = 0;
  vdel(&m->cells[m->cell_of[s]], s);
  m->present[s] = 0;
  return 0;
}

int gr_moved(gr_mgr* m, uint32_t s, float x, float z) {
  if (s >= m->cap || !m->present[s]) return -2;
  m->opid++;
  uint32_t c = cell_index(m, x, z);
  if (c != m->cell_of[s]) {
    vdel(&m->cells[m->cell_of[s]], s);
    vpush(&m->cells[c], s);
    m->cell_of[s] = c;
  }
  m->x[s] = x;
  m->z[s] = z;
  query(m, s, x, z, &g_scratch);
  gr_vec* nb = &m->nb[s];
  uint32_t keep = 0;
  for (uint32_t i = 0; i < nb->n; ++i) {
    uint32_t o = nb->v[i];
    if (m->stampA[o] == m->opid) {
      m->stampN[o] = m->opid;
      nb->v[keep++] = o;
    } else {
      gemit(m, s, o, 0);
      vdel(&m->nb[o], s);
    }
  }
  nb->n = keep;
  for (uint32_t i = 0; i < g_scratch.n; ++i) {
    uint32_t o = g_scratch.v[i];
    if (m->stampN[o] == m->opid) continue;
    vpush(nb, o);
    vpush(&m->nb[o], s);
    gemit(m, s, o, 1);
  }
  return 0;
}

int gr_moved_batch(gr_mgr* m, uint32_t n, const uint32_t* slots, const float* x, const float* z) {
  for (uint32_t i = 0; i < n; ++i) {
    int r = gr_moved(m, slots[i], x[i], z[i]);
    if (r) return r;
  }
  return 0;
}

/* Bulk Enter in array order with events suppressed (restore path). Uses the sequential definition
 * directly, so it is O(N k) and exact. */
int gr_bulk_enter(gr_mgr* m, uint32_t n, const uint32_t* slots, const float* x, const float* z) {
  int rec = m->record;
  m->record = 0;
  for (uint32_t i = 0; i < n; ++i) {
    int r = gr_enter(m, slots[i], x[i], z[i]);
    if (r) {
      m->record = rec;
      return r;
    }
  }
  m->record = rec;
  return 0;
}

static int u32cmp(const void* a, const void* b) {
  uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return x < y ? -1 : x > y;
}

int64_t gr_export_relation(gr_mgr* m, uint32_t* row_ptr, uint32_t* cols, uint64_t cols_cap) {
  uint64_t nnz = 0;
  for (uint32_t s = 0; s < m->cap; ++s) nnz += m->present[s] ? m->nb[s].n : 0;
  if (nnz > cols_cap) return -(int64_t)nnz;
  uint64_t o = 0;
  for (uint32_t s = 0; s < m->cap; ++s) {
    row_ptr[s] = (uint32_t)o;
    if (!m->present[s]) continue;
    memcpy(cols + o, m->nb[s].v, m->nb[s].n * sizeof(uint32_t));
    qsort(cols + o, m->nb[s].n, sizeof(uint32_t), u32cmp);
    o += m->nb[s].n;
  }
  row_ptr[m->cap] = (uint32_t)o;
  return (int64_t)o;
}
