/*
 * TEST INFRASTRUCTURE ONLY — never linked into or called by the product (libgwaoi).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 *
 * oracle (i): a faithful CPU restatement of go-aoi v0.2.0's XZListAOIManager
 * (module github.com/xiaonanln/go-aoi, rev 5e9d87993768c88f87e40b2b66d6be3fdabde228, pinned at
 * /root/reference/Gopkg.lock:155-159, constraint Gopkg.toml:84-86). That module is NOT vendored in
 * /root/reference and there is no Go toolchain in this image, so the structure below restates the
 * published upstream source [UPSTREAM-RECALLED] and is anchored on goworld's call sites:
 *   NewXZListAOIManager(dist)  <- engine/entity/Space.go:105
 *   Enter(aoi, x, z)           <- engine/entity/Space.go:211, 221
 *   Leave(aoi)                 <- engine/entity/Space.go:243
 *   Moved(aoi, x, z)           <- engine/entity/Space.go:259
 *   callbacks OnEnterAOI/OnLeaveAOI <- engine/entity/Entity.go:227-233
 * PARITY UNPINNED: the reference holds no AOI golden vector, known-answer test or fixture
 * (SURVEY.md §4, §8c); the only AOI check it has (DoTestAOI, examples/test_client/ClientEntity.go:367-379
 * with examples/test_game/Avatar.go:267-280) is encoded as a known-answer test in tests/.
 *
 * Upstream structure restated here:
 *   xzaoi { aoi; neighbors map[*xzaoi]struct{}; xPrev,xNext,yPrev,yNext *xzaoi; markVal int }
 *   two doubly linked lists sorted non-decreasing by x and by z ("y" in go-aoi is GoWorld's Z).
 *   Insert: scan from head, insert before the first node with coord >= new coord.
 *   Remove: unlink, nil the node's links.
 *   Move(node, oldCoord): bubble forward (coord > old) past nodes with coord < new, or backward past
 *     nodes with coord > new.
 *   Mark: walk prev while prev.x >= fl32(x - D), next while next.x <= fl32(x + D); markVal += 1.
 *   adjust(m): Mark(X); Mark(Z); for each neighbour n: markVal == 2 -> keep (markVal = -2), else
 *     delete both directions and fire m.OnLeaveAOI(n), n.OnLeaveAOI(m);
 *     GetClearMarkedNeighbors(X): every node in m's X strip with markVal == 2 becomes a neighbour
 *     (m.OnEnterAOI(n), n.OnEnterAOI(m)); every X-strip node's markVal = 0;  ClearMark(Z).
 *   Enter: new node, set coords, Insert into both lists, adjust.
 *   Leave: Remove from both lists, adjust (no marks -> every neighbour leaves).
 *   Moved: set coords; Move in X if x changed, in Z if z changed; adjust.
 * Float arithmetic: Coord is float32; every bound is one binary32 add/sub (compile -ffp-contract=off).
 *
 * One recorded event per pair event (the pair of callbacks mover->other, other->mover), in emission
 * order, in the same 8-byte layout as gwaoi_event.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define XZ_NIL (-1)
#define XZ_EV_ENTER 0x80000000u

typedef struct {
  uint32_t mover;
  uint32_t other;
} xz_event;

typedef struct {
  int32_t xprev, xnext, zprev, znext;
  int32_t mark;
  float x, z;
  int present;
  uint32_t* nb; /* neighbours (the Go map, here an unordered array) */
  uint32_t nn, ncap;
} xz_node;

typedef struct {
  float dist;
  uint32_t cap;
  int32_t xhead, xtail, zhead, ztail;
  xz_node* nodes;
  xz_event* ev;
  uint64_t nev, evcap;
  int record;
} xz_mgr;

static void nb_add(xz_node* n, uint32_t s) {
  if (n->nn == n->ncap) {
    n->ncap = n->ncap ? n->ncap * 2 : 8;
    n->nb = (uint32_t*)realloc(n->nb, n->ncap * sizeof(uint32_t));
  }
  n->nb[n->nn++] = s;
}

static void nb_del(xz_node* n, uint32_t s) {
  for (uint32_t i = 0; i < n->nn; ++i) {
    if (n->nb[i] == s) {
      n->nb[i] = n->nb[--n->nn];
      return;
    }
  }
}

static void emit(xz_mgr* m, uint32_t mover, uint32_t other, int enter) {
  if (!m->record) return;
  if (m->nev == m->evcap) {
    m->evcap = m->evcap ? m->evcap * 2 : 1024;
    m->ev = (xz_event*)realloc(m->ev, m->evcap * sizeof(xz_event));
  }
  m->ev[m->nev].mover = mover;
  m->ev[m->nev].other = other | (enter ? XZ_EV_ENTER : 0u);
  m->nev++;
}

xz_mgr* xz_create(float dist, uint32_t cap) {
  xz_mgr* m = (xz_mgr*)calloc(1, sizeof(xz_mgr));
  m->dist = dist;
  m->cap = cap;
  m->xhead = m->xtail = m->zhead = m->ztail = XZ_NIL;
  m->nodes = (xz_node*)calloc(cap ? cap : 1, sizeof(xz_node));
  for (uint32_t i = 0; i < cap; ++i) {
    m->nodes[i].xprev = m->nodes[i].xnext = m->nodes[i].zprev = m->nodes[i].znext = XZ_NIL;
  }
  m->record = 1;
  return m;
}

void xz_destroy(xz_mgr* m) {
  if (!m) return;
  for (uint32_t i = 0; i < m->cap; ++i) free(m->nodes[i].nb);
  free(m->nodes);
  free(m->ev);
  free(m);
}

void xz_set_record(xz_mgr* m, int record) { m->record = record; }
uint64_t xz_event_count(const xz_mgr* m) { return m->nev; }
const xz_event* xz_events(const xz_mgr* m) { return m->ev; }
void xz_clear_events(xz_mgr* m) { m->nev = 0; }

/* ---- xAOIList / yAOIList (one generic body, axis selected by pointer offsets) ---- */

#define AX_X 0
#define AX_Z 1
static inline float crd(const xz_node* n, int ax) { return ax == AX_X ? n->x : n->z; }
static inline int32_t* prv(xz_node* n, int ax) { return ax == AX_X ? &n->xprev : &n->zprev; }
static inline int32_t* nxt(xz_node* n, int ax) { return ax == AX_X ? &n->xnext : &n->znext; }
static inline int32_t* head(xz_mgr* m, int ax) { return ax == AX_X ? &m->xhead : &m->zhead; }
static inline int32_t* tail(xz_mgr* m, int ax) { return ax == AX_X ? &m->xtail : &m->ztail; }
#define N(i) (&m->nodes[(i)])

static void list_insert(xz_mgr* m, int ax, int32_t a) {
  float c = crd(N(a), ax);
  if (*head(m, ax) != XZ_NIL) {
    int32_t p = *head(m, ax);
    while (p != XZ_NIL && crd(N(p), ax) < c) p = *nxt(N(p), ax);
    if (p == XZ_NIL) { /* append at tail */
      int32_t t = *tail(m, ax);
      *nxt(N(t), ax) = a;
      *prv(N(a), ax) = t;
      *tail(m, ax) = a;
    } else { /* insert before p */
      int32_t pr = *prv(N(p), ax);
      *nxt(N(a), ax) = p;
      *prv(N(p), ax) = a;
      *prv(N(a), ax) = pr;
      if (pr != XZ_NIL) *nxt(N(pr), ax) = a;
      else *head(m, ax) = a;
    }
  } else {
    *head(m, ax) = a;
    *tail(m, ax) = a;
  }
}

static void list_remove(xz_mgr* m, int ax, int32_t a) {
  int32_t pr = *prv(N(a), ax), nx = *nxt(N(a), ax);
  if (pr != XZ_NIL) {
    *nxt(N(pr), ax) = nx;
    *prv(N(a), ax) = XZ_NIL;
  } else {
    *head(m, ax) = nx;
  }
  if (nx != XZ_NIL) {
    *prv(N(nx), ax) = pr;
    *nxt(N(a), ax) = XZ_NIL;
  } else {
    *tail(m, ax) = pr;
  }
}

static void list_move(xz_mgr* m, int ax, int32_t a, float old) {
  float c = crd(N(a), ax);
  if (c > old) { /* moving towards the tail */
    int32_t nx = *nxt(N(a), ax);
    if (nx == XZ_NIL || crd(N(nx), ax) >= c) return;
    int32_t pr = *prv(N(a), ax);
    if (pr != XZ_NIL) *nxt(N(pr), ax) = nx;
    else *head(m, ax) = nx;
    *prv(N(nx), ax) = pr;
    pr = nx;
    nx = *nxt(N(nx), ax);
    while (nx != XZ_NIL && crd(N(nx), ax) < c) {
      pr = nx;
      nx = *nxt(N(nx), ax);
    }
    *nxt(N(pr), ax) = a;
    *prv(N(a), ax) = pr;
    if (nx != XZ_NIL) *prv(N(nx), ax) = a;
    else *tail(m, ax) = a;
    *nxt(N(a), ax) = nx;
  } else { /* moving towards the head */
    int32_t pr = *prv(N(a), ax);
    if (pr == XZ_NIL || crd(N(pr), ax) <= c) return;
    int32_t nx = *nxt(N(a), ax);
    if (nx != XZ_NIL) *prv(N(nx), ax) = pr;
    else *tail(m, ax) = pr;
    *nxt(N(pr), ax) = nx;
    nx = pr;
    pr = *prv(N(pr), ax);
    while (pr != XZ_NIL && crd(N(pr), ax) > c) {
      nx = pr;
      pr = *prv(N(pr), ax);
    }
    *prv(N(nx), ax) = a;
    *nxt(N(a), ax) = nx;
    if (pr != XZ_NIL) *nxt(N(pr), ax) = a;
    else *head(m, ax) = a;
    *prv(N(a), ax) = pr;
  }
}

static void list_mark(xz_mgr* m, int ax, int32_t a) {
  float c = crd(N(a), ax);
  float lo = c - m->dist;
  for (int32_t p = *prv(N(a), ax); p != XZ_NIL && crd(N(p), ax) >= lo; p = *prv(N(p), ax)) N(p)->mark += 1;
  float hi = c + m->dist;
  for (int32_t p = *nxt(N(a), ax); p != XZ_NIL && crd(N(p), ax) <= hi; p = *nxt(N(p), ax)) N(p)->mark += 1;
}

static void enter_pair(xz_mgr* m, int32_t a, int32_t p) {
  nb_add(N(a), (uint32_t)p); /* aoi.neighbors[prev] = struct{}{}; aoi.callback.OnEnterAOI(prev.aoi) */
  emit(m, (uint32_t)a, (uint32_t)p, 1);
  nb_add(N(p), (uint32_t)a); /* prev.neighbors[aoi] = struct{}{}; prev.callback.OnEnterAOI(aoi.aoi) */
}

static void list_get_clear_marked_neighbors(xz_mgr* m, int32_t a) { /* X list only */
  float c = N(a)->x;
  float lo = c - m->dist;
  for (int32_t p = N(a)->xprev; p != XZ_NIL && N(p)->x >= lo; p = N(p)->xprev) {
    if (N(p)->mark == 2) enter_pair(m, a, p);
    N(p)->mark = 0;
  }
  float hi = c + m->dist;
  for (int32_t p = N(a)->xnext; p != XZ_NIL && N(p)->x <= hi; p = N(p)->xnext) {
    if (N(p)->mark == 2) enter_pair(m, a, p);
    N(p)->mark = 0;
  }
}

static void list_clear_mark(xz_mgr* m, int32_t a) { /* Z list only */
  float c = N(a)->z;
  float lo = c - m->dist;
  for (int32_t p = N(a)->zprev; p != XZ_NIL && N(p)->z >= lo; p = N(p)->zprev) N(p)->mark = 0;
  float hi = c + m->dist;
  for (int32_t p = N(a)->znext; p != XZ_NIL && N(p)->z <= hi; p = N(p)->znext) N(p)->mark = 0;
}

static void adjust(xz_mgr* m, int32_t a) {
  list_mark(m, AX_X, a);
  list_mark(m, AX_Z, a);
  xz_node* an = N(a);
  uint32_t keep = 0;
  for (uint32_t i = 0; i < an->nn; ++i) {
    uint32_t nbi = an->nb[i];
    if (N(nbi)->mark == 2) {
      N(nbi)->mark = -2; /* neighbour kept */
      an->nb[keep++] = nbi;
    } else { /* was a neighbour, not any more */
      emit(m, (uint32_t)a, nbi, 0); /* aoi.callback.OnLeaveAOI(neighbor.aoi) */
      nb_del(N(nbi), (uint32_t)a);  /* delete(neighbor.neighbors, aoi); neighbor...OnLeaveAOI(aoi.aoi) */
    }
  }
  an->nn = keep;
  list_get_clear_marked_neighbors(m, a);
  list_clear_mark(m, a);
}

int xz_enter(xz_mgr* m, uint32_t slot, float x, float z) {
  if (slot >= m->cap || m->nodes[slot].present) return -2;
  xz_node* n = N(slot);
  n->x = x;
  n->z = z;
  n->present = 1;
  n->mark = 0;
  n->nn = 0;
  n->xprev = n->xnext = n->zprev = n->znext = XZ_NIL;
  list_insert(m, AX_X, (int32_t)slot);
  list_insert(m, AX_Z, (int32_t)slot);
  adjust(m, (int32_t)slot);
  return 0;
}

int xz_leave(xz_mgr* m, uint32_t slot) {
  if (slot >= m->cap || !m->nodes[slot].present) return -2;
  list_remove(m, AX_X, (int32_t)slot);
  list_remove(m, AX_Z, (int32_t)slot);
  adjust(m, (int32_t)slot);
  m->nodes[slot].present = 0;
  return 0;
}

int xz_moved(xz_mgr* m, uint32_t slot, float x, float z) {
  if (slot >= m->cap || !m->nodes[slot].present) return -2;
  xz_node* n = N(slot);
  float ox = n->x, oz = n->z;
  n->x = x;
  n->z = z;
  if (ox != x) list_move(m, AX_X, (int32_t)slot, ox);
  if (oz != z) list_move(m, AX_Z, (int32_t)slot, oz);
  adjust(m, (int32_t)slot);
  return 0;
}

/* n Moved calls in array order; returns the first error or 0. */
int xz_moved_batch(xz_mgr* m, uint32_t n, const uint32_t* slots, const float* x, const float* z) {
  for (uint32_t i = 0; i < n; ++i) {
    int r = xz_moved(m, slots[i], x[i], z[i]);
    if (r) return r;
  }
  return 0;
}

/* ---- bulk load: the state n sequential Enter calls (in array order) would leave ---------------
 * Used only to set up large oracle instances (sequential Insert is O(N) per Enter). Equivalent
 * state: both lists sorted with the tie order sequential Insert produces (a later-entered node goes
 * before earlier nodes of equal coordinate), and N(a,b) = in(later, earlier) — after Enter(b) the
 * pair holds iff a is inside b's box, and a later Enter of a third entity never touches it.
 * Neighbour pairs are found with a uniform grid; events are not recorded (restore path,
 * EntityManager.go:615-649 attaches clients only after the restore). */
typedef struct {
  float c;
  uint32_t order;
  uint32_t slot;
} bl_key;

static int bl_cmp(const void* pa, const void* pb) {
  const bl_key* a = (const bl_key*)pa;
  const bl_key* b = (const bl_key*)pb;
  if (a->c < b->c) return -1;
  if (a->c > b->c) return 1;
  /* equal coordinate: later-entered first */
  if (a->order > b->order) return -1;
  if (a->order < b->order) return 1;
  return 0;
}

static int inbox(float cx, float cz, float d, float px, float pz) {
  float lx = cx - d, hx = cx + d, lz = cz - d, hz = cz + d;
  return px >= lx && px <= hx && pz >= lz && pz <= hz;
}

int xz_bulk_enter(xz_mgr* m, uint32_t n, const uint32_t* slots, const float* x, const float* z) {
  if (m->xhead != XZ_NIL) return -1; /* only into an empty manager */
  for (uint32_t i = 0; i < n; ++i) {
    if (slots[i] >= m->cap || m->nodes[slots[i]].present) return -2;
    xz_node* nd = N(slots[i]);
    nd->present = 1;
    nd->x = x[i];
    nd->z = z[i];
    nd->mark = 0;
    nd->nn = 0;
  }
  if (n == 0) return 0;
  bl_key* k = (bl_key*)malloc(n * sizeof(bl_key));
  for (int ax = 0; ax < 2; ++ax) {
    for (uint32_t i = 0; i < n; ++i) {
      k[i].c = ax == AX_X ? x[i] : z[i];
      k[i].order = i;
      k[i].slot = slots[i];
    }
    qsort(k, n, sizeof(bl_key), bl_cmp);
    for (uint32_t i = 0; i < n; ++i) {
      xz_node* nd = N(k[i].slot);
      *prv(nd, ax) = i ? (int32_t)k[i - 1].slot : XZ_NIL;
      *nxt(nd, ax) = i + 1 < n ? (int32_t)k[i + 1].slot : XZ_NIL;
    }
    *head(m, ax) = (int32_t)k[0].slot;
    *tail(m, ax) = (int32_t)k[n - 1].slot;
  }
  free(k);
  /* grid over the bounding box, cell side 2D (a candidate pair lies in adjacent cells) */
  float minx = x[0], maxx = x[0], minz = z[0], maxz = z[0];
  for (uint32_t i = 1; i < n; ++i) {
    if (x[i] < minx) minx = x[i];
    if (x[i] > maxx) maxx = x[i];
    if (z[i] < minz) minz = z[i];
    if (z[i] > maxz) maxz = z[i];
  }
  double cs = 2.0 * (double)m->dist * 1.0001 + 1e-30;
  int64_t ncx = (int64_t)(((double)maxx - minx) / cs) + 1, ncz = (int64_t)(((double)maxz - minz) / cs) + 1;
  while (ncx * ncz > 4 * (int64_t)n + 16) {
    cs *= 2;
    ncx = (int64_t)(((double)maxx - minx) / cs) + 1;
    ncz = (int64_t)(((double)maxz - minz) / cs) + 1;
  }
  uint32_t* cnt = (uint32_t*)calloc((size_t)(ncx * ncz + 1), sizeof(uint32_t));
  uint32_t* idx = (uint32_t*)malloc(n * sizeof(uint32_t));
  uint32_t* cell = (uint32_t*)malloc(n * sizeof(uint32_t));
  for (uint32_t i = 0; i < n; ++i) {
    int64_t cx = (int64_t)(((double)x[i] - minx) / cs), cz = (int64_t)(((double)z[i] - minz) / cs);
    if (cx >= ncx) cx = ncx - 1;
    if (cz >= ncz) cz = ncz - 1;
    cell[i] = (uint32_t)(cz * ncx + cx);
    cnt[cell[i] + 1]++;
  }
  for (int64_t c = 0; c < ncx * ncz; ++c) cnt[c + 1] += cnt[c];
  uint32_t* fill = (uint32_t*)malloc((size_t)(ncx * ncz) * sizeof(uint32_t));
  memcpy(fill, cnt, (size_t)(ncx * ncz) * sizeof(uint32_t));
  for (uint32_t i = 0; i < n; ++i) idx[fill[cell[i]]++] = i;
  free(fill);
  for (uint32_t i = 0; i < n; ++i) {
    int64_t cx = cell[i] % ncx, cz = cell[i] / ncx;
    for (int64_t dz = -1; dz <= 1; ++dz) {
      for (int64_t dx = -1; dx <= 1; ++dx) {
        int64_t qx = cx + dx, qz = cz + dz;
        if (qx < 0 || qz < 0 || qx >= ncx || qz >= ncz) continue;
        uint32_t c = (uint32_t)(qz * ncx + qx);
        for (uint32_t t = cnt[c]; t < cnt[c + 1]; ++t) {
          uint32_t j = idx[t];
          if (j >= i) continue; /* visit each pair once, from the later-entered side */
          if (inbox(x[i], z[i], m->dist, x[j], z[j])) {
            nb_add(N(slots[i]), slots[j]);
            nb_add(N(slots[j]), slots[i]);
          }
        }
      }
    }
  }
  free(cnt);
  free(idx);
  free(cell);
  return 0;
}

/* ---- inspection ---- */

int xz_present(const xz_mgr* m, uint32_t slot) { return slot < m->cap && m->nodes[slot].present; }

static int u32cmp(const void* a, const void* b) {
  uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return x < y ? -1 : x > y;
}

/* CSR of the relation, rows sorted ascending. row_ptr: cap+1. Returns nnz, or -(needed) if cols_cap
 * is too small (cols untouched then). */
int64_t xz_export_relation(xz_mgr* m, uint32_t* row_ptr, uint32_t* cols, uint64_t cols_cap) {
  uint64_t nnz = 0;
  for (uint32_t s = 0; s < m->cap; ++s) nnz += m->nodes[s].present ? m->nodes[s].nn : 0;
  if (nnz > cols_cap) return -(int64_t)nnz;
  uint64_t o = 0;
  for (uint32_t s = 0; s < m->cap; ++s) {
    row_ptr[s] = (uint32_t)o;
    if (!m->nodes[s].present) continue;
    memcpy(cols + o, m->nodes[s].nb, m->nodes[s].nn * sizeof(uint32_t));
    qsort(cols + o, m->nodes[s].nn, sizeof(uint32_t), u32cmp);
    o += m->nodes[s].nn;
  }
  row_ptr[m->cap] = (uint32_t)o;
  return (int64_t)o;
}

/* Structural invariants: lists sorted and doubly linked over exactly the present nodes, all marks 0,
 * neighbour sets symmetric and free of duplicates. Returns 0 if all hold, else a code. */
int xz_check_invariants(xz_mgr* m) {
  uint32_t npresent = 0;
  for (uint32_t s = 0; s < m->cap; ++s) {
    if (!m->nodes[s].present) continue;
    npresent++;
    if (m->nodes[s].mark != 0) return 1;
  }
  for (int ax = 0; ax < 2; ++ax) {
    uint32_t cnt = 0;
    int32_t p = *head(m, ax), last = XZ_NIL;
    while (p != XZ_NIL) {
      if (!m->nodes[p].present) return 2;
      if (*prv(N(p), ax) != last) return 3;
      if (last != XZ_NIL && crd(N(last), ax) > crd(N(p), ax)) return 4;
      last = p;
      p = *nxt(N(p), ax);
      if (++cnt > npresent) return 5;
    }
    if (cnt != npresent || *tail(m, ax) != last) return 6;
  }
  for (uint32_t s = 0; s < m->cap; ++s) {
    xz_node* n = N(s);
    if (!n->present) continue;
    for (uint32_t i = 0; i < n->nn; ++i) {
      uint32_t o = n->nb[i];
      if (o == s || !m->nodes[o].present) return 7;
      int found = 0;
      for (uint32_t j = 0; j < m->nodes[o].nn; ++j) found += m->nodes[o].nb[j] == s;
      if (found != 1) return 8;
    }
  }
  return 0;
}
