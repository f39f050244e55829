/*
 * abi_smoke.c — drives libgwaoi through its C ABI (include/gwaoi.h) in the call order of the Go
 * wrapper in INTEGRATION.md §2, from plain C (gcc, no C++ and no HIP headers): the boundary a cgo
 * binding links against.
 *
 *   Enter      -> gwaoi_enter, then Flush (SyncEnterLeave: the callbacks fire inside Space.enter,
 *                 /root/reference/engine/entity/Space.go:211-217)
 *   Moved      -> written into the manager's pinned staging arrays (gwaoi_stage_buffers); every 16 calls
 *                 the filled part is pushed early (gwaoi_stage_moves_pinned_partial, ABI 2.1) and Flush
 *                 pushes the rest with ONE gwaoi_stage_moves_pinned_async call (checked on the device, the
 *                 verdict read by gwaoi_tick). The scenario runs again with the synchronous
 *                 gwaoi_stage_moves_pinned, and with host slices and ONE gwaoi_stage_moves call (copy-in).
 *   Flush      -> push the pending moves + gwaoi_tick, events replayed in order
 *   Leave      -> pending moves first (call order), gwaoi_leave, then Flush
 *
 * Every tick's events are checked against a brute-force sequential model of the reference
 * semantics (per op, the mover's float32 box test against every present entity,
 * LEAVE/ENTER where the pair state changes), including a slot moved twice in one tick. Test
 * infrastructure: exit status 0 = pass. Built by __graft_entry__.build() / tests/test_abi.py, run on
 * the GPU box by tests/test_integration.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gwaoi.h"
#include "gwaoi_tools.h"

#define CAP 96
#define D 100.0f

static float px[CAP], pz[CAP];
static int present[CAP];
static uint8_t rel[CAP][CAP];
static uint32_t want[4 * CAP * CAP][2];
static size_t nwant;

/* the reference predicate: o inside the box of m, bounds fl32(m +- D), inclusive */
static int inbox(int m, int o) {
  const float lx = px[m] - D, hx = px[m] + D, lz = pz[m] - D, hz = pz[m] + D;
  return px[o] >= lx && px[o] <= hx && pz[o] >= lz && pz[o] <= hz;
}

/* one reference call: LEAVE then ENTER events, other slot ascending (the canonical order) */
static void model_op(int kind, int m, float x, float z) { /* kind: 0 move, 1 enter, 2 leave */
  if (kind == 2) {
    present[m] = 0;
  } else {
    px[m] = x;
    pz[m] = z;
    present[m] = 1;
  }
  for (int pass = 0; pass < 2; ++pass)
    for (int o = 0; o < CAP; ++o) {
      if (o == m || !present[o]) continue;
      const int now = kind != 2 && inbox(m, o);
      if (now == rel[m][o]) continue;
      if ((pass == 0 && !now) || (pass == 1 && now)) {
        want[nwant][0] = (uint32_t)m;
        want[nwant][1] = (uint32_t)o | (now ? GWAOI_EV_ENTER : 0u);
        ++nwant;
      }
    }
  for (int o = 0; o < CAP; ++o) {
    if (o == m) continue;
    const int now = kind != 2 && present[o] && inbox(m, o);
    rel[m][o] = rel[o][m] = (uint8_t)now;
  }
}

static gwaoi_mgr* mgr;
static uint32_t host_slot[4 * CAP];
static float host_x[4 * CAP], host_z[4 * CAP];
static uint32_t *pend_slot, pin_cap;
static float *pend_x, *pend_z;
static uint32_t npend;
static int pinned;
static int failures;

#define CHK(call)                                                                        \
  do {                                                                                   \
    int rc_ = (call);                                                                    \
    if (rc_ != GWAOI_OK) {                                                               \
      fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #call, rc_, gwaoi_last_error()); \
      exit(2);                                                                           \
    }                                                                                    \
  } while (0)

static void push(void) {
  if (npend && pinned == 2) CHK(gwaoi_stage_moves_pinned_async(mgr, npend)); /* ABI 2.1: the Go wrapper's push */
  if (npend && pinned == 1) CHK(gwaoi_stage_moves_pinned(mgr, npend));
  if (npend && !pinned) CHK(gwaoi_stage_moves(mgr, pend_slot, pend_x, pend_z, npend));
  npend = 0;
}

static void flush(const char* what) {
  push();
  gwaoi_events ev;
  CHK(gwaoi_tick(mgr, &ev));
  int ok = ev.count == nwant && ev.n_enter + ev.n_leave == ev.count;
  for (size_t i = 0; ok && i < nwant; ++i)
    ok = ev.events[i].mover == want[i][0] && ev.events[i].other == want[i][1];
  if (!ok) {
    fprintf(stderr, "%s: %llu events, expected %zu\n", what, (unsigned long long)ev.count, nwant);
    ++failures;
  }
  nwant = 0;
}

static void enter(uint32_t s, float x, float z) {
  CHK(gwaoi_enter(mgr, s, x, z));
  model_op(1, (int)s, x, z);
  flush("enter");
}

static void moved(uint32_t s, float x, float z) { /* staged on the host side, like the Go wrapper */
  if (npend == pin_cap) push();
  pend_slot[npend] = s;
  pend_x[npend] = x;
  pend_z[npend] = z;
  ++npend;
  if (pinned == 2 && npend % 16 == 0) CHK(gwaoi_stage_moves_pinned_partial(mgr, npend)); /* incremental push */
  model_op(0, (int)s, x, z);
}

static void leave(uint32_t s) {
  push(); /* keep the call order */
  CHK(gwaoi_leave(mgr, s));
  model_op(2, (int)s, 0.f, 0.f);
  flush("leave");
}

static void scenario(int use_pinned) {
  memset(present, 0, sizeof present);
  memset(rel, 0, sizeof rel);
  nwant = npend = 0;
  pinned = use_pinned;
  CHK(gwaoi_create(D, CAP, 0, &mgr));
  if (pinned) {
    CHK(gwaoi_stage_buffers(mgr, &pend_slot, &pend_x, &pend_z, &pin_cap));
    if (pin_cap != CAP) ++failures, fprintf(stderr, "staging capacity %u\n", pin_cap);
  } else {
    pend_slot = host_slot, pend_x = host_x, pend_z = host_z, pin_cap = 4 * CAP;
  }
  /* MySpace.OnSpaceCreated: 10 monsters at the origin (examples/test_game/MySpace.go:27-34) */
  for (uint32_t s = 0; s < 10; ++s) enter(s, 0.f, 0.f);
  /* a crowd on a coarse lattice: exact-D offsets and ties */
  for (uint32_t s = 10; s < 60; ++s) enter(s, (float)((s * 37) % 9) * 50.f - 200.f, (float)((s * 11) % 7) * 50.f - 150.f);
  /* ticks of batched moves, one slot moved twice in a tick (the library splits the batch) */
  uint32_t r = 12345u;
  for (int t = 0; t < 6; ++t) {
    for (uint32_t s = 0; s < 60; ++s) {
      r = r * 1664525u + 1013904223u;
      if ((r >> 28) < 6) continue; /* partial movers */
      const float dx = (float)((int)((r >> 8) % 41) - 20), dz = (float)((int)((r >> 16) % 41) - 20);
      moved(s, px[s] + dx, pz[s] + dz);
    }
    moved(7, px[7] + 1.0f, pz[7]);
    flush("tick");
  }
  leave(3);
  moved(4, 100.0f, 0.0f);
  leave(5); /* flushes moved(4) first */
  enter(3, 0.f, 0.f);
  if (pinned) { /* a refused pinned batch stages nothing (slot 80 is not in a Space) */
    pend_slot[0] = 0, pend_x[0] = 0.f, pend_z[0] = 0.f;
    pend_slot[1] = 80, pend_x[1] = 1.f, pend_z[1] = 1.f;
    if (pinned == 1 && gwaoi_stage_moves_pinned(mgr, 2) != GWAOI_ERR_STATE)
      ++failures, fprintf(stderr, "pinned absent accepted\n");
    if (pinned == 2) { /* async: the pass that reads the device's verdict reports it, nothing applied */
      gwaoi_events e2;
      CHK(gwaoi_stage_moves_pinned_async(mgr, 2));
      if (gwaoi_tick(mgr, &e2) != GWAOI_ERR_STATE) ++failures, fprintf(stderr, "async absent accepted\n");
    }
    flush("refused batch");
  }
  /* misuse is reported, not crashed on: Enter twice, Moved/Leave of an absent slot, NaN */
  if (gwaoi_enter(mgr, 0, 1.f, 1.f) != GWAOI_ERR_STATE) ++failures, fprintf(stderr, "enter twice accepted\n");
  if (gwaoi_moved(mgr, 80, 1.f, 1.f) != GWAOI_ERR_STATE) ++failures, fprintf(stderr, "moved of absent accepted\n");
  if (gwaoi_leave(mgr, 81) != GWAOI_ERR_STATE) ++failures, fprintf(stderr, "leave of absent accepted\n");
  if (gwaoi_moved(mgr, 0, NAN, 1.f) != GWAOI_ERR_INVALID) ++failures, fprintf(stderr, "NaN accepted\n");
  if (gwaoi_enter(mgr, 90, INFINITY, 1.f) != GWAOI_ERR_INVALID) ++failures, fprintf(stderr, "Inf accepted\n");
  uint32_t npres = 0, nst = 0;
  CHK(gwaoi_count(mgr, &npres, &nst));
  if (npres != 59 || nst != 0) ++failures, fprintf(stderr, "count %u staged %u\n", npres, nst);
  CHK(gwaoi_destroy(mgr));
}

int main(void) {
  int ndev = 0;
  if (gwaoi_device_count(&ndev) != GWAOI_OK || ndev < 1) {
    fprintf(stderr, "abi_smoke: no HIP device\n");
    return 3;
  }
  if (gwaoi_abi_version() != GWAOI_ABI_VERSION) {
    fprintf(stderr, "abi_smoke: library ABI %d, headers %d\n", gwaoi_abi_version(), GWAOI_ABI_VERSION);
    return 4;
  }
  scenario(2); /* the Go wrapper of ABI 2.1: async push, incremental pushes */
  scenario(1);
  scenario(0);
  if (failures) {
    fprintf(stderr, "abi_smoke: %d failure(s)\n", failures);
    return 1;
  }
  printf("abi_smoke ok: %s\n", gwaoi_version());
  return 0;
}
