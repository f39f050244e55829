/*
 * gwaoi_strips.h — one Space partitioned into X-strips over several GPUs (SURVEY.md §8(e), config 4:
 * a 16M-entity open world over the 8 GPUs of a node, halo rows exchanged over RCCL/xGMI).
 *
 * GPU r owns the entities whose START-of-tick x lies in its strip [xa, xb). Its REGION is the strip
 * widened by a halo H = D + max_step + margin on each side: every entity that can share a box with
 * an owned entity during the tick (either position, either perspective) has its start or end x in
 * the region. GPU r runs one gwaoi manager (slot = global entity id) over the region and applies, in
 * global id order, the op of every entity whose start or end x is in the region:
 *     present at the start and at the end  -> Moved
 *     end only (came into the region)      -> Enter
 *     start only (left the region)         -> Leave
 * owned entities loud, halo copies GWAOI_OP_SILENT. The local op order is the global op order, so the
 * events of owned movers are exactly those of one manager running the whole world (each pair event
 * is reported once, by the GPU that owns its mover). Entities that enter or leave the region are more
 * than D away from every owned entity at both ends of the tick (H > D + max_step), so those ops raise
 * no event for an owned mover. Ownership moves with the entity: next tick's owner is the strip of
 * this tick's end x, which already holds the entity as a halo copy — no separate migration message.
 *
 * Per tick: (1) end positions of owned entities (gwaoi_strip_walk: the bench's seeded walk, or
 * gwaoi_strip_ingest: external moves); (2) gwaoi_strip_select: owned entities with start or end x
 * within the neighbours' regions -> two record lists; (3) gwaoi_strip_exchange swaps them with the
 * neighbours over RCCL/xGMI on the GPU's stream (or the host moves them: any transport);
 * (4) gwaoi_strip_absorb[_n] the received lists;
 * (5) gwaoi_strip_emit: the op list in id order + the state advance; (6) gwaoi_stage_ops_device +
 * gwaoi_tick. Host side: goworld_amd/strips.py. All functions enqueue on `stream` (a hipStream_t;
 * NULL = the null stream) and return at once; counts land in device memory.
 *
 * State arrays (device, length g->n): flags (uint8, GWAOI_STRIP_*), sx/sz start-of-tick positions,
 * ex/ez end-of-tick positions. Exchange records are 4 x uint32: {id, x bits, z bits, 0}.
 */
#ifndef GWAOI_STRIPS_H
#define GWAOI_STRIPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GWAOI_STRIP_PRESENT 1u /* in this GPU's manager at the start of the tick */
#define GWAOI_STRIP_OWNED 2u   /* start-of-tick x in this GPU's strip */
#define GWAOI_STRIP_END 4u     /* end-of-tick position known here this tick */

#define GWAOI_STRIP_ERR_STEP 1u     /* an owned entity moved further than max_step in one tick */
#define GWAOI_STRIP_ERR_NOT_OWNED 2u /* ingest named an entity this GPU does not own */
#define GWAOI_STRIP_ERR_OVERFLOW 4u  /* a select list exceeded its capacity */
#define GWAOI_STRIP_ERR_SLOTS 8u     /* local slots: the region holds more entities than cap_l */

typedef struct {
  uint32_t n;       /* global entity count: ids 0..n-1 */
  float xa, xb;     /* own strip: start-of-tick x in [xa, xb) = owned */
  float ra, rb;     /* own region [ra, rb) = [xa - H, xb + H) (initial halo) */
  float left_hi;    /* owned entity goes to the left neighbour if its start or end x < left_hi */
  float right_lo;   /* ... to the right neighbour if its start or end x >= right_lo */
  float max_step;   /* largest |x_end - x_start| of an owned entity the halo width covers */
  int32_t has_left, has_right;
} gwaoi_strip_geom;

/* Tick 0 of the seeded workload (include/gwaoi_workload.h, all n ids): end position of every entity in
 * the region, OWNED for the strip. The first gwaoi_strip_emit then yields the Enter pass. */
int gwaoi_strip_init_walk(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, float* ex, float* ez,
                          uint64_t seed, float L);
/* End positions of the owned entities for tick `tick` of the seeded walk (bench workload). */
int gwaoi_strip_walk(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, const float* sx, const float* sz,
                     float* ex, float* ez, uint64_t seed, uint64_t tick, float L, float step, uint32_t* d_err);
/* End positions of owned entities from external moves (ids, x, z in device memory). */
int gwaoi_strip_ingest(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, const float* sx, float* ex, float* ez,
                       const uint32_t* d_ids, const float* d_x, const float* d_z, uint32_t n, uint32_t* d_err);
/* Owned entities to send: d_left / d_right receive up to `cap` records each; d_counts[0..1] their
 * counts (zeroed here). */
int gwaoi_strip_select(void* stream, const gwaoi_strip_geom* g, const uint8_t* flags, const float* sx,
                       const float* ex, const float* ez, uint32_t* d_left, uint32_t* d_right, uint32_t cap,
                       uint32_t* d_counts, uint32_t* d_err);
/* Received records: end positions of halo entities. */
int gwaoi_strip_absorb(void* stream, uint8_t* flags, float* ex, float* ez, const uint32_t* d_recs, uint32_t n);
/* The tick's op list in id order (ids, x, z, kinds; *d_n_ops = count) and the state advance (flags,
 * start positions) for the next tick. d_scratch: gwaoi_strip_scratch_words(n) words. */
int gwaoi_strip_emit(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, float* sx, float* sz, const float* ex,
                     const float* ez, uint32_t* d_ids, float* d_x, float* d_z, uint8_t* d_kinds, uint32_t* d_scratch,
                     uint32_t* d_n_ops);
size_t gwaoi_strip_scratch_words(uint32_t n);

/* ---- local slots ----
 * The rank's manager can index its entities by a LOCAL slot instead of the global id, so its per-pass
 * work (op apply, grid build) follows the rank's population, not the world's id range (a 16M-id world
 * on 8 GPUs: ~2M present per rank). The op list stays in global id order (that order is what makes
 * the merged events equal one manager's), only the slot the manager sees changes. State (device):
 * g2l[n] (global id -> local slot, GWAOI_STRIP_NO_SLOT = none), l2g[cap_l], a ring of free slots
 * fq[cap_l rounded up to a power of two] (any cap_l >= 1 since ABI 2.1; 2.0 required a power of two, so
 * the manager's capacity, and with it every pass's per-slot work, was up to 2x the slots needed),
 * pend[cap_l] (slots of this tick's Leaves, returned to the ring at
 * the next emit, after the caller has translated the tick's events with l2g) and ctr[4] =
 * {allocations, releases, pending, error bits}. */
#define GWAOI_STRIP_NO_SLOT 0xFFFFFFFFu
int gwaoi_strip_local_init(void* stream, uint32_t n, uint32_t cap_l, uint32_t* g2l, uint32_t* fq, uint32_t* ctr);
/* gwaoi_strip_emit with d_slots = local slots: Enter ops take a free slot, Leave ops queue theirs. When
 * the tick's Enters exceed the free slots, nothing is emitted (*d_n_ops = 0, state not advanced, the
 * manager's pass is empty and it stays usable) and ctr[3] gets GWAOI_STRIP_ERR_SLOTS. */
int gwaoi_strip_emit_local(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, float* sx, float* sz,
                           const float* ex, const float* ez, uint32_t* d_slots, float* d_x, float* d_z,
                           uint8_t* d_kinds, uint32_t* d_scratch, uint32_t* d_n_ops, uint32_t* g2l, uint32_t* l2g,
                           uint32_t* fq, uint32_t* pend, uint32_t cap_l, uint32_t* ctr);
/* Events {mover, other | flags} of a tick from local slots to global ids, in place (n pairs). */
int gwaoi_strip_translate_events(void* stream, const uint32_t* l2g, uint32_t* d_events, uint32_t n);

/* Skewed-crowd variant of gwaoi_strip_init_walk (gww_skew_init_coord). */
int gwaoi_strip_init_skew(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, float* ex, float* ez,
                          uint64_t seed, float L, uint32_t nhot, float sigma, uint32_t hot_every);
/* gwaoi_strip_absorb with the record count in device memory (min(*d_n, n_max) records). A count above
 * n_max (the sender's list was cut at its capacity) sets GWAOI_STRIP_ERR_OVERFLOW in *d_err (if not
 * NULL), so the receiving rank fails its protocol check too. (ABI 2: d_err added.) */
int gwaoi_strip_absorb_n(void* stream, uint8_t* flags, float* ex, float* ez, const uint32_t* d_recs,
                         const uint32_t* d_n, uint32_t n_max, uint32_t* d_err);

/* ---- region state (ABI 2.1) ----
 * The per-tick kernels above index the strip's state by global id and sweep the whole id range (g->n): a
 * 16M-id world on 8 GPUs makes every rank scan 16M ids to find its ~2M, and the ids of one region are spread
 * over the id space, so each 64-byte line of a state array holds about two of them. With a region state the
 * strip's state lives in LOCAL-slot order (the manager's own slots): walk and select sweep the cap_l slots
 * (contiguous), absorb maps the few received ids through g2l (an entity new to the region takes a free slot
 * there), and the emit walks the region list (the last op list: ids ascending, with their slots) merged with
 * the tick's new ids, so the op list stays in global id order. Per tick the work follows the region, and
 * every sweep reads whole lines. Tick 0 (gwaoi_strip_region_start) enters the region's entities from the
 * global-id arrays of gwaoi_strip_init_walk / _init_skew, which are not needed afterwards.
 *   Limits: at most cap_new ids may come into the region, and at most cap_new Leaves leave it, per tick (the
 * halo crossings of one tick: hundreds at the bench sizes); cap_new <= 8 x chunk, chunk <= 16384 (one
 * block's LDS sort per chunk of the tick's new ids or Leaves). Past either limit, or with no free slot for a
 * new id, ctr[6] gets GWAOI_STRIP_ERR_NEWLIST / lctr[3] GWAOI_STRIP_ERR_SLOTS, the emit emits nothing and the
 * region state is no longer consistent: the caller stops the strip (the manager itself stays usable). */
#define GWAOI_STRIP_ERR_NEWLIST 16u /* region state: more than cap_new new ids or Leaves in one tick */
#define GWAOI_STRIP_TOMB 0x80000000u /* region list: the entry left the region (a Leave of the last emit) */
typedef struct {
  uint8_t* flags;     /* [cap_l] GWAOI_STRIP_* per local slot (0: free) */
  float *sx, *sz;     /* [cap_l] start-of-tick positions */
  float *ex, *ez;     /* [cap_l] end-of-tick positions */
  uint32_t* g2l;      /* [n] global id -> local slot (GWAOI_STRIP_NO_SLOT) */
  uint32_t* l2g;      /* [cap_l] local slot -> global id */
  uint32_t* fq;       /* [cap_l rounded up to a power of two] free-slot ring */
  uint32_t* pend;     /* [cap_l] slots of the last emit's Leaves (back to the ring at the next emit) */
  uint32_t* lctr;     /* [4] ring counters, as gwaoi_strip_local_init */
  uint32_t* rl[2];    /* [cap_l] region list (ids ascending, GWAOI_STRIP_TOMB on Leaves), double buffered */
  uint32_t* rs[2];    /* [cap_l] the list entries' slots */
  uint32_t* nw;       /* [2 * cap_new] the tick's new ids, then their slots (absorb appends) */
  uint32_t* lv;       /* [cap_new] list positions of the last emit's Leaves */
  uint32_t* srt;      /* [3 * cap_new] the emit's sorted copies: new ids, their slots, Leave positions */
  uint32_t* ctr;      /* [8] device, per list buffer p: [p] list length, [2 + p] new ids, [4 + p] tombstones;
                         [6] GWAOI_STRIP_ERR_* bits */
  uint32_t* scratch;  /* [gwaoi_strip_scratch_words(n)] (gwaoi_strip_region_start) */
  uint32_t n, cap_l, cap_new, chunk; /* chunk: 0 = 16384, else a power of two in [16, 16384] */
  uint32_t cur;       /* the current list buffer (flipped by gwaoi_strip_region_emit) */
} gwaoi_strip_region;
/* Zero the slot flags and counters, empty g2l and fill the ring (every pointer above allocated) */
int gwaoi_strip_region_init(void* stream, gwaoi_strip_region* R);
/* Tick 0: every entity of the region (global-id arrays flags / ex / ez of gwaoi_strip_init_walk) enters, in
 * id order, taking slots 0, 1, ...; the op list (local slots) and the region list. More than cap_l: nothing
 * emitted (*d_n_ops = 0), lctr[3] |= GWAOI_STRIP_ERR_SLOTS. */
int gwaoi_strip_region_start(void* stream, const gwaoi_strip_geom* g, gwaoi_strip_region* R, const uint8_t* flags,
                             const float* ex, const float* ez, uint32_t* d_slots, float* d_x, float* d_z,
                             uint8_t* d_kinds, uint32_t* d_n_ops);
int gwaoi_strip_region_walk(void* stream, const gwaoi_strip_geom* g, const gwaoi_strip_region* R, uint64_t seed,
                            uint64_t tick, float Lw, float step, uint32_t* d_err);
int gwaoi_strip_region_ingest(void* stream, const gwaoi_strip_geom* g, const gwaoi_strip_region* R,
                              const uint32_t* d_ids, const float* d_x, const float* d_z, uint32_t n, uint32_t* d_err);
int gwaoi_strip_region_select(void* stream, const gwaoi_strip_geom* g, const gwaoi_strip_region* R, uint32_t* d_left,
                              uint32_t* d_right, uint32_t cap, uint32_t* d_counts, uint32_t* d_err);
/* as gwaoi_strip_absorb_n (d_n may be NULL: n_max records) */
int gwaoi_strip_region_absorb(void* stream, const gwaoi_strip_region* R, const uint32_t* d_recs, const uint32_t* d_n,
                              uint32_t n_max, uint32_t* d_err);
/* both neighbours' messages in one launch (either may be empty: n_max 0) */
int gwaoi_strip_region_absorb2(void* stream, const gwaoi_strip_region* R, const uint32_t* d_left, const uint32_t* d_nl,
                               uint32_t nl_max, const uint32_t* d_right, const uint32_t* d_nr, uint32_t nr_max,
                               uint32_t* d_err);
/* The op list (local slots) in global id order, the state advance and the next region list (R->cur flips) */
int gwaoi_strip_region_emit(void* stream, const gwaoi_strip_geom* g, gwaoi_strip_region* R, uint32_t* d_slots,
                            float* d_x, float* d_z, uint8_t* d_kinds, uint32_t* d_n_ops);

/* ---- the halo exchange over RCCL (xGMI), device-resident end to end ----
 * One communicator per strip world, one rank per GPU. Rank 0 makes the id; the caller hands the 128
 * bytes to every rank over whatever channel the deployment has (the game processes' own transport,
 * torch.distributed in goworld_amd/strips.py); then every rank calls gwaoi_strip_comm_init. */
#define GWAOI_STRIP_COMM_ID_BYTES 128 /* ncclUniqueId */
typedef struct gwaoi_strip_comm gwaoi_strip_comm;
int gwaoi_strip_comm_id(uint8_t* id /* [GWAOI_STRIP_COMM_ID_BYTES] */);
int gwaoi_strip_comm_init(const uint8_t* id, int nranks, int rank, int device, gwaoi_strip_comm** out);
int gwaoi_strip_comm_destroy(gwaoi_strip_comm* comm);
/* One tick's exchange, one RCCL group enqueued on `stream`, no host synchronisation: to left_peer the
 * count d_counts[0] and the records d_left[0..cap), from it d_counts_in[0] and d_left_in[0..cap); the
 * same with right_peer, d_counts[1] / d_right / d_counts_in[1] / d_right_in. A peer < 0 means no
 * neighbour on that side (its received count is set to 0). Messages have fixed sizes (cap records of
 * 4 x uint32), so the select lists' counts never travel to the host; absorb with
 * gwaoi_strip_absorb_n(d_left_in, d_counts_in + 0, cap) and (d_right_in, d_counts_in + 1, cap). A
 * peer equal to the caller's own rank is a loopback (send and receive match in issue order). */
int gwaoi_strip_exchange(gwaoi_strip_comm* comm, void* stream, int left_peer, int right_peer, const uint32_t* d_left,
                         const uint32_t* d_right, const uint32_t* d_counts, uint32_t cap, uint32_t* d_left_in,
                         uint32_t* d_right_in, uint32_t* d_counts_in);

#ifdef __cplusplus
}
#endif
#endif /* GWAOI_STRIPS_H */
