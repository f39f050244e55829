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

/* ---- region lists (ABI 2.1) ----
 * The per-tick kernels above sweep the whole id range (g->n): with a 16M-id world on 8 GPUs every rank
 * scans 16M ids to find its ~2M. With a region list they walk the ids present in the region instead:
 * walk and select over the list, absorb appends the ids that come into the region, and the emit merges the
 * list with the sorted new ids (the op list stays in global id order) and writes the next tick's list. Per
 * tick the work follows the region, not the world. Local slots only (gwaoi_strip_emit_local_list). */
#define GWAOI_STRIP_ERR_NEWLIST 16u /* more ids came into the region in one tick than the list emit takes
                                       (cap_new, at most 16384): nothing emitted; emit by id range instead,
                                       then rebuild the list (gwaoi_strip_list_from_ops) */
typedef struct {
  uint32_t* rl;       /* [cap] ids present in the region at the start of the tick, ascending */
  uint32_t* rl_next;  /* [cap] the next tick's list, written by the emit: the caller swaps rl and rl_next */
  uint32_t* nw;       /* [cap_new] ids that came into the region this tick (absorbed while not present) */
  uint32_t* ctr;      /* [4] device: {list length, emitted, new ids, GWAOI_STRIP_ERR_* bits} */
  uint32_t* scratch;  /* [gwaoi_strip_list_scratch_words(cap)] */
  uint32_t cap;       /* largest region population (the manager's local slot count, cap_l) */
  uint32_t cap_new;   /* new ids per tick at most (<= 16384) */
} gwaoi_strip_list;
size_t gwaoi_strip_list_scratch_words(uint32_t cap);
/* rl_next (and the counters) from a tick's op list, e.g. tick 0's Enter pass or an id-range emit; then swap */
int gwaoi_strip_list_from_ops(void* stream, const gwaoi_strip_list* L, const uint32_t* d_slots, const uint8_t* d_kinds,
                              const uint32_t* l2g, const uint32_t* d_n_ops);
int gwaoi_strip_walk_list(void* stream, const gwaoi_strip_geom* g, const gwaoi_strip_list* L, uint8_t* flags,
                          const float* sx, const float* sz, float* ex, float* ez, uint64_t seed, uint64_t tick,
                          float Lw, float step, uint32_t* d_err);
int gwaoi_strip_select_list(void* stream, const gwaoi_strip_geom* g, const gwaoi_strip_list* L, const uint8_t* flags,
                            const float* sx, const float* ex, const float* ez, uint32_t* d_left, uint32_t* d_right,
                            uint32_t cap, uint32_t* d_counts, uint32_t* d_err);
/* gwaoi_strip_absorb_n (d_n may be NULL: n_max records) that also lists the ids coming into the region */
int gwaoi_strip_absorb_list(void* stream, const gwaoi_strip_list* L, uint8_t* flags, float* ex, float* ez,
                            const uint32_t* d_recs, const uint32_t* d_n, uint32_t n_max, uint32_t* d_err);
/* gwaoi_strip_emit_local over the list: the op list in id order, the state advance and rl_next. With
 * GWAOI_STRIP_ERR_NEWLIST (or no free slots: GWAOI_STRIP_ERR_SLOTS in ctr[3]) nothing is emitted and rl_next
 * is a copy of rl. */
int gwaoi_strip_emit_local_list(void* stream, const gwaoi_strip_geom* g, const gwaoi_strip_list* L, uint8_t* flags,
                                float* sx, float* sz, const float* ex, const float* ez, uint32_t* d_slots, float* d_x,
                                float* d_z, uint8_t* d_kinds, uint32_t* d_n_ops, uint32_t* g2l, uint32_t* l2g,
                                uint32_t* fq, uint32_t* pend, uint32_t cap_l, uint32_t* ctr);

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
