/*
 * gwaoi.h — C ABI of the MI355X-native, tick-batched AOI engine (libgwaoi.so).
 *
 * This is the drop-in boundary for GoWorld's AOI hot path. In the reference the path is the
 * go-aoi v0.2.0 (rev 5e9d879, /root/reference/Gopkg.lock:155-159) interface
 *
 *     type AOIManager interface { Enter(aoi *AOI, x, y Coord); Leave(aoi *AOI); Moved(aoi *AOI, x, y Coord) }
 *     func NewXZListAOIManager(aoidist Coord) AOIManager
 *     type AOICallback interface { OnEnterAOI(other *AOI); OnLeaveAOI(other *AOI) }
 *
 * held by engine/entity/Space.go:33, constructed at Space.go:105 and called at Space.go:211,221,243,259;
 * the callbacks are implemented by *Entity at engine/entity/Entity.go:227-233. Each entry point below
 * names the reference call it replaces.
 *
 * Contract (mirrors the reference's):
 *   - Identity is a dense uint32 "slot" (cgo may not retain Go pointers); the Go side keeps slot -> *AOI.
 *   - One manager is driven by one thread at a time (GameService main goroutine, GameService.go:88-192).
 *   - No exceptions cross the ABI: every function returns GWAOI_OK (0) or a negative GWAOI_ERR_* code;
 *     gwaoi_last_error() gives a message (thread-local). Misuse the reference would panic on
 *     (Enter twice, Leave/Moved of an absent AOI) is reported as GWAOI_ERR_STATE instead.
 *   - Ops are STAGED and applied by gwaoi_tick() in staging order. The events returned are exactly the
 *     pair events the reference would have raised by running the same calls one by one:
 *       Enter(m)  -> ENTER(m,o) for every present o inside m's box,
 *       Leave(m)  -> LEAVE(m,o) for every current neighbour o,
 *       Moved(m)  -> LEAVE(m,o) for neighbours now outside m's new box, ENTER(m,o) for new ones,
 *     where "o inside m's box" is the go-aoi float32 predicate
 *       fl32(m.x-D) <= o.x <= fl32(m.x+D)  &&  fl32(m.z-D) <= o.z <= fl32(m.z+D).
 *     Each pair event stands for the two reference callbacks m.OnXAOI(o) then o.OnXAOI(m).
 *     Staging a slot that already has an op in the current batch first flushes the batch (a
 *     "sub-tick"), so the sequential semantics hold for ANY call sequence.
 *   - Events are ordered canonically: by staging order of the mover, then LEAVE before ENTER, then
 *     other-slot ascending. Replaying them in this order reproduces a valid sequential execution of the
 *     reference (the reference's own order inside one Moved follows Go map iteration, i.e. is random).
 */
#ifndef GWAOI_H
#define GWAOI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GWAOI_OK 0
#define GWAOI_ERR_INVALID (-1)  /* bad argument (null pointer, slot >= capacity, bad space id, dist <= 0) */
#define GWAOI_ERR_STATE (-2)    /* Enter of a present slot, Leave/Moved of an absent slot */
#define GWAOI_ERR_HIP (-3)      /* HIP runtime failure (no GPU, launch failure, ...) */
#define GWAOI_ERR_NOMEM (-4)    /* device or pinned host allocation failed */
#define GWAOI_ERR_DEVICE_CHECK (-5) /* device-staged batch failed validation (duplicate / absent slot) */

#define GWAOI_EV_ENTER 0x80000000u /* bit 31 of gwaoi_event.other: 1 = ENTER, 0 = LEAVE */
#define GWAOI_EV_SLOT_MASK 0x7fffffffu

typedef struct gwaoi_mgr gwaoi_mgr;

/* One pair event: the reference's mover.OnXAOI(other); other.OnXAOI(mover). 8 bytes. */
typedef struct {
  uint32_t mover; /* slot whose Enter/Leave/Moved raised the event */
  uint32_t other; /* other slot | GWAOI_EV_ENTER for enter events */
} gwaoi_event;

/* Events of one gwaoi_tick(). `events` points into memory owned by the manager (host-pinned, or
 * device memory with GWAOI_TICK_DEVICE_EVENTS), valid until the next gwaoi_tick*/ /* call. */
typedef struct {
  const gwaoi_event* events;
  uint64_t count;
  uint64_t n_enter;
  uint64_t n_leave;
  uint32_t n_subticks; /* device pipeline passes this tick ran (>1 when a slot was staged twice) */
  uint32_t n_ops;      /* ops applied */
} gwaoi_events;

/* One AOI Space inside a manager. A manager may batch many independent Spaces. */
typedef struct {
  float dist;                 /* AOI distance D of the Space (Space.EnableAOI(d), Space.go:91-105) */
  float min_x, min_z;         /* grid extent hint. Correctness never depends on it: entities outside */
  float max_x, max_z;         /* are clamped into edge cells (only slower). min >= max => auto extent. */
} gwaoi_space_desc;

/* Replaces aoi.NewXZListAOIManager(aoidist) (Space.go:105) for one Space. capacity = max slot + 1
 * (1 .. 2^30 - 1). */
int gwaoi_create(float dist, uint32_t capacity, int device, gwaoi_mgr** out);
/* Many Spaces in one manager (one pipeline pass per tick for all of them). */
int gwaoi_create_spaces(const gwaoi_space_desc* spaces, uint32_t nspaces, uint32_t capacity, int device,
                        gwaoi_mgr** out);
int gwaoi_destroy(gwaoi_mgr* mgr);

/* Run the manager's work on a caller-owned hipStream_t (e.g. torch.cuda.current_stream().cuda_stream).
 * NULL restores the manager's own stream. */
int gwaoi_set_stream(gwaoi_mgr* mgr, void* hip_stream);

/* XZListAOIManager.Enter(aoi, x, z)  <- Space.enter (Space.go:211,221). Staged. */
int gwaoi_enter(gwaoi_mgr* mgr, uint32_t slot, float x, float z);
int gwaoi_enter_space(gwaoi_mgr* mgr, uint32_t space, uint32_t slot, float x, float z);
/* n Enter calls in array order into one Space (bulk load: EntityManager.RestoreFreezedEntities ->
 * restoreEntity -> Space.enter(isRestore) -> aoiMgr.Enter, EntityManager.go:591-652, Space.go:218-223). */
int gwaoi_stage_enters(gwaoi_mgr* mgr, uint32_t space, const uint32_t* slots, const float* x, const float* z,
                       uint32_t n);
/* XZListAOIManager.Leave(aoi)  <- Space.leave (Space.go:243). Staged. */
int gwaoi_leave(gwaoi_mgr* mgr, uint32_t slot);
/* XZListAOIManager.Moved(aoi, x, z)  <- Space.move (Space.go:259). Staged. */
int gwaoi_moved(gwaoi_mgr* mgr, uint32_t slot, float x, float z);
/* n Moved calls in array order (GameService.HandleSyncPositionYawFromClient loop, GameService.go:398-410). */
int gwaoi_stage_moves(gwaoi_mgr* mgr, const uint32_t* slots, const float* x, const float* z, uint32_t n);
/* Zero-copy variant for the cgo wrapper's per-tick flush (replaces the copy-in of gwaoi_stage_moves).
 * gwaoi_stage_buffers returns three library-owned pinned host arrays of `*capacity` entries (allocated on
 * the first call, owned by the manager, the same arrays every call); the caller writes n Moved calls
 * into them (Go: unsafe.Slice over the C pointers) and calls gwaoi_stage_moves_pinned(mgr, n). That
 * call copies the arrays to the device once and validates them THERE (slot range, slot in a Space,
 * finite coordinates: GWAOI_ERR_INVALID / GWAOI_ERR_STATE with nothing staged, as gwaoi_stage_moves);
 * a slot that repeats splits the batch into sub-passes on the device's report, exactly as
 * gwaoi_stage_moves does. Ops staged before it run first. When it returns, the buffers may be
 * rewritten. */
int gwaoi_stage_buffers(gwaoi_mgr* mgr, uint32_t** slots, float** x, float** z, uint32_t* capacity);
int gwaoi_stage_moves_pinned(gwaoi_mgr* mgr, uint32_t n);
/* ABI 2.1. Incremental push for a wrapper whose Moved calls arrive over the tick (GameService.go:398-410
 * handles one position packet at a time): entries [pushed, upto) of the pinned arrays are copied to the
 * device NOW (asynchronous DMA; nothing validated, nothing staged), so the final
 * gwaoi_stage_moves_pinned[_async](n) copies only entries [upto, n). Entries below `upto` must not be
 * rewritten before that call; `upto` never decreases within a batch (GWAOI_ERR_INVALID). Ops staged before
 * it run first, as at the final call; a pass of host-staged ops in between discards what was pushed (the
 * final call copies it again). */
int gwaoi_stage_moves_pinned_partial(gwaoi_mgr* mgr, uint32_t upto);
/* ABI 2.1. gwaoi_stage_moves_pinned without the host round trip: the copy, the device checks and the
 * repeat search are enqueued and the batch is staged at once; the pass that runs it (gwaoi_tick, or any
 * call that flushes staged ops) applies none of it if the checks refused it and then returns
 * GWAOI_ERR_INVALID / GWAOI_ERR_STATE (what gwaoi_stage_moves_pinned would have returned; the manager
 * stays usable). A repeated slot splits the batch into sub-passes exactly as gwaoi_stage_moves_pinned
 * does. When it returns, the buffers may be rewritten. */
int gwaoi_stage_moves_pinned_async(gwaoi_mgr* mgr, uint32_t n);
/* Same, from DEVICE arrays (inputs resident in HBM). Must be the only ops of the batch; slots must be
 * distinct and present — checked on the device, reported by gwaoi_tick as GWAOI_ERR_DEVICE_CHECK
 * (the manager is then unusable and must be destroyed). The arrays must stay valid until gwaoi_tick. */
int gwaoi_stage_moves_device(gwaoi_mgr* mgr, const uint32_t* d_slots, const float* d_x, const float* d_z,
                             uint32_t n);

/* Mixed Enter/Leave/Moved batch from DEVICE arrays: kinds[i] is GWAOI_OP_MOVE, GWAOI_OP_ENTER (into
 * Space 0) or GWAOI_OP_LEAVE, optionally | GWAOI_OP_SILENT: the op is applied (it changes the relation
 * and is seen by every later op) but none of its own mover's events are emitted. SILENT is how a
 * GPU holding a halo copy of an entity owned by another GPU applies that entity's op without
 * reporting its events twice (X-strip partition, include/gwaoi_strips.h). Validated on the device
 * (Enter of a present slot, Moved/Leave of an absent one, a slot twice -> GWAOI_ERR_DEVICE_CHECK).
 * A manager that has taken a mixed device batch keeps its presence state on the device only: the
 * host-staged calls above then return GWAOI_ERR_STATE. */
#define GWAOI_OP_MOVE 0u
#define GWAOI_OP_ENTER 1u
#define GWAOI_OP_LEAVE 2u
#define GWAOI_OP_SILENT 0x80u
int gwaoi_stage_ops_device(gwaoi_mgr* mgr, const uint32_t* d_slots, const float* d_x, const float* d_z,
                           const uint8_t* d_kinds, uint32_t n);
/* The same with the Space of each Enter: d_spaces[i] (checked < the manager's Space count; a bad id
 * fails the batch like the checks above). d_spaces may be null (every Enter into Space 0). This is
 * the bulk restore of a multi-Space manager from HBM (one pass with S0 empty);
 * with GWAOI_OP_SILENT on every op it rebuilds the relation without reporting the pairs. */
int gwaoi_stage_ops_device_spaces(gwaoi_mgr* mgr, const uint32_t* d_slots, const float* d_x, const float* d_z,
                                  const uint8_t* d_kinds, const uint32_t* d_spaces, uint32_t n);
/* The same with the op count in device memory: the batch is the first *d_n ops (read on the
 * device when the pass runs; must be <= n_max, the bound the kernels are launched for). A batch
 * produced on the GPU (X-strip op lists, GPU-decoded position records) goes in without the host
 * waiting for its size; gwaoi_events.n_ops reports the count. */
int gwaoi_stage_ops_device_n(gwaoi_mgr* mgr, const uint32_t* d_slots, const float* d_x, const float* d_z,
                             const uint8_t* d_kinds, const uint32_t* d_spaces, const uint32_t* d_n, uint32_t n_max);

/* After mixed device batches (e.g. a silent bulk restore from HBM, EntityManager.go:591-652): pull the
 * presence state back into the host mirror so the host-staged calls above are accepted again. No op may
 * be staged. Auto-extent Spaces do not see the adopted coordinates (give restored Spaces extents). */
int gwaoi_adopt_device_state(gwaoi_mgr* mgr);

/* Planning hint: about `expected` entities will be present in Space `space` (default: capacity / number
 * of Spaces). The cell size of a Space with a declared extent is planned from its density; a manager
 * whose slot space is larger than its population (an X-strip rank whose slots are the whole world's
 * ids, include/gwaoi_strips.h) should say so, or its cells come out too fine for the LDS sweep.
 * Correctness never depends on it; takes effect at the next pass. 0 restores the default. */
int gwaoi_set_population_hint(gwaoi_mgr* mgr, uint32_t space, uint32_t expected);

/* Apply every staged op; blocks until the events are on the host (or in device memory, see flags). */
#define GWAOI_TICK_DEVICE_EVENTS 1u /* leave events in device memory (no D2H copy) */
int gwaoi_tick(gwaoi_mgr* mgr, gwaoi_events* out);
int gwaoi_tick_ex(gwaoi_mgr* mgr, uint32_t flags, gwaoi_events* out);

/* Number of present slots / staged ops. */
int gwaoi_count(const gwaoi_mgr* mgr, uint32_t* n_present, uint32_t* n_staged);

/* Export the current relation N (the union of every entity's InterestedIn set, Entity.go:53) as CSR
 * over slots: row_ptr has capacity+1 entries, cols[row_ptr[s] .. row_ptr[s+1]) = neighbours of s in
 * ascending slot order. Pending ops are flushed first (their events are discarded: call gwaoi_tick
 * first if you need them). If cols_cap is too small, *nnz is set and GWAOI_ERR_INVALID returned. */
int gwaoi_export_relation(gwaoi_mgr* mgr, uint32_t* row_ptr, uint32_t* cols, uint64_t cols_cap,
                          uint64_t* nnz);

/* The relation's NET changes over the last gwaoi_tick, for a consumer that keeps its own copy of the
 * sets (Entity.InterestedIn / InterestedBy, Entity.go:53-54, read at Entity.go:1241 and
 * examples/unity_demo/Monster.go:50,79,89) and patches it instead of re-exporting the whole relation
 * or replaying every event into maps. One entry per changed pair and direction: {mover = row,
 * other = col | GWAOI_EV_ENTER} when col joined row's set, {row, col} when it left. Pairs that entered
 * and left within the tick are omitted. Entries come in pairs (row a col b, then row b col a), in the
 * order of each pair's last event. Cost O(events): computed on the GPU from the tick's events (still
 * in HBM), copied into `out` (host, `cap` entries). Call after gwaoi_tick and before the next call
 * that runs a pass (else GWAOI_ERR_STATE), and not after a tick with SILENT ops. If cap is too small,
 * *n is set and GWAOI_ERR_INVALID returned. (ABI 2.) */
int gwaoi_export_relation_delta(gwaoi_mgr* mgr, gwaoi_event* out, uint64_t cap, uint64_t* n);

/* The same relation as a device-resident CSR view (the replay sink's neighbour sets,
 * Entity.InterestedIn / InterestedBy, Entity.go:53-54,236-246, which under the XZ manager are one
 * symmetric set per entity). row_ptr[capacity + 1] and cols[nnz] are HBM buffers owned by the manager
 * (rows in ascending slot order), built on the manager's stream and valid until the next call that
 * runs a pass. Pending ops are flushed first, as in gwaoi_export_relation. */
typedef struct {
  const uint32_t* row_ptr;
  const uint32_t* cols;
  uint64_t nnz;
} gwaoi_relation_view;
int gwaoi_relation_device(gwaoi_mgr* mgr, gwaoi_relation_view* out);

/* Per-stage device time of the pipeline, accumulated over ticks while timing is enabled (hipEvents on
 * the manager's stream). */
typedef struct {
  uint64_t ticks;          /* pipeline passes timed */
  double ms_apply;         /* op application + per-slot bookkeeping */
  double ms_grid;          /* cell binning + counting sort (count, scan, scatter) */
  double ms_sweep;         /* neighbour sweep + event emission (the dominant kernel) */
  double ms_order;         /* canonical event ordering (scan, place, slice sort) */
  double ms_total;         /* first to last kernel of the pass */
  uint64_t sweep_movers;   /* movers processed by the sweep */
  uint64_t events;         /* events emitted */
  uint64_t grid_records;   /* records of the passes' cell-sorted grids (main + ghost) */
  uint64_t grid_cells;     /* cells of those grids */
  uint64_t dense_movers;   /* movers swept one wave each (boxes beyond their tile's LDS region) */
  union {                  /* of the dense movers, those that took the band walk; this was
                              * the reserved refined_cells word of ABI 2 (always 0 there): same layout */
    uint64_t band_movers;
    uint64_t chunked_movers; /* deprecated alias (ABI 2.0 round 4 name) */
  };
} gwaoi_stats;
int gwaoi_set_timing(gwaoi_mgr* mgr, int enable);
int gwaoi_get_stats(const gwaoi_mgr* mgr, gwaoi_stats* out);
int gwaoi_reset_stats(gwaoi_mgr* mgr);

/* Library version string and the thread-local message of the last failing call. */
const char* gwaoi_version(void);
/* ABI revision of the headers the library was built from. A binding compiled against these headers
 * checks gwaoi_abi_version() == GWAOI_ABI_VERSION once at start-up: a struct that grew
 * (e.g. gwaoi_ingest_result.n_nonfinite, ABI 2) would otherwise be written past its end.
 *   1: round-1 surface;  2: gwaoi_ingest_result.n_nonfinite, gwaoi_strip_absorb_n's d_err,
 *   gwaoi_stage_buffers / gwaoi_stage_moves_pinned, gwaoi_export_relation_delta.
 * Minor revisions add calls and keep every struct layout (a binding of 2.0 runs against 2.1):
 *   2.1: gwaoi_stage_moves_pinned_partial, gwaoi_stage_moves_pinned_async, gwaoi_abi_minor;
 *        gwaoi_stats.band_movers is the round-4 name chunked_movers (kept as an alias, same word);
 *        gwaoi_tools.h: gwaoi_debug_set_chunked (removed in 2.0's last revision) is replaced by
 *        gwaoi_debug_set_band (mode, out counter), a test hook outside the ABI proper. */
#define GWAOI_ABI_VERSION 2
#define GWAOI_ABI_MINOR 1
int gwaoi_abi_version(void);
int gwaoi_abi_minor(void);
const char* gwaoi_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* GWAOI_H */
