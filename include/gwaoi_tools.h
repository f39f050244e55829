/*
 * gwaoi_tools.h — bench / test tooling exported by libgwaoi.so next to the AOI ABI (gwaoi.h).
 * Not part of the drop-in boundary: no reference interface corresponds to these. They let tests and
 * bench.py keep inputs resident in HBM without depending on PyTorch for device memory.
 */
#ifndef GWAOI_TOOLS_H
#define GWAOI_TOOLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int gwaoi_device_count(int* n);
int gwaoi_dev_malloc(int device, size_t bytes, void** out);
int gwaoi_dev_free(int device, void* p);
int gwaoi_dev_htod(int device, void* dst, const void* src, size_t bytes);
int gwaoi_dev_dtoh(int device, void* dst, const void* src, size_t bytes);
int gwaoi_dev_sync(int device);

/* Device generator of include/gwaoi_workload.h (bit-identical to the host functions there).
 * wl_init: positions at tick 0.  wl_step: x_out = step(x_prev) for `tick` (x_out may alias x_prev).
 * wl_iota: d[i] = i. All run on the null stream of `device` and are synchronous. */
int gwaoi_wl_init(int device, float* d_x, float* d_z, uint32_t n, uint64_t seed, float L);
int gwaoi_wl_step(int device, const float* d_xprev, const float* d_zprev, float* d_xout, float* d_zout,
                  uint32_t n, uint64_t seed, uint64_t tick, float L, float s);
int gwaoi_wl_iota(int device, uint32_t* d, uint32_t n);
/* nspaces Spaces of n_per entities (slot = space * n_per + i, Space seed = seed0 + space): placement
 * (nhot > 0: config 5's skewed crowd, gww_skew_init_coord) and one walk step. */
int gwaoi_wl_init_spaces(int device, float* d_x, float* d_z, uint32_t n_per, uint32_t nspaces, uint64_t seed0,
                         float L, uint32_t nhot, float sigma, uint32_t hot_every);
int gwaoi_wl_step_spaces(int device, const float* d_xprev, const float* d_zprev, float* d_xout, float* d_zout,
                         uint32_t n_per, uint32_t nspaces, uint64_t seed0, uint64_t tick, float L, float s);

/* Bench tool: pack n ingest records (include/gwaoi_sync.h, 32 B each: d_ids[i] | x[i], y, z[i], yaw) into
 * d_out, with y = 0 and yaw = tick * 0.01 — the client position stream of one tick, resident in HBM. */
int gwaoi_wl_pack_ingest(int device, const uint8_t* d_ids, const float* d_x, const float* d_z, uint32_t n,
                         uint32_t tick, uint8_t* d_out);
/* Test hook: set the manager's next op sequence number (exercises the sequence renormalisation that
 * otherwise runs every ~2^31 ops). */
struct gwaoi_mgr;
int gwaoi_debug_set_next_seq(struct gwaoi_mgr* mgr, uint32_t next_seq);
/* Test hook: 0 = every mover walks from global memory (k_sweep_dense: the band walk, else its ring),
 * the A/B of the LDS-staged path; 1 = the default (LDS-staged tiles; movers of tiles over the LDS budget
 * walk from global memory). */
int gwaoi_debug_set_sweep_lds(struct gwaoi_mgr* mgr, int enable);
/* Test hook: cell size = D / cells_per_dist for grids built from now on (default 4). */
int gwaoi_debug_set_cells_per_dist(struct gwaoi_mgr* mgr, float cells_per_dist);
/* Test hook: absolute cell side for every Space (0 = back to D / cells_per_dist). */
int gwaoi_debug_set_cell_side(struct gwaoi_mgr* mgr, float side);
/* Diagnostic builds only (GW_STAMPS=1): per-block phase timestamps of the last sweep launch
 * (8 x uint64 per block). Returns GWAOI_ERR_INVALID/-1 in a product build. */
int gwaoi_debug_read_stamps(void* host, size_t bytes);
/* Test hook: the largest entry count the relation view (gwaoi_relation_device) and the sync fan-out
 * (gwaoi_collect_sync) accept before failing with GWAOI_ERR_NOMEM (default and maximum 2^32 - 1: their
 * offsets are uint32). Lowering it exercises the overflow guard without a 2^32-entry workload. */
int gwaoi_debug_set_index_limit(struct gwaoi_mgr* mgr, uint64_t limit);
/* Relation view mode: 0 = update the view from the tick's events when it allows (default), 1 = rebuild
 * it from the grid on every call (even with no pass since the last one: timing); -1 leaves the mode.
 * Reports how many views each path has built, and why the last rebuild was not an update (1 no view
 * yet, 2 mode 1, 3 passes ran outside the event accumulation, 4 SILENT ops, 5 too many events, 6 size
 * bound, 7 a row with too many changes, 8 inconsistent size). */
int gwaoi_debug_set_relation_mode(struct gwaoi_mgr* mgr, int mode, uint64_t* n_incremental, uint64_t* n_full,
                                  int* last_rebuild_reason);
/* Test hook: small passes (a pass with few ops is judged against the last full build's grid plus an
 * overlay of the slots with ops since, without rebuilding the grid). mode 0 = off, 1 = auto (default),
 * 2 = whenever the overlay has room; < 0 leaves the mode. *n_small (optional): small passes run. */
int gwaoi_debug_set_small_pass(struct gwaoi_mgr* mgr, int mode, uint64_t* n_small);
/* Grid build mode: 0 = the one-pass tile build whenever the previous tile build's starts fit the grid
 * (default; a pass whose plan overflows is re-run with the counting build), 1 = always the counting
 * build; -1 leaves the mode. Reports the builds of each kind and the re-runs since the manager was made. */
int gwaoi_debug_set_build_mode(struct gwaoi_mgr* mgr, int mode, uint64_t* n_fused, uint64_t* n_counting,
                               uint64_t* n_reruns);
/* The band walk of the global-memory movers (k_sweep_dense): 1 = on (default: per pass that
 * walks from global memory, the grid's records are sorted per cell by search key and each ordinary move
 * reads only the key windows of the two boxes' symmetric difference), 0 = off (every such mover reads its
 * whole ring of cells), 2 = the same as 1 (there is no per-mover cost model any more: every mover with a
 * band plan takes the band walk); -1 leaves the mode. *n_band_movers (optional): movers that took the band walk
 * since the manager was made. */
int gwaoi_debug_set_band(struct gwaoi_mgr* mgr, int mode, uint64_t* n_band_movers);
/* Sync fan-out path (gwaoi_collect_sync): 0 = the records written straight into their gate packets when
 * n_gates <= 8 (default), 1 = always the pair list + gate partition; -1 leaves the mode. *direct_reruns
 * (optional): direct collects whose packet buffer was too small and were written again. Requires
 * gwaoi_sync_enable. */
int gwaoi_debug_set_fanout_mode(struct gwaoi_mgr* mgr, int mode, uint64_t* direct_reruns);
/* Count the tiles the LDS sweeps walked, per sweep size: tiles[0] small, [1] mid, [2] big,
 * accumulated over the passes since counting was enabled (enable 1: start, or keep, counting; 0: read and
 * stop; -1: read). One atomic per tile when on; the product path does not count. */
int gwaoi_debug_sweep_sizes(struct gwaoi_mgr* mgr, int enable, uint64_t* tiles);
/* Diagnostics: resident sweep workgroups per CU (HIP occupancy API) and the sweep's LDS bytes. */
int gwaoi_debug_sweep_occupancy(int device, int* blocks_per_cu, int* lds_bytes);

#ifdef __cplusplus
}
#endif
#endif /* GWAOI_TOOLS_H */
