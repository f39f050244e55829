// gwaoi_runtime.hip — host runtime of libgwaoi: manager state, op staging, the per-tick pipeline
// and the C ABI of include/gwaoi.h (the drop-in boundary for go-aoi's AOIManager,
// /root/reference/engine/entity/Space.go:33,105,211,221,243,259).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <limits>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "gwaoi.h"
#include "gwaoi_internal.h"
#include "gwaoi_tools.h"

namespace {

thread_local std::string g_err;

void set_err(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}

#define HIPCHK(x)                                                                               \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      set_err("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_));                   \
      return GWAOI_ERR_HIP;                                                                     \
    }                                                                                           \
  } while (0)

#define RCHK(x)              \
  do {                       \
    int r_ = (x);            \
    if (r_ != GWAOI_OK) return r_; \
  } while (0)

constexpr uint32_t kSeqLimit = 0x7ff00000u;  // renormalise seqs before they pass this
constexpr uint32_t kSlabIdleViews = 8;       // incremental relation views in a row before the slab is freed
#ifndef GW_CELLS_PER_SLOT
#define GW_CELLS_PER_SLOT 3  // grid cell budget per slot of capacity (cells beyond it coarsen the grid)
#endif

template <class T>
int dalloc(T** p, size_t n) {
  *p = nullptr;
  if (!n) n = 1;
  hipError_t e = hipMalloc((void**)p, n * sizeof(T));
  if (e != hipSuccess) {
    set_err("hipMalloc(%zu bytes): %s", n * sizeof(T), hipGetErrorString(e));
    *p = nullptr;
    return GWAOI_ERR_NOMEM;
  }
  return GWAOI_OK;
}

template <class T>
int halloc(T** p, size_t n) {
  *p = nullptr;
  if (!n) n = 1;
  hipError_t e = hipHostMalloc((void**)p, n * sizeof(T), hipHostMallocDefault);
  if (e != hipSuccess) {
    set_err("hipHostMalloc(%zu bytes): %s", n * sizeof(T), hipGetErrorString(e));
    *p = nullptr;
    return GWAOI_ERR_NOMEM;
  }
  return GWAOI_OK;
}

struct SpaceHost {
  gwaoi_space_desc desc;
  bool auto_extent;
  uint32_t pop_hint = 0;  // gwaoi_set_population_hint (0: capacity / nspaces)
  // auto-extent tracking (host-staged coordinates)
  float seen_minx, seen_minz, seen_maxx, seen_maxz;
  bool seen_any;
  // extent the current geometry covers
  float gx0, gz0, gx1, gz1;
};

struct Grid {  // one pass's cell-sorted records (two buffers, alternating between passes)
  gw::Rec* rec = nullptr;
  uint32_t* cs = nullptr;
  gw::Geom* d_geom = nullptr;
  uint32_t* d_tile_space = nullptr;  // tile -> space
  std::vector<gw::Geom> h_geom;  // what d_geom holds
  uint32_t ncells = 0;
  uint32_t ntiles = 0;
  uint32_t cs_zeroed = 0;  // leading cs words known to be zero (zeroed by the previous pass's k_place)
};

}  // namespace

struct gwaoi_mgr {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  uint32_t cap = 0;
  uint32_t nspaces = 0;
  std::vector<SpaceHost> spaces;
  float cells_per_dist = 4.0f;
  float cell_side = 0.0f;  // > 0: absolute cell side for every Space (test hook), else D / cells_per_dist
  bool density_cells = true;  // finer cells for crowded large-D Spaces (compute_geometry); off once a hook sets the size
  uint32_t max_cells = 0;
  bool broken = false;

  // ---- host mirror of the staged state ----
  std::vector<uint8_t> h_present;
  std::vector<uint32_t> h_space_of;
  std::vector<uint32_t> h_stamp;  // pass id the slot was staged in
  uint32_t pass_id = 1;           // id of the pass being staged
  uint32_t n_present = 0;         // after staged ops
  uint32_t n_present_dev = 0;     // after the last executed pass

  // ---- staged ops (pinned) ----
  uint32_t* h_op_slot = nullptr;
  float* h_op_x = nullptr;
  float* h_op_z = nullptr;
  uint8_t* h_op_kind = nullptr;
  uint32_t* h_op_space = nullptr;
  uint32_t* h_leaves = nullptr;
  // device addresses of the pinned op arrays (small passes read them over PCIe instead of copying them);
  // null when the runtime gives none
  const uint32_t* hd_op_slot = nullptr;
  const float* hd_op_x = nullptr;
  const float* hd_op_z = nullptr;
  const uint8_t* hd_op_kind = nullptr;
  const uint32_t* hd_op_space = nullptr;
  uint32_t n_ops = 0, n_leaves = 0;
  bool geom_dirty = true;
  // device-staged batch
  const uint32_t* dv_slot = nullptr;
  const float* dv_x = nullptr;
  const float* dv_z = nullptr;
  const uint8_t* dv_kind = nullptr;  // mixed device batch (gwaoi_stage_ops_device), else null
  const uint32_t* dv_space = nullptr;  // Space of each device Enter (null: Space 0)
  const uint32_t* dv_count = nullptr;  // device-counted batch: *dv_count ops (dv_n = the bound)
  uint32_t dv_n = 0;
  bool dev_managed = false;          // presence lives on the device only (mixed device batches)

  // ---- device state ----
  float *pos_x = nullptr, *pos_z = nullptr, *old_x = nullptr, *old_z = nullptr;
  uint32_t *seq = nullptr, *space_of = nullptr, *old_seq = nullptr, *opq = nullptr;
  uint32_t *key_of = nullptr, *local_of = nullptr;
  uint32_t *d_op_slot = nullptr, *d_op_space = nullptr, *d_leaves = nullptr, *d_dense = nullptr;
  // relation view (gwaoi_relation_device): CSR in HBM, allocated on first use, grown on demand
  uint32_t *rel_rp = nullptr, *rel_cols = nullptr, *rel_tmp = nullptr;
  uint64_t rel_cap = 0, rel_tmp_cap = 0;  // capacities of rel_cols / rel_tmp (swapped by the incremental path)
  // incremental view (relation_delta): the view is valid for the state after pass `rel_passes`
  uint32_t *rel_rp2 = nullptr, *rel_dn = nullptr, *rel_dcur = nullptr, *rel_dch = nullptr, *rel_flag = nullptr;  // rel_dcur, rel_flag: inside rel_dn's allocation
  uint64_t rel_dch_cap = 0;  // changes rel_dch (and its row array behind it) hold
  bool rel_valid = false;
  uint64_t rel_passes = 0, rel_nnz = 0;
  int rel_mode = 0;  // 0: incremental when possible, 1: always rebuild from the grid (gwaoi_debug_set_relation_mode)
  uint64_t rel_stat_incr = 0, rel_stat_full = 0;
  int rel_why = 0;  // why the last view was rebuilt (gwaoi_debug_set_relation_mode)
  unsigned long long* rel_tot = nullptr;  // device: [0] the count pass's 64-bit entry total, [1] longest row
  uint4* rel_tstat = nullptr;              // device: the count pass's per-tile totals
  uint32_t* rel_slab = nullptr;           // count pass output: the rows by grid record (k_row_sort_slab)
  bool rel_no_slab = false;               // no room for the slab at the last rebuild: the two-walk path
  uint64_t rel_slab_recs = 0;             // grid records the slab holds rows for
  uint32_t rel_incr_streak = 0;           // views updated incrementally in a row (the slab is freed after a few)
  uint4* rel_fix = nullptr;               // rows longer than the slab sort's network (2 x cap entries)
  uint64_t index_limit = 0xFFFFFFFFull;   // uint32-indexed outputs (relation view, fan-out) fail above it
  float *d_op_x = nullptr, *d_op_z = nullptr;
  uint8_t* d_op_kind = nullptr;
  Grid grid[2];
  int cur = 0;  // grid holding the current state
  uint32_t next_seq = 1;
  uint32_t* rank_cnt = nullptr;  // [cap + 1]
  uint32_t* uns = nullptr;       // [cap / 32 + 2]: ops whose events are out of canonical order (zero between passes)
  int sweep_lds = 1;             // 0: global-memory sweep path only (A/B)
  uint32_t* part = nullptr;     // scan chunk sums
  uint32_t part_words = 0;
  gw::ScanCtx scan;
  uint32_t* thist = nullptr;     // tile-bucketed build: [max tiles * nblk + 1]
  uint32_t* ttot = nullptr;      // tile totals, two buffers of kMaxLdsTiles: a build sums into one and zeroes the other
  int ttot_sel = 0;              // the buffer the next tile build sums into
  uint32_t* tstart = nullptr;    // tile starts, two buffers of kMaxLdsTiles + 1 (with ttot_sel): this build's, and
                                 // the previous tile build's (the one-pass build's bucket plan)
  int build_mode = 0;            // gwaoi_debug_set_build_mode: 1 = always the counting build
  bool plan_ok = false;          // the previous tile build's starts describe a grid of the geometry in plan_geom
  std::vector<gw::Geom> plan_geom;
  uint64_t builds_fused = 0, builds_counting = 0, build_reruns = 0, dense_reruns = 0;
  uint32_t* tile_walk = nullptr; // tile-bucketed build: per tile of the pass's grid, holds a reported mover
  uint32_t* tile_acted = nullptr;  // per tile: slots of the pass's ops (k_bin_tsort; duplicate-slot check)
  bool rerun_counting = false;   // the previous pass re-ran its build: this one uses the counting build
  // the band walk of k_sweep_dense: the grid's records sorted per cell by search key, built
  // after the grid of every pass that launches k_sweep_dense (gwaoi_debug_set_band: 0 off)
  bool big_sweep = true;  // Spaces over the small LDS sweep's region budget take the big one (debug_set_sweep_lds 3: off)
  int band_mode = 1;  // 0 off, 1 (or 2) on: every mover with a band plan
  float *band_xk = nullptr, *band_zk = nullptr;
  uint32_t* band_zi = nullptr;
  uint32_t* band_hd = nullptr;   // [2 nspaces]
  uint32_t* band_dense2 = nullptr;  // [cap] the dense movers the band walk leaves to the ring walk
  uint64_t band_cap = 0;         // records the arrays hold (0: not allocated)
  uint8_t* band_tab = nullptr;   // key tables (BandArgs.tab): 2 x band_tab_half bytes, or null
  uint32_t band_tab_half = 0;
  uint64_t band_builds = 0, band_movers = 0;
  uint32_t* d_size_tiles = nullptr;  // [3] gwaoi_debug_sweep_sizes (null: not counted)
  uint32_t* tile_ev = nullptr;   // per tile: events k_sweep queued in the tile's region of ev_tmp
  uint32_t* tile_ent = nullptr;  // per tile: their enter events
  uint32_t nblk = 0;
  uint32_t* ctr_buf = nullptr;   // [2][CTR_N]: pass P uses half P&1 and zeroes the other (k_place)
  uint32_t* ctr = nullptr;       // current half
  int ctr_sel = 0;
  uint32_t* h_ctr = nullptr;     // pinned
  uint32_t* h_pub = nullptr;     // mapped coherent host memory: [kPubWords] counters + sequence word
  uint32_t* d_pub = nullptr;     // its device address
  uint32_t pub_seq = 0;
  uint32_t last_dense = ~0u;     // dense movers of the last pass (k_sweep_dense launched when non-zero)
  bool last_unsorted = true;     // the last pass needed k_slice_sort (its grid: one thread per op)
  // small passes (run_small_pass): the overlay of slots with an op since the grid was last built
  uint32_t* ov_tag = nullptr;    // [cap] grid generation in which the slot joined the overlay
  uint32_t* ov_idx = nullptr;    // [cap] its overlay entry
  gw::Rec* ov_rec = nullptr;     // [ov_cap] entries
  uint32_t* ov_count = nullptr;  // device: entries
  uint32_t ov_cap = 0;
  uint32_t grid_gen = 1;         // generation of the current grid (ov_tag values of earlier ones are stale)
  uint64_t ov_bound = 0;         // ops of the small passes since the grid was built (>= entries)
  int small_mode = 1;            // 0: off, 1: auto, 2: whenever the overlay has room (tests)
  uint64_t small_passes = 0;
  struct {                       // the last timed pass, collected once its events are complete
    bool pending = false;
    uint32_t n_ops = 0, nev = 0, records = 0, ncells = 0, dense = 0, band = 0;
  } tpend;
  // events
  uint4* ev_tmp = nullptr;
  uint2* ev_out = nullptr;   // device, accumulated over the passes of one tick
  gwaoi_event* h_ev = nullptr;  // pinned + mapped, accumulated over the passes of one tick
  uint2* d_hev = nullptr;       // device alias of h_ev (the copy-out kernel writes it over PCIe)
  uint64_t ev_cap = 0;       // capacity of ev_out
  uint64_t hev_cap = 0;      // capacity of h_ev (0 until a pass delivers events to the host)
  uint32_t tmp_cap = 0;      // capacity of ev_tmp
  uint64_t tick_events = 0, tick_enter = 0;  // accumulated over the passes since the last tick
  uint32_t tick_passes = 0, tick_ops = 0;
  bool acc_open = false;                      // a pass ran since the last gwaoi_tick
  uint64_t passes_run = 0;   // pipeline passes completed by this manager
  uint64_t acc_base = 0;     // passes_run when the event accumulation (ev_out) was opened
  bool acc_silent = false;   // a pass of the accumulation may have applied SILENT ops (not in ev_out)

  gw::SyncState* sync = nullptr;  // sync fan-out / ingest state (gwaoi_sync.hip), on demand

  // pinned host staging (gwaoi_stage_buffers / gwaoi_stage_moves_pinned), allocated on first use
  uint32_t* h_pin_slot = nullptr;
  float *h_pin_x = nullptr, *h_pin_z = nullptr;
  unsigned long long* d_pin_first = nullptr;  // [cap] repeat detection (k_pin_check)
  uint32_t pin_id = 0;
  uint32_t* d_pin_out = nullptr;   // [4]
  uint32_t* h_pin_out = nullptr;   // [4 + 4 nspaces]: out, then the per-Space beyond-extent keys
  uint32_t* d_pin_seen = nullptr;  // [4 nspaces]
  float4* d_pin_ext = nullptr;     // [nspaces]
  float4* h_pin_ext = nullptr;
  bool pin_seen_dirty = true;
  // incremental push (gwaoi_stage_moves_pinned_partial): entries [0, pin_pushed) are on the device already
  uint32_t pin_pushed = 0;
  // deferred verdict (gwaoi_stage_moves_pinned_async): the batch waits in dv_* as a device-counted batch
  // whose count k_pin_count writes (0 when refused); run_pass reads the verdict after the pass
  bool pin_pending = false;
  bool pin_validated = false;        // the pending sub-pass's check validated the batch (its first)
  uint32_t pin_n = 0;                // the batch's size
  uint32_t* d_pin_n = nullptr;       // the sub-pass's op count (device)
  uint32_t* h_pin_v = nullptr;       // the check's four words, mapped coherent host memory
  uint32_t* d_pin_v = nullptr;       // its device alias

  // relation delta export (gwaoi_export_relation_delta): the last tick's events are still in ev_out
  bool dx_ready = false;         // set by gwaoi_tick, cleared when the next accumulation opens
  bool dx_silent = false;        // that tick applied SILENT ops (their pairs are not in the events)
  uint64_t dx_events = 0;
  unsigned long long* dx_keys = nullptr;
  uint32_t *dx_cnt = nullptr, *dx_last = nullptr, *dx_slot = nullptr, *dx_flags = nullptr, *dx_part = nullptr;
  uint2* dx_out = nullptr;
  uint64_t dx_slots = 0, dx_cap = 0;  // hash slots; events the per-event buffers hold

  // timing
  bool timing = false;
  hipEvent_t tev[5] = {};
  gwaoi_stats stats = {};
};

namespace {

// ------------------------------------------------------------------------------------------------
// geometry

void space_extent(const SpaceHost& sh, float* x0, float* z0, float* x1, float* z1) {
  if (!sh.auto_extent) {
    *x0 = sh.desc.min_x;
    *z0 = sh.desc.min_z;
    *x1 = sh.desc.max_x;
    *z1 = sh.desc.max_z;
    return;
  }
  if (!sh.seen_any) {
    *x0 = *z0 = -1000.0f;  // Space.GetSpaceRange default (Space.go:51-53)
    *x1 = *z1 = 1000.0f;
    return;
  }
  const float D = sh.desc.dist;
  const float wx = sh.seen_maxx - sh.seen_minx, wz = sh.seen_maxz - sh.seen_minz;
  *x0 = sh.seen_minx - 0.125f * wx - D;
  *x1 = sh.seen_maxx + 0.125f * wx + D;
  *z0 = sh.seen_minz - 0.125f * wz - D;
  *z1 = sh.seen_maxz + 0.125f * wz + D;
}

#ifndef GW_MID_PLAN
#define GW_MID_PLAN 1550.0
#endif
constexpr double kMidPlanRecs = GW_MID_PLAN;  // the same for the mid sweep (GW_MID_CAP 1850 staged)
constexpr double kBigPlanRecs = 2400.0;  // planned records of a big-sweep region at most (GW_BIG_CAP 2800 staged)
static_assert(kMidPlanRecs < gw::kSweepMidCap && kBigPlanRecs < gw::kSweepBigCap,
              "a region's planned records must stay below what its sweep stages (else every tile overflows)");
constexpr double kCellOccupancy = 0.5;  // planned entities per cell (config 2: 1M in 35,000^2, cells of 25)
#ifndef GW_TILE_MOVERS
#define GW_TILE_MOVERS 440.0
#endif
constexpr double kTileMovers = GW_TILE_MOVERS;  // planned entities per 32 x 32-cell tile (k_sweep: 512 threads)

void compute_geometry(gwaoi_mgr* m, std::vector<gw::Geom>& out) {
  out.resize(m->nspaces);
  const uint64_t share = std::max<uint64_t>(gw::kTileCells, m->max_cells / std::max<uint32_t>(1, m->nspaces));
  uint32_t base = 0;
  for (uint32_t s = 0; s < m->nspaces; ++s) {
    SpaceHost& sh = m->spaces[s];
    float x0, z0, x1, z1;
    space_extent(sh, &x0, &z0, &x1, &z1);
    if (!std::isfinite(x0) || !std::isfinite(x1) || !(x1 > x0)) { x0 = -1000.f; x1 = 1000.f; }
    if (!std::isfinite(z0) || !std::isfinite(z1) || !(z1 > z0)) { z0 = -1000.f; z1 = 1000.f; }
    double c = m->cell_side > 0 ? (double)m->cell_side : (double)sh.desc.dist / (double)m->cells_per_dist;
    if (m->density_cells && !sh.auto_extent) {
      // D / 4 cells hold ~0.5 entities at config-2 density (D 100). A large-D Space at that density
      // gets cells of the same side instead of D / 4 (down to D / 16): a mover's ring of border cells
      // then holds proportionally fewer candidates. Density is planned from the capacity share over
      // the Space's declared extent.
      const double area = ((double)x1 - x0) * ((double)z1 - z0);
      const double pop = sh.pop_hint ? (double)sh.pop_hint : (double)m->cap / std::max<uint32_t>(1, m->nspaces);
      const double cr = std::sqrt(kCellOccupancy * area / std::max(1.0, pop));
      if (cr < 0.75 * c) {
        c = std::max(cr, (double)sh.desc.dist / 16.0);
      } else {
        // Tile fill: the sweep walks a tile's movers one per thread of a kSweepBlock-thread block, so
        // a 32 x 32-cell tile of a uniform crowd should hold a little less than one round of them
        // (the count per tile is Poisson-like: +-sqrt). At config 2 (D 100) this is cells of 22.95
        // instead of 25: 441 movers per tile instead of 522, of which two thirds of the tiles needed a
        // second round; k_sweep 110 -> 98 us. Only for Spaces many tiles wide (a small Space's tiles
        // are mostly partial: its cell count, not its tile fill, sets the cost).
        const double ct = std::sqrt(kTileMovers * area / std::max(1.0, pop)) / gw::kTile;
        const double w = std::min((double)x1 - x0, (double)z1 - z0);
        if (ct < c && w >= 8.0 * gw::kTile * c) c = std::max(ct, (double)sh.desc.dist / 7.0);
      }
    }
    if (!(c > 0)) c = 1.0;
#ifndef GW_DENSE_CELL_DIV
#define GW_DENSE_CELL_DIV 0  // A/B: k > 0 gives a Space whose LDS region cannot fit cells of D / k
#endif
    if (GW_DENSE_CELL_DIV > 0 && m->cell_side <= 0) {
      // its movers all take the dense walk, whose cost follows the candidates of its ring (ring width
      // ~ one cell), not the region: finer cells thin the ring
      const int rch = (int)std::ceil((double)sh.desc.dist * (1.0 + 1e-5) / c) + 1;
      if ((gw::kTile + 2 * rch) * (gw::kTile + 2 * rch) > gw::kSweepRegCells)
        c = std::min(c, (double)sh.desc.dist / GW_DENSE_CELL_DIV);
    }
    // tiles of kTile x kTile cells; cell counts padded to whole tiles
    auto dims = [&](double cc, int64_t* tx, int64_t* tz) {
      const int64_t nx = (int64_t)(((double)x1 - x0) / cc) + 1, nz = (int64_t)(((double)z1 - z0) / cc) + 1;
      *tx = (nx + gw::kTile - 1) / gw::kTile;
      *tz = (nz + gw::kTile - 1) / gw::kTile;
    };
    int64_t tx, tz;
    dims(c, &tx, &tz);
    const double c_want = c;
    bool grown = false;
    while ((uint64_t)(tx * tz) * gw::kTileCells > share || tx * gw::kTile > (1 << 22) || tz * gw::kTile > (1 << 22)) {
      c *= 1.25;
      dims(c, &tx, &tz);
      grown = true;
    }
    if (grown) {
      // back down to the finest cells that keep this tile count (config 3: a 1,600-wide Space at D / 4
      // = 25 needs 65 cells, one over two tiles; the 1.25x steps gave cells of 31.25, with 1.5x the
      // ring candidates, where 25.0000x fits two tiles exactly)
      const double cf = std::max({c_want, ((double)x1 - x0) / (double)(tx * gw::kTile),
                                  ((double)z1 - z0) / (double)(tz * gw::kTile)}) * (1.0 + 1e-6);
      int64_t fx, fz;
      dims(cf, &fx, &fz);
      if (cf < c && fx <= tx && fz <= tz) c = cf, tx = fx, tz = fz;
    }
    gw::Geom g;
    g.x0 = x0;
    g.z0 = z0;
    g.inv_c = (float)(1.0 / c);
    g.D = sh.desc.dist;
    g.ncx = (int32_t)(tx * gw::kTile);
    g.ncz = (int32_t)(tz * gw::kTile);
    g.ntx = (int32_t)tx;
    g.ntz = (int32_t)tz;
    g.base = base;
    g.tile_base = base / gw::kTileCells;
    // halo for the sweep's LDS staging: a query box spans (D + margin) / c cells on each side of the
    // mover's cell, +1 for a mover whose old position is in the neighbouring cell; larger moves take
    // the global path. Region = (kTile + 2 reach)^2 cells must fit the kernel's region budget.
    const double maxc = std::max({std::fabs((double)x0), std::fabs((double)x1), std::fabs((double)z0),
                                  std::fabs((double)z1)});
    const double span = ((double)sh.desc.dist * (1.0 + 1e-5) + (maxc + sh.desc.dist) * 1e-6) / c;
    int reach = (int)std::ceil(span) + 1;  // (ceil(span + 0.25): config 2 -0.7%, skew +1.3%, r06_a2: not kept)
    g.pad = 0;
    const int rw = gw::kTile + 2 * reach;  // region width (cells)
    if (rw * rw > gw::kSweepRegCells) {  // the small LDS sweep's region budget: not this Space
      // the big sweep (one 1024-thread block per CU) when its region fits and the planned population of
      // a region does too (a larger one would only overflow every tile into the dense walk)
      const double area = ((double)x1 - x0) * ((double)z1 - z0);
      const double pop = sh.pop_hint ? (double)sh.pop_hint : (double)m->cap / std::max<uint32_t>(1, m->nspaces);
      const double per_cell = pop * c * c / std::max(1.0, area);
      // (the mid sweep first: two blocks per CU, when its smaller region and record budget hold)
      if (m->big_sweep && rw <= gw::kSweepMidRows && (double)(rw * rw) * per_cell <= kMidPlanRecs)
        g.pad = (uint32_t)reach | gw::kPadMid;
      else if (m->big_sweep && rw <= gw::kSweepBigRows && (double)(rw * rw) * per_cell <= kBigPlanRecs)
        g.pad = (uint32_t)reach;
      reach = 0;  // (the small LDS path off for this Space)
    }
    g.reach = reach;
    base += (uint32_t)(tx * tz) * gw::kTileCells;
    sh.gx0 = x0;
    sh.gz0 = z0;
    sh.gx1 = x1;
    sh.gz1 = z1;
    out[s] = g;
  }
}

uint32_t total_cells(const std::vector<gw::Geom>& g) {
  uint32_t t = 0;
  for (auto& x : g) t += (uint32_t)(x.ncx * x.ncz);
  return t;
}

uint32_t total_tiles(const std::vector<gw::Geom>& g) { return total_cells(g) / gw::kTileCells; }

bool same_geom(const std::vector<gw::Geom>& a, const std::vector<gw::Geom>& b) {
  return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(gw::Geom)) == 0;
}

// ------------------------------------------------------------------------------------------------

// Event buffers: ev_tmp (sweep staging), ev_out (device, accumulated over a tick's passes) and the
// mapped pinned host copy h_ev, allocated only once a pass delivers events to the host (a
// device-events-only user never pins host memory). In copy mode the host capacity equals ev_cap.
int ensure_host_events(gwaoi_mgr* m, uint64_t need, uint64_t keep) {
  if (need <= m->hev_cap) return GWAOI_OK;
  gwaoi_event* nh = nullptr;
  hipError_t he = hipHostMalloc((void**)&nh, need * sizeof(gwaoi_event), hipHostMallocMapped | hipHostMallocCoherent);
  void* dh = nullptr;
  if (he == hipSuccess) he = hipHostGetDevicePointer(&dh, nh, 0);
  if (he != hipSuccess) {
    set_err("mapped host event buffer (%llu events): %s", (unsigned long long)need, hipGetErrorString(he));
    if (nh) hipHostFree(nh);
    return GWAOI_ERR_NOMEM;
  }
  if (keep && m->h_ev) std::memcpy(nh, m->h_ev, keep * sizeof(gwaoi_event));
  if (m->h_ev) hipHostFree(m->h_ev);
  m->h_ev = nh;
  m->d_hev = (uint2*)dh;
  m->hev_cap = need;
  return GWAOI_OK;
}

int ensure_events(gwaoi_mgr* m, uint64_t need_out, uint32_t need_tmp, uint64_t keep, bool host) {
  if (need_tmp > m->tmp_cap) {
    uint32_t nc = std::max<uint32_t>(need_tmp, m->tmp_cap * 2);
    if (m->ev_tmp) hipFree(m->ev_tmp);
    m->ev_tmp = nullptr;
    RCHK(dalloc(&m->ev_tmp, nc));
    m->tmp_cap = nc;
  }
  if (need_out > m->ev_cap) {
    uint64_t nc = std::max<uint64_t>(need_out, m->ev_cap * 2);
    uint2* nd = nullptr;
    RCHK(dalloc(&nd, nc));
    if (keep) {
      HIPCHK(hipMemcpyAsync(nd, m->ev_out, keep * sizeof(uint2), hipMemcpyDeviceToDevice, m->stream));
      HIPCHK(hipStreamSynchronize(m->stream));
    }
    if (m->ev_out) hipFree(m->ev_out);
    m->ev_out = nd;
    m->ev_cap = nc;
  }
  if (host) RCHK(ensure_host_events(m, m->ev_cap, keep));
  return GWAOI_OK;
}

// The band walk's keys over grid gi (records <= bound): per record its {x, z} search keys, per cell the
// records sorted by each, per Space the keys' spread. The arrays are allocated on first use for
// the grid's largest size (2 records per slot); without the memory the dense walk reads whole rings.
#ifndef GW_BAND_TABLE
#define GW_BAND_TABLE_HOST 1
#else
#define GW_BAND_TABLE_HOST GW_BAND_TABLE
#endif
int build_band_keys(gwaoi_mgr* m, int gi, uint32_t bound, bool* built) {
  *built = false;
  Grid& G = m->grid[gi];
  if (!G.ntiles || !bound) return GWAOI_OK;
  if (!m->band_cap) {
    const uint64_t n = 2 * (uint64_t)m->cap;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < n * 20 + 4ull * m->cap + (64ull << 20)) return GWAOI_OK;
    // (x and z keys in one allocation: the band walk reads both through one buffer descriptor)
    if (dalloc(&m->band_xk, 2 * n) || dalloc(&m->band_zi, n) ||
        dalloc(&m->band_hd, 2 * (size_t)m->nspaces) || dalloc(&m->band_dense2, m->cap)) {  // (no room: the ring walk)
      for (void* p : {(void*)m->band_xk, (void*)m->band_zi, (void*)m->band_hd,
                      (void*)m->band_dense2})
        if (p) hipFree(p);
      m->band_xk = m->band_zk = nullptr, m->band_zi = m->band_hd = m->band_dense2 = nullptr;
      return GWAOI_OK;
    }
    m->band_zk = m->band_xk + n;
    m->band_cap = n;
    // the key tables: 64 B per axis per 4 records of address space (only the sorted cells of >= 4 records
    // write theirs); without them (no room) the walk reads its cells whole
    const uint64_t half = (n / 4 + 1) * (uint64_t)gw::kBandBuckets;
    if (GW_BAND_TABLE_HOST && half < (1ull << 30) && hipMemGetInfo(&fr, &tot) == hipSuccess && fr > 2 * half + (64ull << 20) &&
        dalloc(&m->band_tab, 2 * half) == GWAOI_OK) {
      m->band_tab_half = (uint32_t)half;
    } else {
      (void)hipGetLastError();
      m->band_tab = nullptr;
    }
  }
  HIPCHK(hipMemsetAsync(m->band_hd, 0, 2 * (size_t)m->nspaces * sizeof(uint32_t), m->stream));
  gw::BandArgs b{};
  b.g = {G.rec, G.cs, G.d_geom, G.d_tile_space};
  b.space_of = m->space_of;
  b.nspaces = m->nspaces;
  // every record of the grid (the grid holds at most 2 cap records, main + ghost): the records are swapped
  // in below, so a bound below the grid's real count would publish a half-copied grid
  b.rec_bound = (uint32_t)m->band_cap;
  b.nrec = G.cs + G.ncells;
  // the records sorted by x key inside their cells go into the other grid's record buffer (this pass does
  // not read it: it was the build's bucket buffer), which then becomes this grid's
  b.rec_out = m->grid[gi ^ 1].rec;
  b.xk = m->band_xk;
  b.zk = m->band_zk;
  b.zi = m->band_zi;
  b.hd = m->band_hd;
  b.tab = m->band_tab;
  b.tab_half = m->band_tab_half;
  gw::launch_band_keys(b, m->stream);
  HIPCHK(hipGetLastError());
  std::swap(G.rec, m->grid[gi ^ 1].rec);
  m->band_builds++;
  *built = true;
  return GWAOI_OK;
}

int upload_geom(gwaoi_mgr* m, Grid& g, const std::vector<gw::Geom>& geo) {
  if (same_geom(g.h_geom, geo)) return GWAOI_OK;
  g.h_geom = geo;
  g.ncells = total_cells(geo);
  g.ntiles = total_tiles(geo);
  std::vector<uint32_t> ts(g.ntiles);
  for (uint32_t s = 0; s < geo.size(); ++s)
    for (uint32_t t = 0; t < (uint32_t)(geo[s].ntx * geo[s].ntz); ++t) ts[geo[s].tile_base + t] = s;
  HIPCHK(hipStreamSynchronize(m->stream));  // the staging vectors below are pageable
  HIPCHK(hipMemcpy(g.d_geom, g.h_geom.data(), geo.size() * sizeof(gw::Geom), hipMemcpyHostToDevice));
  if (g.ntiles) HIPCHK(hipMemcpy(g.d_tile_space, ts.data(), g.ntiles * sizeof(uint32_t), hipMemcpyHostToDevice));
  return GWAOI_OK;
}

// Grids of up to kMaxLdsTiles tiles are built tile-bucketed (no global atomics); larger ones by the
// cell-atomic counting sort, which needs zeroed cell counts.
bool tile_build(const Grid& g) { return g.ntiles <= gw::kMaxLdsTiles; }

// Build grid `gi` from the per-slot state (pos, seq, space_of).
// Build grid `gi` for the pass whose ops have seqs [base, base + n_ops) (n_ops = 0: the current
// state only, no ghosts).
// kBuildAuto: the one-pass build when the previous tile build's starts fit this grid, else counting;
// kBuildCounting: the counting build (outside a pass: nothing would see an overflow); kBuildRerun: the
// re-run of a pass whose one-pass build overflowed (the same buffers, counting build).
enum BuildMode { kBuildAuto, kBuildCounting, kBuildRerun };
int build_grid(gwaoi_mgr* m, int gi, uint32_t base, uint32_t n_ops, const uint8_t* op_kind, BuildMode mode = kBuildAuto) {
  const bool counting = mode == kBuildRerun;
  Grid& g = m->grid[gi];
  const bool tiles = tile_build(g);
  if (!tiles && g.cs_zeroed < g.ncells + 1)
    HIPCHK(hipMemsetAsync(g.cs, 0, (size_t)(g.ncells + 1) * sizeof(uint32_t), m->stream));
  g.cs_zeroed = 0;
  gw::BinArgs b{};
  b.pos_x = m->pos_x;
  b.pos_z = m->pos_z;
  b.seq = m->seq;
  b.space_of = m->space_of;
  b.old_x = m->old_x;
  b.old_z = m->old_z;
  b.old_seq = m->old_seq;
  b.opq = m->opq;
  b.base = base;
  b.n_ops = n_ops;
  b.geom = g.d_geom;
  b.nspaces = m->nspaces;
  b.cap = m->cap;
  b.key_of = m->key_of;
  b.local_of = m->local_of;
  b.cs = g.cs;
  b.rec = g.rec;
  b.ntiles = g.ntiles;
  b.nblk = m->nblk;
  b.chunk = gw::bin_chunk(m->cap);
  b.thist = m->thist;
  const int sel = counting ? m->ttot_sel ^ 1 : m->ttot_sel;  // a re-run uses the failed build's buffers
  b.ttot = m->ttot + sel * gw::kMaxLdsTiles;
  b.ttot_next = m->ttot + (sel ^ 1) * gw::kMaxLdsTiles;
  b.tstart = m->tstart + sel * (gw::kMaxLdsTiles + 1);
  b.tprev = m->tstart + (sel ^ 1) * (gw::kMaxLdsTiles + 1);
  b.tile_space = g.d_tile_space;
  b.trec = m->grid[gi ^ 1].rec;  // the other grid's records are not read by this pass
  b.trec_cap = 2 * m->cap;
  b.op_kind = op_kind;
  b.tile_walk = m->tile_walk;
  b.tile_acted = m->tile_acted;
  b.ctr = m->ctr;
  b.fused = 0;
  if (tiles) {
    // the one-pass build only when its plan fits the bucket buffer: the last tile's planned start is
    // the previous build's records x 5/4 + 16 per tile (plan_start); a full world whose entities mostly
    // change cell (2 records each) would otherwise overflow every pass. After a re-run (the plan did not
    // hold), one counting build first.
    const uint64_t plan_end = (uint64_t)m->h_ctr[gw::CTR_RECORDS] * 5u / 4u + 16ull * g.ntiles;
    b.fused = mode == kBuildAuto && m->build_mode == 0 && m->plan_ok && same_geom(m->plan_geom, g.h_geom) &&
              !m->rerun_counting && plan_end <= b.trec_cap;
    m->rerun_counting = false;
    if (counting) HIPCHK(hipMemsetAsync(b.ttot, 0, (size_t)gw::kMaxLdsTiles * sizeof(uint32_t), m->stream));
    gw::launch_bin_tiles(b, m->stream);
    if (!counting) m->ttot_sel ^= 1;
    (b.fused ? m->builds_fused : m->builds_counting)++;
    if (!m->plan_ok || !same_geom(m->plan_geom, g.h_geom)) m->plan_geom = g.h_geom;
    m->plan_ok = true;
  } else {
    m->plan_ok = false;
    gw::launch_bin_count(b, m->stream);
    gw::launch_scan(m->scan, g.cs, g.ncells + 1, m->stream);
    gw::launch_bin_scatter(b, m->stream);
  }
  HIPCHK(hipGetLastError());
  return GWAOI_OK;
}

// Rank-compress every present slot's seq (order preserved) when the counter nears its limit.
int renormalise(gwaoi_mgr* m) {
  HIPCHK(hipStreamSynchronize(m->stream));
  std::vector<uint32_t> q(m->cap);
  HIPCHK(hipMemcpy(q.data(), m->seq, m->cap * sizeof(uint32_t), hipMemcpyDeviceToHost));
  std::vector<std::pair<uint32_t, uint32_t>> v;
  v.reserve(m->n_present_dev);
  for (uint32_t s = 0; s < m->cap; ++s)
    if (q[s]) v.emplace_back(q[s], s);
  std::sort(v.begin(), v.end());
  for (size_t i = 0; i < v.size(); ++i) q[v[i].second] = (uint32_t)i + 1;
  HIPCHK(hipMemcpy(m->seq, q.data(), m->cap * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemsetAsync(m->opq, 0, (size_t)m->cap * sizeof(uint32_t), m->stream));  // stale op seqs
  RCHK(build_grid(m, m->cur, 0, 0, nullptr, kBuildCounting));
  // the grid now holds every slot's current state with the new seqs: the overlay (copies of records
  // with the old seqs) starts over, as after any full build
  m->grid_gen++;
  m->ov_bound = 0;
  HIPCHK(hipMemsetAsync(m->ov_count, 0, sizeof(uint32_t), m->stream));
  m->next_seq = (uint32_t)v.size() + 1;
  HIPCHK(hipStreamSynchronize(m->stream));
  return GWAOI_OK;
}

void reset_tick(gwaoi_mgr* m) {
  m->tick_events = 0;
  m->tick_enter = 0;
  m->tick_passes = 0;
  m->tick_ops = 0;
}

// Stage times of the last timed pass into the stats (its hipEvents are complete or about to be).
int collect_timing(gwaoi_mgr* m) {
  if (!m->tpend.pending) return GWAOI_OK;
  m->tpend.pending = false;
  HIPCHK(hipEventSynchronize(m->tev[4]));
  float t01, t12, t23, t34, t04;
  HIPCHK(hipEventElapsedTime(&t01, m->tev[0], m->tev[1]));
  HIPCHK(hipEventElapsedTime(&t12, m->tev[1], m->tev[2]));
  HIPCHK(hipEventElapsedTime(&t23, m->tev[2], m->tev[3]));
  HIPCHK(hipEventElapsedTime(&t34, m->tev[3], m->tev[4]));
  HIPCHK(hipEventElapsedTime(&t04, m->tev[0], m->tev[4]));
  m->stats.ticks++;
  m->stats.ms_apply += t01;
  m->stats.ms_grid += t12;
  m->stats.ms_sweep += t23;
  m->stats.ms_order += t34;
  m->stats.ms_total += t04;
  m->stats.sweep_movers += m->tpend.n_ops;
  m->stats.events += m->tpend.nev;
  m->stats.grid_records += m->tpend.records;
  m->stats.grid_cells += m->tpend.ncells;
  m->stats.dense_movers += m->tpend.dense;
  m->stats.band_movers += m->tpend.band;
  return GWAOI_OK;
}

// End of a pass: the counters to h_ctr, every kernel of the pass complete. With the mapped
// publication buffer, a one-thread kernel writes them there and the host spins on the sequence word
// (polling the stream for errors now and then); host event delivery (GPU writes into mapped memory
// by k_copy_out) keeps the stream synchronisation.
// The order stage's last kernel publishes (k_slice_sort's last block, OrderArgs.pub) when
// publish_seq() gave it a sequence word; otherwise (host event delivery, no mapped buffer) the counters
// are copied and the stream synchronised.
uint32_t publish_seq(gwaoi_mgr* m, bool copy_events) {
  if (!m->h_pub || copy_events) return 0u;
  return ++m->pub_seq ? m->pub_seq : ++m->pub_seq;  // never 0 (the initial value)
}

int wait_pub(gwaoi_mgr* m, uint32_t seq) {
  hipStream_t st = m->stream;
  volatile uint32_t* flag = m->h_pub + gw::kPubWords;
  for (uint64_t spin = 1; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq; ++spin) {
    if ((spin & 0xFFFF) == 0) {
      const hipError_t e = hipStreamQuery(st);
      if (e == hipSuccess) {  // everything done: the flag must be visible now
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
          set_err("end-of-pass publication lost (flag %u, want %u)", *flag, seq);
          return GWAOI_ERR_HIP;
        }
        break;
      }
      if (e != hipErrorNotReady) HIPCHK(e);
    }
    __builtin_ia32_pause();
  }
  return GWAOI_OK;
}

int finish_pass(gwaoi_mgr* m, uint32_t seq) {
  hipStream_t st = m->stream;
  if (!seq) {
    HIPCHK(hipMemcpyAsync(m->h_ctr, m->ctr, gw::CTR_N * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return GWAOI_OK;
  }
  RCHK(wait_pub(m, seq));
  std::memcpy(m->h_ctr, m->h_pub, gw::kPubWords * sizeof(uint32_t));
  return GWAOI_OK;
}

#ifndef GW_RD_MAPPED
#define GW_RD_MAPPED 1
#endif
// Device words a[0, na) and b[0, nb) to the host, every kernel launched before complete: through the
// publication buffer (a one-thread kernel, the host spins on the sequence word) when there is one,
// else DMA copies and a stream synchronisation. The relation's size read-backs between its launches.
int read_words(gwaoi_mgr* m, const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb, uint32_t* out) {
  hipStream_t st = m->stream;
  if (GW_RD_MAPPED && m->h_pub && na + nb <= (uint32_t)gw::kPubWords) {
    const uint32_t seq = ++m->pub_seq ? m->pub_seq : ++m->pub_seq;
    gw::launch_publish_words(a, na, b, nb, m->d_pub, seq, st);
    HIPCHK(hipGetLastError());
    RCHK(wait_pub(m, seq));
    std::memcpy(out, m->h_pub, (na + nb) * sizeof(uint32_t));
    return GWAOI_OK;
  }
  if (na) HIPCHK(hipMemcpyAsync(out, a, na * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  if (nb) HIPCHK(hipMemcpyAsync(out + na, b, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return GWAOI_OK;
}

// ---- small passes -------------------------------------------------------------------------------
// A pass with few ops (an Enter or Leave flushed on its own, EntityManager.go:229-273 / Space.go:188-251,
// a handful of Moved calls) does not rebuild the grid: k_apply adds its ops' slots to the overlay, and
// each op's mover is judged against the current grid plus the overlay (k_sweep_small, one wave per op).
// The overlay grows until a pass with many ops rebuilds the grid (or a consumer of the grid refreshes it,
// ensure_grid_current). Cost: O(ops x (box + overlay)) instead of the full build and sweep over every slot.
constexpr uint32_t kSmallMaxOps = 1024;                   // ops of a small pass at most
constexpr uint64_t kSmallWork = 1ull << 22;               // ops x overlay entries at most (the overlay scan)
constexpr size_t kOverlayCap = 16384;

bool small_pass_ok(gwaoi_mgr* m, uint32_t n_ops) {
  if (!m->small_mode || m->geom_dirty || m->sweep_lds != 1 || !m->passes_run || !m->grid[m->cur].ntiles) return false;
  const uint64_t ov = m->ov_bound + n_ops;
  if (ov > m->ov_cap) return false;
  if (m->small_mode == 2) return true;
  // a full pass over the present slots costs about as much as ~16k overlay-walk ops: stay below a small
  // fraction of it
  return n_ops <= kSmallMaxOps && (uint64_t)n_ops * ov <= kSmallWork && (uint64_t)n_ops * 64 <= m->n_present_dev;
}

int run_small_pass(gwaoi_mgr* m, bool copy_events, uint32_t base, uint32_t n_ops) {
  const bool dev = m->dv_n != 0;
  const bool dev_mixed = dev && m->dv_kind;
  hipStream_t st = m->stream;
  RCHK(collect_timing(m));
  if (m->timing) HIPCHK(hipEventRecord(m->tev[0], st));
  // host ops: k_apply reads them from the pinned arrays over PCIe (five DMA copies cost more than the
  // whole small pass's kernels) and leaves device copies of slot and kind for the sweep
  const bool mapped = !dev && m->hd_op_slot;
  if (!dev && !mapped) {
    HIPCHK(hipMemcpyAsync(m->d_op_slot, m->h_op_slot, n_ops * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(m->d_op_x, m->h_op_x, n_ops * sizeof(float), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(m->d_op_z, m->h_op_z, n_ops * sizeof(float), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(m->d_op_kind, m->h_op_kind, n_ops, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(m->d_op_space, m->h_op_space, n_ops * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  }
  gw::ApplyArgs a{};
  a.n_dev = dev ? m->dv_count : nullptr;
  a.op_slot = dev ? m->dv_slot : mapped ? m->hd_op_slot : m->d_op_slot;
  a.op_x = dev ? m->dv_x : mapped ? m->hd_op_x : m->d_op_x;
  a.op_z = dev ? m->dv_z : mapped ? m->hd_op_z : m->d_op_z;
  a.op_kind = dev ? m->dv_kind : mapped ? m->hd_op_kind : m->d_op_kind;
  a.op_space = dev ? m->dv_space : mapped ? m->hd_op_space : m->d_op_space;
  a.cp_slot = mapped ? m->d_op_slot : nullptr;
  a.cp_kind = mapped ? m->d_op_kind : nullptr;
  a.nspaces = m->nspaces;
  a.leaves = dev_mixed ? m->d_leaves : nullptr;  // (the presence delta of a mixed batch is counted with it)
  a.n_ops = n_ops;
  a.base = base;
  a.cap = m->cap;
  a.check = dev ? 1 : 0;
  a.pos_x = m->pos_x;
  a.pos_z = m->pos_z;
  a.seq = m->seq;
  a.space_of = m->space_of;
  a.old_x = m->old_x;
  a.old_z = m->old_z;
  a.old_seq = m->old_seq;
  a.opq = m->opq;
  a.ctr = m->ctr;
  a.rank_cnt = m->rank_cnt;
  a.gen = m->grid_gen;
  a.ov_tag = m->ov_tag;
  a.ov_idx = m->ov_idx;
  a.ov_rec = m->ov_rec;
  a.ov_count = m->ov_count;
  a.ov_cap = m->ov_cap;
  // a single host op (the Go wrapper's flushed Enter / Leave): applied, swept and ordered by one kernel
  const bool one_op = mapped && n_ops == 1;
  if (!one_op) gw::launch_apply(a, st);
  HIPCHK(hipGetLastError());
  if (m->timing) HIPCHK(hipEventRecord(m->tev[1], st));
  if (m->timing) HIPCHK(hipEventRecord(m->tev[2], st));
  const uint64_t keep = m->tick_events;
  const Grid& G = m->grid[m->cur];
  if (m->tmp_cap < 4096u) RCHK(ensure_events(m, m->ev_cap, 4096u, keep, false));
  for (int attempt = 0;; ++attempt) {
    if (attempt) {
      HIPCHK(hipMemsetAsync(m->rank_cnt, 0, ((size_t)n_ops + 1) * sizeof(uint32_t), st));
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_EVENTS, 0, sizeof(uint32_t), st));
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_ENTER, 0, sizeof(uint32_t), st));
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_DENSE, 0, 2 * sizeof(uint32_t), st));  // + CTR_HOLES
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_UNSORTED, 0, 4 * sizeof(uint32_t), st));  // .. CTR_SMALL_OVF
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_SDONE, 0, 2 * sizeof(uint32_t), st));
    }
    if (copy_events) RCHK(ensure_host_events(m, m->ev_cap, keep));
    const bool one = one_op && attempt == 0;  // (a re-run sweeps the op applied by the first attempt)
    const bool fused = n_ops <= gw::kOrderSmallOps;  // one-block order stage (k_order_small)
    gw::OrderArgs o{};
    o.g = {m->ctr, m->tmp_cap, keep, m->ev_cap};
    o.ev_tmp = m->ev_tmp;
    o.ev_fix = nullptr;
    o.tile_ev = m->tile_ev;
    o.tile_ent = m->tile_ent;
    o.ntiles_fix = 0;
    o.scratch = reinterpret_cast<uint2*>(m->ev_tmp);
    o.rank_off = m->rank_cnt;
    o.uns = m->uns;
    o.ev_out = m->ev_out + keep;
    o.host_out = copy_events ? m->d_hev + keep : nullptr;
    o.n_ops = n_ops;
    o.zero_cs = nullptr;  // (the next full build's target was zeroed by the last full pass)
    o.zero_n = 0;
    o.ctr_next = m->ctr_buf + (m->ctr_sel ^ 1) * gw::CTR_N;
    o.grid_total = G.cs + G.ncells;
    o.op_slot = mapped ? m->d_op_slot : a.op_slot;
    o.opq = m->opq;
    o.base = base;
    o.cap = m->cap;
    o.check_ops = dev ? 1 : 0;  // (no per-tile acted counts: k_slice_sort checks every op's slot)
    o.tile_acted = nullptr;
    o.ntiles_acted = 0;
    o.n_dev = a.n_dev;
    // (a single op's pass publishes even with host delivery: its kernel writes the slice into the mapped
    // host buffer itself, before the publication)
    o.pub_seq = publish_seq(m, copy_events && !one);
    o.pub = o.pub_seq ? m->d_pub : nullptr;
    o.sorted_hint = !o.check_ops ? 1 : 0;  // few blocks: a small pass sorts few slices
    o.place_blocks = 16;
    gw::SmallArgs sa{};
    sa.g = {G.rec, G.cs, G.d_geom, G.d_tile_space};
    sa.base = base;
    sa.n_ops = n_ops;
    sa.n_dev = a.n_dev;
    sa.op_slot = mapped ? m->d_op_slot : a.op_slot;
    sa.op_kind = mapped ? m->d_op_kind : a.op_kind;
    sa.space_of = m->space_of;
    sa.pos_x = m->pos_x;
    sa.pos_z = m->pos_z;
    sa.old_x = m->old_x;
    sa.old_z = m->old_z;
    sa.old_seq = m->old_seq;
    sa.opq = m->opq;
    sa.gen = m->grid_gen;
    sa.ov_tag = m->ov_tag;
    sa.ov_rec = m->ov_rec;
    sa.ov_count = m->ov_count;
    sa.ev_tmp = m->ev_tmp;
    sa.ev_cap = m->tmp_cap;
    sa.rank_cnt = m->rank_cnt;
    sa.ctr = m->ctr;
    sa.one_op = one ? 1 : 0;
    sa.ap = a;
    sa.od = o;
    if (one) {
      sa.one_slot = m->h_op_slot[0];
      sa.one_kind = m->h_op_kind[0];
      sa.one_x = m->h_op_x[0];
      sa.one_z = m->h_op_z[0];
      sa.one_space = m->h_op_space[0];
    }
    gw::launch_sweep_small(sa, st);
    HIPCHK(hipGetLastError());
    if (m->timing) HIPCHK(hipEventRecord(m->tev[3], st));
    if (one) {
      if (!o.pub) gw::launch_copy_out(o, st);  // (published: the kernel wrote the host slice itself)
    } else {
      if (!fused) gw::launch_scan(m->scan, m->rank_cnt, n_ops + 1, st);
      if (fused)
        gw::launch_order_small(o, st);
      else
        gw::launch_order(o, st);
    }
    HIPCHK(hipGetLastError());
    if (m->timing) HIPCHK(hipEventRecord(m->tev[4], st));
    RCHK(finish_pass(m, o.pub_seq));
    if ((fused || one) && m->h_ctr[gw::CTR_SMALL_OVF] && !m->h_ctr[gw::CTR_ERR]) {
      // more events than k_order_small's LDS: the general kernels, on the counts it scanned
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_SMALL_OVF, 0, sizeof(uint32_t), st));
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_SDONE, 0, sizeof(uint32_t), st));
      o.pub_seq = publish_seq(m, copy_events);
      o.pub = o.pub_seq ? m->d_pub : nullptr;
      gw::launch_order(o, st);
      HIPCHK(hipGetLastError());
      if (m->timing) HIPCHK(hipEventRecord(m->tev[4], st));
      RCHK(finish_pass(m, o.pub_seq));
    }
    if (m->h_ctr[gw::CTR_ERR]) {
      m->broken = true;
      set_err("device-staged batch failed validation (flags 0x%x: 1=duplicate slot, 2=absent slot, 4=slot >= "
              "capacity, 8=Enter of a present slot, 16=Space id out of range, 32=op count above its bound, "
              "64=non-finite coordinate); the manager is unusable",
              m->h_ctr[gw::CTR_ERR]);
      return GWAOI_ERR_DEVICE_CHECK;
    }
    const uint32_t slots = m->h_ctr[gw::CTR_EVENTS], nev = m->h_ctr[gw::CTR_NEV];
    if (slots > m->tmp_cap || keep + nev > m->ev_cap) {
      RCHK(ensure_events(m, keep + nev, slots, keep, copy_events));
      if (attempt < 3) continue;
      set_err("event buffer overflow persisted");
      return GWAOI_ERR_NOMEM;
    }
    m->tick_events += nev;
    m->tick_enter += m->h_ctr[gw::CTR_ENTER];
    if (m->timing) {
      m->tpend.pending = true;
      m->tpend.n_ops = m->h_ctr[gw::CTR_NOPS];
      m->tpend.nev = nev;
      m->tpend.records = 0;
      m->tpend.ncells = 0;
      m->tpend.dense = 0;
      m->tpend.band = 0;
    }
    break;
  }
  m->ov_bound += n_ops;
  m->small_passes++;
  m->passes_run++;
  m->ctr_sel ^= 1;
  m->ctr = m->ctr_buf + m->ctr_sel * gw::CTR_N;
  m->tick_passes++;
  m->tick_ops += m->h_ctr[gw::CTR_NOPS];
  m->n_ops = 0;
  m->n_leaves = 0;
  m->dv_n = 0;
  m->dv_slot = nullptr;
  m->dv_x = m->dv_z = nullptr;
  m->pass_id++;
  if (dev_mixed) m->n_present += m->h_ctr[gw::CTR_PRESENT];  // signed delta, two's complement
  m->n_present_dev = m->n_present;
  m->dv_kind = nullptr;
  m->dv_space = nullptr;
  m->dv_count = nullptr;
  return GWAOI_OK;  // (last_unsorted and the dense hint stay the last full pass's)
}

// The grid of the last full build plus an overlay is current for the sweep, not for readers of the grid
// itself (relation view, sync fan-out, strips): rebuild it from the slots' state first.
int ensure_grid_current(gwaoi_mgr* m) {
  if (!m->ov_bound) return GWAOI_OK;
  RCHK(build_grid(m, m->cur, m->next_seq, 0, nullptr, kBuildCounting));
  m->grid_gen++;
  m->ov_bound = 0;
  HIPCHK(hipMemsetAsync(m->ov_count, 0, sizeof(uint32_t), m->stream));
  return GWAOI_OK;
}

// Run the device pipeline over the staged batch (host ops or the device batch). Events accumulate
// (device buffer always, host buffer when copy_events) until the next gwaoi_tick returns them.
int run_pass_core(gwaoi_mgr* m, bool copy_events) {
  const bool dev = m->dv_n != 0;
  const uint32_t n_ops = dev ? m->dv_n : m->n_ops;
  if (!n_ops) return GWAOI_OK;
  if (!dev) m->pin_pushed = 0;  // host ops are copied into (or their slots and kinds written to) d_op_*
  if (!m->acc_open) {
    reset_tick(m);
    m->acc_open = true;
    m->dx_ready = false;  // ev_out is about to be overwritten
    m->acc_base = m->passes_run;
    m->acc_silent = false;
  }
  if (dev && m->dv_kind) m->acc_silent = true;  // a mixed device batch may hold SILENT ops
  if ((uint64_t)m->next_seq + n_ops >= kSeqLimit) RCHK(renormalise(m));
  const uint32_t base = m->next_seq;
  m->next_seq += n_ops;
  if (small_pass_ok(m, n_ops)) return run_small_pass(m, copy_events, base, n_ops);
  const int og = m->cur, ng = m->cur ^ 1;
  hipStream_t st = m->stream;
  if (m->ov_bound) {  // the grid is rebuilt from the slots' state: the overlay starts over
    m->grid_gen++;
    m->ov_bound = 0;
    HIPCHK(hipMemsetAsync(m->ov_count, 0, sizeof(uint32_t), st));
  }

  // geometry of the new grid: the latest geometry (recomputed when auto extents grew)
  std::vector<gw::Geom> geo = m->grid[og].h_geom;
  if (m->geom_dirty) {
    compute_geometry(m, geo);
    m->geom_dirty = false;
  }
  RCHK(upload_geom(m, m->grid[ng], geo));

  RCHK(collect_timing(m));  // before the events are recorded again
  if (m->timing) HIPCHK(hipEventRecord(m->tev[0], st));
  if (!dev) {
    HIPCHK(hipMemcpyAsync(m->d_op_slot, m->h_op_slot, n_ops * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(m->d_op_x, m->h_op_x, n_ops * sizeof(float), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(m->d_op_z, m->h_op_z, n_ops * sizeof(float), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(m->d_op_kind, m->h_op_kind, n_ops, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(m->d_op_space, m->h_op_space, n_ops * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    if (m->n_leaves)
      HIPCHK(hipMemcpyAsync(m->d_leaves, m->h_leaves, m->n_leaves * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  }
  gw::ApplyArgs a{};
  a.n_dev = dev ? m->dv_count : nullptr;
  a.op_slot = dev ? m->dv_slot : m->d_op_slot;
  a.op_x = dev ? m->dv_x : m->d_op_x;
  a.op_z = dev ? m->dv_z : m->d_op_z;
  const bool dev_mixed = dev && m->dv_kind;
  a.op_kind = dev ? m->dv_kind : m->d_op_kind;
  a.op_space = dev ? m->dv_space : m->d_op_space;
  a.nspaces = m->nspaces;
  a.leaves = dev_mixed ? m->d_leaves : nullptr;
  a.n_ops = n_ops;
  a.base = base;
  a.cap = m->cap;
  a.check = dev ? 1 : 0;
  a.pos_x = m->pos_x;
  a.pos_z = m->pos_z;
  a.seq = m->seq;
  a.space_of = m->space_of;
  a.old_x = m->old_x;
  a.old_z = m->old_z;
  a.old_seq = m->old_seq;
  a.opq = m->opq;
  a.ctr = m->ctr;
  a.rank_cnt = m->rank_cnt;
  a.ov_rec = nullptr;  // (a full pass: no overlay)
  gw::launch_apply(a, st);
  HIPCHK(hipGetLastError());
  if (m->timing) HIPCHK(hipEventRecord(m->tev[1], st));

  RCHK(build_grid(m, ng, base, n_ops, a.op_kind));
  if (m->timing) HIPCHK(hipEventRecord(m->tev[2], st));

  const uint32_t n_new = dev ? m->n_present_dev : m->n_present;
  const uint32_t n_start = m->n_present_dev;  // present at the start of the pass
  const uint64_t keep = m->tick_events;
  // ev_tmp: k_sweep's per-tile regions (F slots, tile builds with the LDS sweep), then the shared region
  const bool fixed = tile_build(m->grid[ng]) && m->sweep_lds != 0 && m->grid[ng].ntiles;
  const uint32_t F = fixed ? m->grid[ng].ntiles * gw::sweep_ev_lds() : 0u;
  if (m->tmp_cap < F + 4096u) RCHK(ensure_events(m, m->ev_cap, F + 4096u, keep, false));
  // events: expected count is small; grow and re-run the (pure) sweep on overflow. Three causes of a
  // re-run, each with its own bound: the one-pass build's plan did not hold (build_rr), the event buffers
  // were too small (ev_rr), the sweep listed dense movers while k_sweep_dense was not launched (the
  // previous pass had none; dense_rr)
  bool rebuild = false, force_dense = false, keys = false;  // keys: band keys built for this pass's grid
  int build_rr = 0, ev_rr = 0, dense_rr = 0;
  for (int attempt = 0;; ++attempt) {
    if (rebuild) {  // the one-pass build's plan did not hold: the same pass with the counting build
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_BOVF, 0, sizeof(uint32_t), st));
      RCHK(build_grid(m, ng, base, n_ops, a.op_kind, kBuildRerun));
      m->build_reruns++;
      m->rerun_counting = true;
      rebuild = false;
      keys = false;
    }
    if (attempt) {  // re-run: reset what the sweep and the order stage accumulate
      // the scan turned the counts into offsets, and the sweep stores non-zero counts only
      HIPCHK(hipMemsetAsync(m->rank_cnt, 0, ((size_t)n_ops + 1) * sizeof(uint32_t), st));
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_EVENTS, 0, sizeof(uint32_t), st));
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_ENTER, 0, sizeof(uint32_t), st));
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_DENSE, 0, 2 * sizeof(uint32_t), st));  // + CTR_HOLES
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_UNSORTED, 0, 3 * sizeof(uint32_t), st));  // + UNS_SOME, BAND_MV
      // (an overflowing order stage returned before k_slice_sort cleared the flags it would have read)
      HIPCHK(hipMemsetAsync(m->uns, 0, ((size_t)n_ops / 32 + 1) * sizeof(uint32_t), st));
      HIPCHK(hipMemsetAsync(m->ctr + gw::CTR_SDONE, 0, 2 * sizeof(uint32_t), st));  // + CTR_RING_MV
    }
    gw::SweepArgs s{};
    const Grid& G = m->grid[ng];
    s.g = {G.rec, G.cs, G.d_geom, G.d_tile_space};
    s.ntiles = G.ntiles;
    {  // the tiles of the big sweep's Spaces, as one range
      uint32_t b0 = ~0u, b1 = 0;
      for (const gw::Geom& sg : G.h_geom)
        if (sg.reach == 0 && sg.pad > 0 && !(sg.pad & gw::kPadMid)) {
          b0 = std::min(b0, sg.tile_base);
          b1 = std::max(b1, sg.tile_base + (uint32_t)(sg.ntx * sg.ntz));
        }
      s.big_t0 = b1 > b0 ? b0 : 0u;
      s.big_n = b1 > b0 ? b1 - b0 : 0u;
      uint32_t m0 = ~0u, m1 = 0;  // and the mid sweep's
      for (const gw::Geom& sg : G.h_geom)
        if (sg.reach == 0 && (sg.pad & gw::kPadMid)) {
          m0 = std::min(m0, sg.tile_base);
          m1 = std::max(m1, sg.tile_base + (uint32_t)(sg.ntx * sg.ntz));
        }
      s.mid_t0 = m1 > m0 ? m0 : 0u;
      s.mid_n = m1 > m0 ? m1 - m0 : 0u;
    }
    s.ncells = G.ncells;
    s.n_rec = dev_mixed ? n_start + n_ops : n_start + n_new;  // upper bound on records (main + ghost)
    s.use_lds = m->sweep_lds;
    s.old_x = m->old_x;
    s.old_z = m->old_z;
    s.old_seq = m->old_seq;
    s.space_of = m->space_of;
    s.pos_x = m->pos_x;
    s.pos_z = m->pos_z;
    s.opq = m->opq;
    s.base = base;
    s.n_ops = n_ops;
    s.op_slot = a.op_slot;
    s.op_kind = a.op_kind;
    s.leave_ops = m->d_leaves;
    s.n_leaves = dev ? 0 : m->n_leaves;
    s.n_leaves_dev = dev_mixed ? m->ctr + gw::CTR_LEAVES : nullptr;
    s.leave_blocks = dev_mixed ? std::min<uint32_t>(256u, (n_ops + gw::sweep_block() - 1) / gw::sweep_block())
                               : (s.n_leaves + gw::sweep_block() - 1) / gw::sweep_block();
    s.ev_tmp = m->ev_tmp + F;
    s.ev_cap = m->tmp_cap - F;
    s.ev_fix = fixed ? m->ev_tmp : nullptr;
    s.tile_ev = m->tile_ev;
    s.tile_ent = m->tile_ent;
    s.rank_cnt = m->rank_cnt;
    s.uns = m->uns;
    s.ctr = m->ctr;
    s.dense = m->d_dense;
    s.dense_cap = m->cap;
    s.dense_hint = force_dense ? ~0u : m->last_dense;
    s.tile_walk = tile_build(G) ? m->tile_walk : nullptr;
    // the band walk's keys: built over this grid when k_sweep_dense runs (the previous pass had dense
    // movers, or this is the re-run that walks them)
    if (s.dense_hint && m->band_mode && !keys) RCHK(build_band_keys(m, ng, s.n_rec, &keys));
    // (after build_band_keys: it allocates the arrays, dense2 included, on first use)
    s.dense2 = keys ? m->band_dense2 : nullptr;
    s.g.rec = G.rec;  // (build_band_keys replaced it by the records sorted by x key inside each cell)
    s.band_xk = keys ? m->band_xk : nullptr;
    s.band_zk = keys ? m->band_zk : nullptr;
    s.band_zi = keys ? m->band_zi : nullptr;
    s.band_hd = keys ? m->band_hd : nullptr;
    s.band_tab = keys ? m->band_tab : nullptr;
    s.band_tab_half = m->band_tab_half;
    s.size_tiles = m->d_size_tiles;
    s.nspaces = m->nspaces;
    gw::launch_sweep(s, st);
    HIPCHK(hipGetLastError());
    if (m->timing) HIPCHK(hipEventRecord(m->tev[3], st));
    if (copy_events) RCHK(ensure_host_events(m, m->ev_cap, keep));
    // canonical order; every step is guarded on the device against a buffer overflow, so the host
    // synchronises once, at the end of the pass
    gw::launch_scan(m->scan, m->rank_cnt, n_ops + 1, st);
    gw::OrderArgs o{};
    o.g = {m->ctr, m->tmp_cap - F, keep, m->ev_cap};
    o.ev_tmp = m->ev_tmp + F;
    o.ev_fix = fixed ? m->ev_tmp : nullptr;
    o.tile_ev = m->tile_ev;
    o.tile_ent = m->tile_ent;
    o.ntiles_fix = fixed ? m->grid[ng].ntiles : 0u;
    o.scratch = reinterpret_cast<uint2*>(m->ev_tmp);
    o.rank_off = m->rank_cnt;
    o.uns = m->uns;
    o.ev_out = m->ev_out + keep;
    o.host_out = copy_events ? m->d_hev + keep : nullptr;
    o.n_ops = n_ops;
    o.zero_cs = m->grid[og].cs;  // the grid the next pass builds into (cell-atomic build only)
    o.zero_n = tile_build(m->grid[og]) ? 0u : m->grid[og].ncells + 1;
    o.ctr_next = m->ctr_buf + (m->ctr_sel ^ 1) * gw::CTR_N;
    o.grid_total = m->grid[ng].cs + m->grid[ng].ncells;
    o.op_slot = a.op_slot;
    o.opq = m->opq;
    o.base = base;
    o.cap = m->cap;
    // device batches: every op on a slot of its own, checked from k_bin_tsort's per-tile acted counts
    // (tile builds) or per op by k_slice_sort
    const bool tiles_check = dev && tile_build(m->grid[ng]);
    o.check_ops = dev && !tiles_check ? 1 : 0;
    o.tile_acted = m->tile_acted;
    o.ntiles_acted = tiles_check ? m->grid[ng].ntiles : 0u;
    o.n_dev = dev ? m->dv_count : nullptr;
    o.pub_seq = publish_seq(m, copy_events);
    o.pub = o.pub_seq ? m->d_pub : nullptr;
    o.sorted_hint = attempt == 0 && !m->last_unsorted && !o.check_ops ? 1 : 0;
    gw::launch_order(o, st);
    HIPCHK(hipGetLastError());
    if (m->timing) HIPCHK(hipEventRecord(m->tev[4], st));
    RCHK(finish_pass(m, o.pub_seq));
    if (m->h_ctr[gw::CTR_ERR]) {
      m->broken = true;
      set_err("device-staged batch failed validation (flags 0x%x: 1=duplicate slot, 2=absent slot, 4=slot >= "
              "capacity, 8=Enter of a present slot, 16=Space id out of range, 32=op count above its bound, "
              "64=non-finite coordinate); the manager is unusable",
              m->h_ctr[gw::CTR_ERR]);
      return GWAOI_ERR_DEVICE_CHECK;
    }
    if (m->h_ctr[gw::CTR_BOVF]) {  // (the sweep saw an empty grid)
      if (build_rr++ < 2) {
        rebuild = true;
        continue;
      }
      set_err("tile build overflow persisted");
      return GWAOI_ERR_NOMEM;
    }
    if (m->h_ctr[gw::CTR_DENSE] && !s.dense_hint) {  // dense movers nobody walked: the sweep again, with them
      if (dense_rr++ < 1) {
        force_dense = true;
        m->dense_reruns++;
        continue;
      }
      set_err("dense movers left unwalked");
      return GWAOI_ERR_STATE;
    }
    const uint32_t slots = m->h_ctr[gw::CTR_EVENTS], nev = m->h_ctr[gw::CTR_NEV];
    if (slots > m->tmp_cap - F || keep + nev > m->ev_cap) {
      RCHK(ensure_events(m, keep + nev, F + slots, keep, copy_events));
      if (ev_rr++ < 3) continue;
      set_err("event buffer overflow persisted");
      return GWAOI_ERR_NOMEM;
    }
    m->tick_events += nev;
    m->tick_enter += m->h_ctr[gw::CTR_ENTER];
    if (m->timing) {  // read the hipEvents later (collect_timing): waiting on them here costs latency
      m->tpend.pending = true;
      m->tpend.n_ops = m->h_ctr[gw::CTR_NOPS];
      m->tpend.nev = nev;
      m->tpend.records = m->h_ctr[gw::CTR_RECORDS];
      m->tpend.ncells = m->grid[ng].ncells;
      m->tpend.dense = m->h_ctr[gw::CTR_DENSE];
      m->tpend.band = m->h_ctr[gw::CTR_BAND_MV];
    }
    break;
  }
  m->cur = ng;
  m->passes_run++;
  m->grid[og].cs_zeroed = tile_build(m->grid[og]) ? 0u : m->grid[og].ncells + 1;
  m->ctr_sel ^= 1;
  m->ctr = m->ctr_buf + m->ctr_sel * gw::CTR_N;
  m->tick_passes++;
  m->tick_ops += m->h_ctr[gw::CTR_NOPS];
  m->n_ops = 0;
  m->n_leaves = 0;
  m->dv_n = 0;
  m->dv_slot = nullptr;
  m->dv_x = m->dv_z = nullptr;
  m->pass_id++;
  if (dev_mixed) m->n_present += m->h_ctr[gw::CTR_PRESENT];  // signed delta, two's complement
  m->last_dense = m->h_ctr[gw::CTR_DENSE];
  m->band_movers += m->h_ctr[gw::CTR_BAND_MV];
  m->last_unsorted = m->h_ctr[gw::CTR_UNSORTED] != 0 || m->h_ctr[gw::CTR_UNS_SOME] != 0;
  m->n_present_dev = m->n_present;
  m->dv_kind = nullptr;
  m->dv_space = nullptr;
  m->dv_count = nullptr;
  return GWAOI_OK;
}

int run_pass(gwaoi_mgr* m, bool copy_events);  // run_pass_core + the verdict of an async pinned batch

// Non-finite coordinates are refused (GWAOI_ERR_INVALID). go-aoi accepts them, and a NaN node in its
// sorted lists stops every Mark walk that reaches it, so third parties lose neighbours (the list
// restatement in the test suite reproduces that); that behaviour depends on list position, not
// on positions, and is not what a game wants from a client float. Deliberate divergence.
int check_coord(const char* what, uint32_t slot, float x, float z) {
  if (std::isfinite(x) && std::isfinite(z)) return GWAOI_OK;
  set_err("%s: slot %u: non-finite coordinate (%g, %g) refused", what, slot, (double)x, (double)z);
  return GWAOI_ERR_INVALID;
}

int check_mgr(const gwaoi_mgr* m) {
  if (!m) {
    set_err("null manager");
    return GWAOI_ERR_INVALID;
  }
  if (m->broken) {
    set_err("manager is unusable after a failed device-staged batch");
    return GWAOI_ERR_STATE;
  }
  return GWAOI_OK;
}

int host_staging_ok(const gwaoi_mgr* m) {
  if (m->dev_managed) {
    set_err("this manager takes mixed device batches (gwaoi_stage_ops_device): its presence state is on the "
            "device, host-staged Enter/Leave/Moved are not accepted");
    return GWAOI_ERR_STATE;
  }
  return GWAOI_OK;
}

int set_dev(const gwaoi_mgr* m) {
  HIPCHK(hipSetDevice(m->device));
  return GWAOI_OK;
}

// Before staging an op on `slot`: a slot may appear once per pass; a second op flushes the batch.
int before_stage(gwaoi_mgr* m, uint32_t slot) {
  if (m->dv_n) RCHK(run_pass(m, true));
  if (m->h_stamp[slot] == m->pass_id) RCHK(run_pass(m, true));
  return GWAOI_OK;
}

void note_coord(gwaoi_mgr* m, uint32_t space, float x, float z) {
  SpaceHost& sh = m->spaces[space];
  if (!sh.auto_extent) return;
  if (!std::isfinite(x) || !std::isfinite(z)) return;
  if (!sh.seen_any) {
    sh.seen_minx = sh.seen_maxx = x;
    sh.seen_minz = sh.seen_maxz = z;
    sh.seen_any = true;
    m->geom_dirty = true;
    return;
  }
  sh.seen_minx = std::min(sh.seen_minx, x);
  sh.seen_maxx = std::max(sh.seen_maxx, x);
  sh.seen_minz = std::min(sh.seen_minz, z);
  sh.seen_maxz = std::max(sh.seen_maxz, z);
  if (x < sh.gx0 || x > sh.gx1 || z < sh.gz0 || z > sh.gz1) m->geom_dirty = true;
}

// ---- pinned staging: DMA, device checks, and the deferred verdict of the async path ----------------------
// entries [from, to) of the pinned arrays into the op arrays (asynchronous, on the manager's stream)
int pin_copy(gwaoi_mgr* m, uint32_t from, uint32_t to) {
  if (to <= from) return GWAOI_OK;
  const size_t k = to - from;
  hipStream_t st = m->stream;
  HIPCHK(hipMemcpyAsync(m->d_op_slot + from, m->h_pin_slot + from, k * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(m->d_op_x + from, m->h_pin_x + from, k * sizeof(float), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(m->d_op_z + from, m->h_pin_z + from, k * sizeof(float), hipMemcpyHostToDevice, st));
  return GWAOI_OK;
}

bool pin_any_auto(const gwaoi_mgr* m) {
  for (const SpaceHost& sh : m->spaces)
    if (sh.auto_extent) return true;
  return false;
}

// k_pin_check / k_pin_cut over ops [seg, n) of the batch in d_op_* (validate: the batch's first check, over
// all of it); with `count`, k_pin_count keeps the verdict on the device (the async path)
int pin_launch(gwaoi_mgr* m, uint32_t n, uint32_t seg, int validate, bool count) {
  hipStream_t st = m->stream;
  const bool any_auto = pin_any_auto(m);
  if (any_auto && validate) {  // the extent each auto-extent Space's grid covers (beyond it: reported)
    const float inf = std::numeric_limits<float>::infinity();
    for (uint32_t sp = 0; sp < m->nspaces; ++sp) {
      const SpaceHost& sh = m->spaces[sp];
      m->h_pin_ext[sp] = sh.auto_extent ? (sh.seen_any ? make_float4(sh.gx0, sh.gz0, sh.gx1, sh.gz1)
                                                       : make_float4(inf, inf, -inf, -inf))  // nothing seen yet
                                        : make_float4(-inf, -inf, inf, inf);
    }
    HIPCHK(hipMemcpyAsync(m->d_pin_ext, m->h_pin_ext, m->nspaces * sizeof(float4), hipMemcpyHostToDevice, st));
  }
  if (++m->pin_id == 0) {  // ids wrapped: forget every stored id
    HIPCHK(hipMemsetAsync(m->d_pin_first, 0, (size_t)m->cap * sizeof(unsigned long long), st));
    m->pin_id = 1;
  }
  gw::PinCheckArgs a{};
  a.slot = m->d_op_slot;
  a.x = m->d_op_x;
  a.z = m->d_op_z;
  a.n = n;
  a.seg = seg;
  a.cap = m->cap;
  a.seq = m->seq;
  a.space_of = m->space_of;
  a.first = m->d_pin_first;
  a.ext = any_auto && validate ? m->d_pin_ext : nullptr;
  a.seen = m->d_pin_seen;
  a.out = m->d_pin_out;
  a.id = m->pin_id;
  a.validate = validate;
  gw::launch_pin_check(a, validate && a.ext && m->pin_seen_dirty, m->nspaces, st);
  if (count) gw::launch_pin_count(m->d_pin_out, n, seg, validate, m->d_pin_n, m->d_pin_v, st);
  HIPCHK(hipGetLastError());
  return GWAOI_OK;
}

// the check's report of coordinates beyond an auto-extent Space's grid: widen what the Space has seen
int pin_note_extent(gwaoi_mgr* m, uint32_t beyond) {
  m->pin_seen_dirty = beyond != 0;
  if (!beyond) return GWAOI_OK;
  uint32_t* k = m->h_pin_out + 4;
  HIPCHK(hipMemcpyAsync(k, m->d_pin_seen, 4 * sizeof(uint32_t) * m->nspaces, hipMemcpyDeviceToHost, m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  for (uint32_t sp = 0; sp < m->nspaces; ++sp) {
    if (!m->spaces[sp].auto_extent || k[4 * sp] > k[4 * sp + 2]) continue;  // none beyond
    note_coord(m, sp, gw::ord_float(k[4 * sp]), gw::ord_float(k[4 * sp + 1]));
    note_coord(m, sp, gw::ord_float(k[4 * sp + 2]), gw::ord_float(k[4 * sp + 3]));
  }
  return GWAOI_OK;
}

int pin_refused(const uint32_t* o) {
  set_err("stage_moves_pinned: entry %u refused (flags 0x%x: 2=slot not in a Space, 4=slot >= capacity, "
          "64=non-finite coordinate); nothing staged",
          o[2], o[0]);
  return (o[0] & (gw::ERR_BAD_SLOT | gw::ERR_BAD_COORD)) ? GWAOI_ERR_INVALID : GWAOI_ERR_STATE;
}

// The pipeline pass, plus the deferred verdict of an async pinned batch: the pass ran as a device-counted
// batch of the sub-pass's ops (none when the check refused the batch); after its end-of-pass sync the check's
// words are in mapped host memory: a refusal is reported now (nothing of the batch was applied), coordinates
// beyond an auto-extent Space widen its extent for the next pass (clamped cells keep this one exact), and a
// repeated slot starts the next sub-pass at the repeat (checked again from there), as the sync path does.
int run_pass(gwaoi_mgr* m, bool copy_events) {
  if (!m->pin_pending) return run_pass_core(m, copy_events);
  for (;;) {
    const int r = run_pass_core(m, copy_events);
    if (r) {
      m->pin_pending = false;
      return r;
    }
    uint32_t o[4];
    std::memcpy(o, (const void*)m->h_pin_v, sizeof(o));
    if (m->pin_validated) {
      if (o[0]) {
        m->pin_pending = false;
        return pin_refused(o);
      }
      RCHK(pin_note_extent(m, o[3]));
      m->pin_validated = false;
    }
    const uint32_t n = m->pin_n, cut = std::min(o[1], n);
    if (cut >= n) {
      m->pin_pending = false;
      return GWAOI_OK;
    }
    // op `cut` repeats a slot of the sub-pass that ran: the rest of the batch from there
    RCHK(pin_launch(m, n, cut, 0, true));
    m->dv_slot = m->d_op_slot + cut;
    m->dv_x = m->d_op_x + cut;
    m->dv_z = m->d_op_z + cut;
    m->dv_count = m->d_pin_n;
    m->dv_n = n - cut;
  }
}

void stage(gwaoi_mgr* m, uint32_t slot, uint8_t kind, float x, float z, uint32_t space) {
  const uint32_t i = m->n_ops++;
  m->h_op_slot[i] = slot;
  m->h_op_x[i] = x;
  m->h_op_z[i] = z;
  m->h_op_kind[i] = kind;
  m->h_op_space[i] = space;
  if (kind == gw::OP_LEAVE) m->h_leaves[m->n_leaves++] = i;
  m->h_stamp[slot] = m->pass_id;
}

void free_all(gwaoi_mgr* m) {
  hipSetDevice(m->device);
  if (m->stream) hipStreamSynchronize(m->stream);
  gw::sync_free(m->sync);
  m->sync = nullptr;
  void* dptrs[] = {m->pos_x, m->pos_z, m->old_x, m->old_z, m->seq, m->space_of, m->old_seq, m->opq,
                   m->key_of, m->local_of, m->d_op_slot, m->d_op_space, m->d_leaves, m->d_dense, m->d_op_x, m->d_op_z,
                   m->d_op_kind, m->rank_cnt, m->uns, m->part, m->thist, m->ttot, m->tstart, m->ctr_buf, m->ev_tmp, m->ev_out,
                   m->rel_rp, m->rel_cols, m->rel_tmp, m->tile_walk, m->tile_acted, m->band_xk, m->band_zi, m->band_hd, m->band_dense2, m->band_tab, m->ov_tag, m->ov_idx, m->ov_rec, m->ov_count, m->tile_ev, m->tile_ent, m->rel_tot, m->rel_tstat, m->rel_slab, m->rel_fix,
                   m->rel_rp2, m->rel_dn, m->rel_dch, m->d_pin_first, m->d_pin_out,
                   m->d_pin_seen, m->d_pin_ext, m->d_pin_n, m->d_size_tiles, m->dx_keys, m->dx_cnt, m->dx_last, m->dx_slot, m->dx_flags,
                   m->dx_part, m->dx_out};
  for (void* p : dptrs)
    if (p) hipFree(p);
  for (int gi = 0; gi < 2; ++gi) {
    Grid& g = m->grid[gi];
    void* gp[] = {g.rec, g.cs, g.d_geom, g.d_tile_space};
    for (void* p : gp)
      if (p) hipFree(p);
  }
  void* hptrs[] = {m->h_op_slot, m->h_op_x, m->h_op_z, m->h_op_kind, m->h_op_space, m->h_leaves, m->h_ctr,
                   m->h_ev, m->h_pub, m->h_pin_slot, m->h_pin_x, m->h_pin_z, m->h_pin_out, m->h_pin_ext, m->h_pin_v};
  for (void* p : hptrs)
    if (p) hipHostFree(p);
  for (auto& e : m->tev)
    if (e) hipEventDestroy(e);
  if (m->own_stream) hipStreamDestroy(m->own_stream);
}

int create_impl(const gwaoi_space_desc* spaces, uint32_t nspaces, uint32_t capacity, int device,
                gwaoi_mgr** out) {
  // slots live in a grid record's 30-bit slot field, and op ranks (< capacity) below the sweep's
  // kNoRank (2^30 - 1)
  if (!out || !spaces || !nspaces || !capacity || capacity > 0x3fffffffu) {
    set_err("gwaoi_create: invalid argument (capacity must be 1 .. 2^30 - 1)");
    return GWAOI_ERR_INVALID;
  }
  *out = nullptr;
  for (uint32_t s = 0; s < nspaces; ++s) {
    if (!(spaces[s].dist > 0) || !std::isfinite(spaces[s].dist)) {
      set_err("space %u: AOI distance must be > 0 (Space.EnableAOI panics otherwise, Space.go:92-94)", s);
      return GWAOI_ERR_INVALID;
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_err("no HIP device available");
    return GWAOI_ERR_HIP;
  }
  if (device < 0 || device >= ndev) {
    set_err("device %d out of range (%d devices)", device, ndev);
    return GWAOI_ERR_INVALID;
  }
  gwaoi_mgr* m = new (std::nothrow) gwaoi_mgr();
  if (!m) return GWAOI_ERR_NOMEM;
  m->device = device;
  m->cap = capacity;
  m->nspaces = nspaces;
  m->spaces.resize(nspaces);
  for (uint32_t s = 0; s < nspaces; ++s) {
    SpaceHost& sh = m->spaces[s];
    std::memset(&sh, 0, sizeof sh);
    sh.desc = spaces[s];
    sh.auto_extent = !(spaces[s].max_x > spaces[s].min_x && spaces[s].max_z > spaces[s].min_z);
  }
  m->max_cells = (uint32_t)std::min<uint64_t>(0x7fff0000u, std::max<uint64_t>(4096, (uint64_t)GW_CELLS_PER_SLOT * capacity) +
                                                             (uint64_t)gw::kTileCells * nspaces);
  m->h_present.assign(capacity, 0);
  m->h_space_of.assign(capacity, 0);
  m->h_stamp.assign(capacity, 0);
  int r = GWAOI_OK;
  auto chk = [&](int x) {
    if (r == GWAOI_OK) r = x;
  };
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&m->own_stream, hipStreamNonBlocking) != hipSuccess) {
    set_err("stream creation failed on device %d", device);
    delete m;
    return GWAOI_ERR_HIP;
  }
  m->stream = m->own_stream;
  const size_t C = capacity;
  chk(dalloc(&m->pos_x, C));
  chk(dalloc(&m->pos_z, C));
  chk(dalloc(&m->old_x, C));
  chk(dalloc(&m->old_z, C));
  chk(dalloc(&m->seq, C));
  chk(dalloc(&m->space_of, C));
  chk(dalloc(&m->old_seq, C));
  chk(dalloc(&m->opq, C));
  chk(dalloc(&m->key_of, 2 * C));
  chk(dalloc(&m->local_of, 2 * C));
  chk(dalloc(&m->d_op_slot, C));
  chk(dalloc(&m->d_op_space, C));
  chk(dalloc(&m->d_leaves, C));
  chk(dalloc(&m->d_dense, C));
  m->ov_cap = (uint32_t)std::min<size_t>(C, kOverlayCap);
  chk(dalloc(&m->ov_tag, C));
  chk(dalloc(&m->ov_idx, C));
  chk(dalloc(&m->ov_rec, m->ov_cap));
  chk(dalloc(&m->ov_count, 1));
  if (r == GWAOI_OK) chk(hipMemset(m->ov_tag, 0, C * sizeof(uint32_t)) == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP);
  if (r == GWAOI_OK) chk(hipMemset(m->ov_count, 0, sizeof(uint32_t)) == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP);
  chk(dalloc(&m->d_op_x, C));
  chk(dalloc(&m->d_op_z, C));
  chk(dalloc(&m->d_op_kind, C));
  chk(dalloc(&m->rank_cnt, C + 1));
  chk(dalloc(&m->uns, C / 32 + 2));
  if (r == GWAOI_OK) chk(hipMemset(m->uns, 0, (C / 32 + 2) * sizeof(uint32_t)) == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP);
  m->nblk = (capacity + gw::bin_chunk(capacity) - 1) / gw::bin_chunk(capacity);
  const uint64_t max_tiles = m->max_cells / gw::kTileCells + 1;
  const uint64_t thist_n = std::min<uint64_t>(max_tiles, gw::kMaxLdsTiles) * m->nblk + 1;
  chk(dalloc(&m->thist, thist_n));
  chk(dalloc(&m->ttot, 2 * (size_t)gw::kMaxLdsTiles));  // k_bin_tscatter zeroes kMaxLdsTiles of the other buffer
  chk(dalloc(&m->tstart, 2 * ((size_t)gw::kMaxLdsTiles + 1)));
  chk(dalloc(&m->tile_walk, std::min<uint64_t>(max_tiles, gw::kMaxLdsTiles)));
  chk(dalloc(&m->tile_acted, std::min<uint64_t>(max_tiles, gw::kMaxLdsTiles)));
  chk(dalloc(&m->tile_ev, std::min<uint64_t>(max_tiles, gw::kMaxLdsTiles)));
  chk(dalloc(&m->tile_ent, std::min<uint64_t>(max_tiles, gw::kMaxLdsTiles)));
  // the scan has at most 1024 chunks up to 16.7M items (scan_ipt), more beyond
  m->part_words = std::max<uint32_t>(1024 + 2, gw::scan_part_words((uint32_t)std::max<uint64_t>(
                                                   {(uint64_t)m->max_cells, (uint64_t)capacity, thist_n}) + 1));
  chk(dalloc(&m->part, m->part_words));
  m->scan.status = m->part;
  chk(dalloc(&m->ctr_buf, 2 * gw::CTR_N));
  m->ctr = m->ctr_buf;
  chk(halloc(&m->h_ctr, gw::CTR_N));
  if (r == GWAOI_OK) {
    void* dp = nullptr;
    if (hipHostMalloc((void**)&m->h_pub, (gw::kPubWords + 1) * sizeof(uint32_t),
                      hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
        hipHostGetDevicePointer(&dp, m->h_pub, 0) == hipSuccess) {
      m->d_pub = (uint32_t*)dp;
      std::memset(m->h_pub, 0, (gw::kPubWords + 1) * sizeof(uint32_t));
    } else {  // the DMA-copy path below still works
      (void)hipGetLastError();
      if (m->h_pub) (void)hipHostFree(m->h_pub);
      m->h_pub = nullptr;
    }
  }
  chk(halloc(&m->h_op_slot, C));
  chk(halloc(&m->h_op_x, C));
  chk(halloc(&m->h_op_z, C));
  chk(halloc(&m->h_op_kind, C));
  chk(halloc(&m->h_op_space, C));
  chk(halloc(&m->h_leaves, C));
  if (r == GWAOI_OK) {
    void *ps = nullptr, *px = nullptr, *pz = nullptr, *pk = nullptr, *pp = nullptr;
    if (hipHostGetDevicePointer(&ps, m->h_op_slot, 0) == hipSuccess &&
        hipHostGetDevicePointer(&px, m->h_op_x, 0) == hipSuccess &&
        hipHostGetDevicePointer(&pz, m->h_op_z, 0) == hipSuccess &&
        hipHostGetDevicePointer(&pk, m->h_op_kind, 0) == hipSuccess &&
        hipHostGetDevicePointer(&pp, m->h_op_space, 0) == hipSuccess) {
      m->hd_op_slot = (const uint32_t*)ps;
      m->hd_op_x = (const float*)px;
      m->hd_op_z = (const float*)pz;
      m->hd_op_kind = (const uint8_t*)pk;
      m->hd_op_space = (const uint32_t*)pp;
    } else {
      (void)hipGetLastError();  // the small pass copies the ops instead
    }
  }
  for (int gi = 0; gi < 2; ++gi) {
    Grid& g = m->grid[gi];
    chk(dalloc(&g.rec, 2 * C));
    chk(dalloc(&g.cs, (size_t)m->max_cells + 1));
    chk(dalloc(&g.d_geom, nspaces));
    chk(dalloc(&g.d_tile_space, (size_t)m->max_cells / gw::kTileCells + 1));
  }
  static bool sweep_ready = false;
  if (!sweep_ready) {
    gw::sweep_init();
    sweep_ready = true;
  }
  if (r == GWAOI_OK)
    r = ensure_events(m, std::max<uint64_t>(1u << 16, C / 2), (uint32_t)std::max<uint64_t>(1u << 16, C / 2), 0, false);
  for (auto& e : m->tev)
    if (r == GWAOI_OK && hipEventCreate(&e) != hipSuccess) {
      set_err("hipEventCreate failed");
      r = GWAOI_ERR_HIP;
    }
  if (r == GWAOI_OK) {
    hipStream_t st = m->stream;
    auto z = [&](void* p, size_t bytes) {
      if (r == GWAOI_OK && hipMemsetAsync(p, 0, bytes, st) != hipSuccess) {
        set_err("hipMemsetAsync failed");
        r = GWAOI_ERR_HIP;
      }
    };
    z(m->ctr_buf, 2 * gw::CTR_N * 4);
    z(m->pos_x, C * 4);
    z(m->opq, C * 4);
    z(m->pos_z, C * 4);
    z(m->seq, C * 4);
    z(m->space_of, C * 4);
    z(m->ttot, 2 * (size_t)gw::kMaxLdsTiles * 4);
    std::vector<gw::Geom> geo;
    compute_geometry(m, geo);
    m->geom_dirty = false;
    for (int gi = 0; gi < 2 && r == GWAOI_OK; ++gi) {
      r = upload_geom(m, m->grid[gi], geo);
      z(m->grid[gi].cs, ((size_t)m->grid[gi].ncells + 1) * 4);
    }
    if (r == GWAOI_OK && hipStreamSynchronize(st) != hipSuccess) {
      set_err("initialisation failed");
      r = GWAOI_ERR_HIP;
    }
  }
  if (r != GWAOI_OK) {
    free_all(m);
    delete m;
    return r;
  }
  *out = m;
  return GWAOI_OK;
}

int pin_args_ok(gwaoi_mgr* m, uint32_t n, const char* what) {
  RCHK(check_mgr(m));
  RCHK(host_staging_ok(m));
  if (!m->h_pin_slot) {
    set_err("%s: no staging buffers (call gwaoi_stage_buffers first)", what);
    return GWAOI_ERR_STATE;
  }
  if (n > m->cap) {
    set_err("%s: %u moves > capacity %u", what, n, m->cap);
    return GWAOI_ERR_INVALID;
  }
  return set_dev(m);
}

}  // namespace

// ================================================================================================
// C ABI

namespace gw {

void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}

int mgr_view(gwaoi_mgr* m, MgrView* out) {
  RCHK(check_mgr(m));
  RCHK(set_dev(m));
  const Grid& g = m->grid[m->cur];
  out->device = m->device;
  out->stream = m->stream;
  out->cap = m->cap;
  out->g = {g.rec, g.cs, g.d_geom, g.d_tile_space};
  out->rec_count = g.cs ? g.cs + g.ncells : nullptr;
  out->rec_bound = 2 * m->cap;
  out->ncells = g.ncells;
  out->ntiles = g.ntiles;
  out->pos_x = m->pos_x;
  out->pos_z = m->pos_z;
  out->seq = m->seq;
  out->space_of = m->space_of;
  out->scan = &m->scan;
  out->sync = &m->sync;
  out->pending = m->n_ops || m->dv_n;
  out->index_limit = m->index_limit;
  out->timing = m->timing;
  return GWAOI_OK;
}

// Readers of the grid itself (the sync fan-out) call this before mgr_view: after small passes the grid
// lags their ops and is rebuilt from the slots' state. mgr_view stays free of side effects, so the sync
// setters and stats calls between single-op passes never rebuild it.
int mgr_grid_current(gwaoi_mgr* m) {
  RCHK(check_mgr(m));
  RCHK(set_dev(m));
  if (m->n_ops || m->dv_n) return GWAOI_OK;  // (staged ops: the caller flushes, then asks again)
  return ensure_grid_current(m);
}

int mgr_flush(gwaoi_mgr* m) {
  RCHK(check_mgr(m));
  RCHK(set_dev(m));
  if (m->n_ops || m->dv_n) RCHK(run_pass(m, true));
  return GWAOI_OK;
}

int mgr_stage_moves_device_n(gwaoi_mgr* m, const uint32_t* d_slots, const float* d_x, const float* d_z,
                             const uint32_t* d_n, uint32_t n_max) {
  RCHK(gwaoi_stage_moves_device(m, d_slots, d_x, d_z, n_max));
  m->dv_count = d_n;
  return GWAOI_OK;
}

}  // namespace gw

extern "C" {

#ifndef GWAOI_SRC_HASH
#define GWAOI_SRC_HASH "unstamped"
#endif
// the source stamp (goworld_amd/build.py source_hash) ties measurements to the build they came from
const char* gwaoi_version(void) { return "gwaoi 0.4.0 (gfx950, abi 2) src " GWAOI_SRC_HASH; }
int gwaoi_abi_version(void) { return GWAOI_ABI_VERSION; }
int gwaoi_abi_minor(void) { return GWAOI_ABI_MINOR; }
const char* gwaoi_last_error(void) { return g_err.c_str(); }

int gwaoi_create(float dist, uint32_t capacity, int device, gwaoi_mgr** out) {
  gwaoi_space_desc d = {dist, 0.f, 0.f, 0.f, 0.f};
  return create_impl(&d, 1, capacity, device, out);
}

int gwaoi_create_spaces(const gwaoi_space_desc* spaces, uint32_t nspaces, uint32_t capacity, int device,
                        gwaoi_mgr** out) {
  return create_impl(spaces, nspaces, capacity, device, out);
}

int gwaoi_destroy(gwaoi_mgr* m) {
  if (!m) return GWAOI_OK;
  free_all(m);
  delete m;
  return GWAOI_OK;
}

int gwaoi_set_stream(gwaoi_mgr* m, void* s) {
  if (!m) return GWAOI_ERR_INVALID;
  RCHK(set_dev(m));
  HIPCHK(hipStreamSynchronize(m->stream));
  m->stream = s ? (hipStream_t)s : m->own_stream;
  return GWAOI_OK;
}

int gwaoi_enter_space(gwaoi_mgr* m, uint32_t space, uint32_t slot, float x, float z) {
  RCHK(check_mgr(m));
  RCHK(host_staging_ok(m));
  if (slot >= m->cap || space >= m->nspaces) {
    set_err("enter: slot %u / space %u out of range", slot, space);
    return GWAOI_ERR_INVALID;
  }
  if (m->h_present[slot]) {
    set_err("enter: slot %u is already in a Space", slot);
    return GWAOI_ERR_STATE;
  }
  RCHK(check_coord("enter", slot, x, z));
  RCHK(set_dev(m));
  RCHK(before_stage(m, slot));
  note_coord(m, space, x, z);
  stage(m, slot, gw::OP_ENTER, x, z, space);
  m->h_present[slot] = 1;
  m->h_space_of[slot] = space;
  m->n_present++;
  return GWAOI_OK;
}

int gwaoi_enter(gwaoi_mgr* m, uint32_t slot, float x, float z) { return gwaoi_enter_space(m, 0, slot, x, z); }

int gwaoi_stage_enters(gwaoi_mgr* m, uint32_t space, const uint32_t* slots, const float* x, const float* z,
                       uint32_t n) {
  RCHK(check_mgr(m));
  if (n && (!slots || !x || !z)) {
    set_err("stage_enters: null array");
    return GWAOI_ERR_INVALID;
  }
  RCHK(host_staging_ok(m));
  // validate the whole array first: nothing is staged unless every entry is acceptable
  if (space >= m->nspaces) {
    set_err("stage_enters: space %u out of range", space);
    return GWAOI_ERR_INVALID;
  }
  std::vector<uint32_t> seen;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t s = slots[i];
    if (s >= m->cap) {
      set_err("stage_enters: entry %u: slot %u out of range", i, s);
      return GWAOI_ERR_INVALID;
    }
    RCHK(check_coord("stage_enters", s, x[i], z[i]));
    if (m->h_present[s]) {
      set_err("stage_enters: entry %u: slot %u is already in a Space", i, s);
      return GWAOI_ERR_STATE;
    }
    seen.push_back(s);
  }
  std::sort(seen.begin(), seen.end());
  if (std::adjacent_find(seen.begin(), seen.end()) != seen.end()) {
    set_err("stage_enters: a slot enters twice");
    return GWAOI_ERR_STATE;
  }
  for (uint32_t i = 0; i < n; ++i) RCHK(gwaoi_enter_space(m, space, slots[i], x[i], z[i]));
  return GWAOI_OK;
}

int gwaoi_leave(gwaoi_mgr* m, uint32_t slot) {
  RCHK(check_mgr(m));
  RCHK(host_staging_ok(m));
  if (slot >= m->cap) {
    set_err("leave: slot %u out of range", slot);
    return GWAOI_ERR_INVALID;
  }
  if (!m->h_present[slot]) {
    set_err("leave: slot %u is not in a Space", slot);
    return GWAOI_ERR_STATE;
  }
  RCHK(set_dev(m));
  RCHK(before_stage(m, slot));
  stage(m, slot, gw::OP_LEAVE, 0.f, 0.f, m->h_space_of[slot]);
  m->h_present[slot] = 0;
  m->n_present--;
  return GWAOI_OK;
}

int gwaoi_moved(gwaoi_mgr* m, uint32_t slot, float x, float z) {
  RCHK(check_mgr(m));
  RCHK(host_staging_ok(m));
  if (slot >= m->cap) {
    set_err("moved: slot %u out of range", slot);
    return GWAOI_ERR_INVALID;
  }
  if (!m->h_present[slot]) {
    set_err("moved: slot %u is not in a Space", slot);
    return GWAOI_ERR_STATE;
  }
  RCHK(check_coord("moved", slot, x, z));
  RCHK(set_dev(m));
  RCHK(before_stage(m, slot));
  note_coord(m, m->h_space_of[slot], x, z);
  stage(m, slot, gw::OP_MOVE, x, z, m->h_space_of[slot]);
  return GWAOI_OK;
}

int gwaoi_stage_moves(gwaoi_mgr* m, const uint32_t* slots, const float* x, const float* z, uint32_t n) {
  RCHK(check_mgr(m));
  if (n && (!slots || !x || !z)) {
    set_err("stage_moves: null array");
    return GWAOI_ERR_INVALID;
  }
  RCHK(host_staging_ok(m));
  // validate the whole array first (Moved changes no presence): all entries are staged or none
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t s = slots[i];
    if (s >= m->cap) {
      set_err("stage_moves: entry %u: slot %u out of range", i, s);
      return GWAOI_ERR_INVALID;
    }
    if (!m->h_present[s]) {
      set_err("stage_moves: entry %u: slot %u is not in a Space", i, s);
      return GWAOI_ERR_STATE;
    }
    RCHK(check_coord("stage_moves", s, x[i], z[i]));
  }
  if (!n) return GWAOI_OK;
  RCHK(set_dev(m));
  if (m->dv_n) RCHK(run_pass(m, true));
  // bulk path (the cgo wrapper's one call per tick): runs of entries without a repeated slot are
  // stamped, then copied into the pinned staging arrays; a repeated slot flushes the batch first
  // (sub-pass), exactly as gwaoi_moved would
  bool any_auto = false;
  for (const SpaceHost& sh : m->spaces) any_auto |= sh.auto_extent;
  uint32_t i = 0;
  while (i < n) {
    uint32_t e = i;
    const uint32_t room = m->cap - m->n_ops;  // a pass holds at most cap ops (one per slot)
    for (; e < n && e - i < room; ++e) {
      const uint32_t s = slots[e];
      if (m->h_stamp[s] == m->pass_id) break;
      m->h_stamp[s] = m->pass_id;
      m->h_op_space[m->n_ops + (e - i)] = m->h_space_of[s];
      if (any_auto) note_coord(m, m->h_space_of[s], x[e], z[e]);
    }
    const uint32_t k = e - i, o = m->n_ops;
    std::memcpy(m->h_op_slot + o, slots + i, (size_t)k * sizeof(uint32_t));
    std::memcpy(m->h_op_x + o, x + i, (size_t)k * sizeof(float));
    std::memcpy(m->h_op_z + o, z + i, (size_t)k * sizeof(float));
    std::memset(m->h_op_kind + o, gw::OP_MOVE, k);
    m->n_ops += k;
    i = e;
    if (i < n) RCHK(run_pass(m, true));  // slots[i] already has an op in this batch
  }
  return GWAOI_OK;
}

int gwaoi_stage_buffers(gwaoi_mgr* m, uint32_t** slots, float** x, float** z, uint32_t* capacity) {
  RCHK(check_mgr(m));
  if (!slots || !x || !z) {
    set_err("stage_buffers: null output");
    return GWAOI_ERR_INVALID;
  }
  RCHK(set_dev(m));
  if (!m->h_pin_slot) {
    const uint32_t ns = m->nspaces;
    int r = halloc(&m->h_pin_slot, m->cap);
    if (!r) r = halloc(&m->h_pin_x, m->cap);
    if (!r) r = halloc(&m->h_pin_z, m->cap);
    if (!r) r = halloc(&m->h_pin_out, 4 + 4 * (size_t)ns);
    if (!r) r = halloc(&m->h_pin_ext, ns);
    if (!r) r = dalloc(&m->d_pin_first, m->cap);
    if (!r) r = dalloc(&m->d_pin_out, 4);
    if (!r) r = dalloc(&m->d_pin_seen, 4 * (size_t)ns);
    if (!r) r = dalloc(&m->d_pin_ext, ns);
    if (!r) r = dalloc(&m->d_pin_n, 1);
    if (r) return r;  // freed with the manager
    // the async path's verdict words: mapped coherent host memory written by k_pin_count (without it,
    // gwaoi_stage_moves_pinned_async takes the synchronous path)
    void* dp = nullptr;
    if (hipHostMalloc((void**)&m->h_pin_v, 4 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) ==
            hipSuccess &&
        hipHostGetDevicePointer(&dp, m->h_pin_v, 0) == hipSuccess) {
      m->d_pin_v = (uint32_t*)dp;
    } else {
      (void)hipGetLastError();
      if (m->h_pin_v) (void)hipHostFree(m->h_pin_v);
      m->h_pin_v = nullptr;
    }
    HIPCHK(hipMemsetAsync(m->d_pin_first, 0, (size_t)m->cap * sizeof(unsigned long long), m->stream));
    m->pin_id = 0;
    m->pin_seen_dirty = true;
    m->pin_pushed = 0;
  }
  *slots = m->h_pin_slot;
  *x = m->h_pin_x;
  *z = m->h_pin_z;
  if (capacity) *capacity = m->cap;
  return GWAOI_OK;
}

// Incremental push: entries [pushed, upto) to the device now (asynchronous DMA), so the final call copies
// only the tail. Ops staged earlier run first, as they would at the final call (a pass of host ops would
// overwrite the device copy of what was pushed: pin_pushed restarts then).
int gwaoi_stage_moves_pinned_partial(gwaoi_mgr* m, uint32_t upto) {
  RCHK(pin_args_ok(m, upto, "stage_moves_pinned_partial"));
  if (m->n_ops || m->dv_n) RCHK(run_pass(m, true));
  if (upto < m->pin_pushed) {
    set_err("stage_moves_pinned_partial: %u entries < the %u already pushed", upto, m->pin_pushed);
    return GWAOI_ERR_INVALID;
  }
  RCHK(pin_copy(m, m->pin_pushed, upto));
  m->pin_pushed = upto;
  return GWAOI_OK;
}

// The Moved batch in the pinned buffers: one DMA copy (of what was not pushed yet), then k_pin_check
// validates it on the GPU and finds the first repeated slot; nothing changes unless the whole batch is
// acceptable. Runs of the batch without a repeat are staged as device batches (all but the last run as
// sub-passes now).
int gwaoi_stage_moves_pinned(gwaoi_mgr* m, uint32_t n) {
  RCHK(pin_args_ok(m, n, "stage_moves_pinned"));
  if (m->n_ops || m->dv_n) RCHK(run_pass(m, true));  // ops staged earlier come first
  const uint32_t pushed = std::min(m->pin_pushed, n);
  m->pin_pushed = 0;
  if (!n) return GWAOI_OK;
  hipStream_t st = m->stream;
  RCHK(pin_copy(m, pushed, n));
  uint32_t seg = 0;
  for (int validate = 1;; validate = 0) {
    RCHK(pin_launch(m, n, seg, validate, false));
    HIPCHK(hipMemcpyAsync(m->h_pin_out, m->d_pin_out, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint32_t* o = m->h_pin_out;
    if (validate && o[0]) return pin_refused(o);
    if (validate) RCHK(pin_note_extent(m, o[3]));
    const uint32_t cut = std::min(o[1], n);
    m->dv_slot = m->d_op_slot + seg;
    m->dv_x = m->d_op_x + seg;
    m->dv_z = m->d_op_z + seg;
    m->dv_n = cut - seg;
    if (cut >= n) break;
    RCHK(run_pass(m, true));  // op `cut` repeats a slot of this run: the run is a sub-pass
    seg = cut;
  }
  return GWAOI_OK;
}

// The same without the host round trip: the DMA copy, the checks and k_pin_count are enqueued, and the batch
// is staged as a device-counted batch whose count the check decides on the device. The verdict is read by
// the pass that runs it (run_pass): a refused batch applies nothing and that call (gwaoi_tick, or a call
// that flushes) returns the refusal; repeats split it into sub-passes there.
int gwaoi_stage_moves_pinned_async(gwaoi_mgr* m, uint32_t n) {
  RCHK(pin_args_ok(m, n, "stage_moves_pinned_async"));
  if (!m->h_pin_v) return gwaoi_stage_moves_pinned(m, n);  // no mapped verdict words: the sync path
  if (m->n_ops || m->dv_n) RCHK(run_pass(m, true));  // ops staged earlier come first
  const uint32_t pushed = std::min(m->pin_pushed, n);
  m->pin_pushed = 0;
  if (!n) return GWAOI_OK;
  RCHK(pin_copy(m, pushed, n));
  RCHK(pin_launch(m, n, 0, 1, true));
  m->pin_pending = true;
  m->pin_validated = true;
  m->pin_n = n;
  m->dv_slot = m->d_op_slot;
  m->dv_x = m->d_op_x;
  m->dv_z = m->d_op_z;
  m->dv_count = m->d_pin_n;
  m->dv_n = n;
  return GWAOI_OK;
}

int gwaoi_stage_moves_device(gwaoi_mgr* m, const uint32_t* d_slots, const float* d_x, const float* d_z,
                             uint32_t n) {
  RCHK(check_mgr(m));
  if (n && (!d_slots || !d_x || !d_z)) {
    set_err("stage_moves_device: null array");
    return GWAOI_ERR_INVALID;
  }
  if (n > m->cap) {
    set_err("stage_moves_device: %u ops > capacity %u", n, m->cap);
    return GWAOI_ERR_INVALID;
  }
  RCHK(set_dev(m));
  if (m->n_ops || m->dv_n) RCHK(run_pass(m, true));
  m->dv_slot = d_slots;
  m->dv_x = d_x;
  m->dv_z = d_z;
  m->dv_n = n;
  return GWAOI_OK;
}

int gwaoi_stage_ops_device(gwaoi_mgr* m, const uint32_t* d_slots, const float* d_x, const float* d_z,
                           const uint8_t* d_kinds, uint32_t n) {
  return gwaoi_stage_ops_device_spaces(m, d_slots, d_x, d_z, d_kinds, nullptr, n);
}

int gwaoi_stage_ops_device_spaces(gwaoi_mgr* m, const uint32_t* d_slots, const float* d_x, const float* d_z,
                                  const uint8_t* d_kinds, const uint32_t* d_spaces, uint32_t n) {
  return gwaoi_stage_ops_device_n(m, d_slots, d_x, d_z, d_kinds, d_spaces, nullptr, n);
}

int gwaoi_stage_ops_device_n(gwaoi_mgr* m, const uint32_t* d_slots, const float* d_x, const float* d_z,
                             const uint8_t* d_kinds, const uint32_t* d_spaces, const uint32_t* d_n, uint32_t n) {
  RCHK(check_mgr(m));
  if (n && (!d_slots || !d_x || !d_z || !d_kinds)) {
    set_err("stage_ops_device: null array");
    return GWAOI_ERR_INVALID;
  }
  if (n > m->cap) {
    set_err("stage_ops_device: %u ops > capacity %u", n, m->cap);
    return GWAOI_ERR_INVALID;
  }
  RCHK(set_dev(m));
  if (m->n_ops || m->dv_n) RCHK(run_pass(m, true));
  m->dev_managed = true;
  m->dv_slot = d_slots;
  m->dv_x = d_x;
  m->dv_z = d_z;
  m->dv_kind = d_kinds;
  m->dv_space = d_spaces;
  m->dv_count = d_n;
  m->dv_n = n;
  return GWAOI_OK;
}

int gwaoi_adopt_device_state(gwaoi_mgr* m) {
  RCHK(check_mgr(m));
  RCHK(set_dev(m));
  if (m->n_ops || m->dv_n) {
    set_err("adopt_device_state: ops are staged; run gwaoi_tick first");
    return GWAOI_ERR_STATE;
  }
  std::vector<uint32_t> q(m->cap), sp(m->cap);
  HIPCHK(hipStreamSynchronize(m->stream));
  HIPCHK(hipMemcpy(q.data(), m->seq, (size_t)m->cap * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(sp.data(), m->space_of, (size_t)m->cap * sizeof(uint32_t), hipMemcpyDeviceToHost));
  uint32_t np = 0;
  for (uint32_t s = 0; s < m->cap; ++s) {
    m->h_present[s] = q[s] != 0;
    m->h_space_of[s] = sp[s];
    np += q[s] != 0;
  }
  m->n_present = m->n_present_dev = np;
  m->dev_managed = false;
  return GWAOI_OK;
}

int gwaoi_tick_ex(gwaoi_mgr* m, uint32_t flags, gwaoi_events* out) {
  RCHK(check_mgr(m));
  RCHK(set_dev(m));
  const bool copy = !(flags & GWAOI_TICK_DEVICE_EVENTS);
  // Passes forced earlier by re-staging a slot (before_stage) already accumulated their events.
  int r = run_pass(m, copy);
  if (r) return r;
  if (!m->acc_open) reset_tick(m);  // nothing ran since the last tick
  m->acc_open = false;
  m->dx_ready = true;
  m->dx_silent = m->acc_silent;
  m->dx_events = m->tick_events;
  if (out) {
    out->events = copy ? m->h_ev : (const gwaoi_event*)m->ev_out;
    out->count = m->tick_events;
    out->n_enter = m->tick_enter;
    out->n_leave = m->tick_events - m->tick_enter;
    out->n_subticks = m->tick_passes;
    out->n_ops = m->tick_ops;
  }
  return GWAOI_OK;
}

int gwaoi_tick(gwaoi_mgr* m, gwaoi_events* out) { return gwaoi_tick_ex(m, 0, out); }

int gwaoi_count(const gwaoi_mgr* m, uint32_t* n_present, uint32_t* n_staged) {
  if (!m) return GWAOI_ERR_INVALID;
  if (n_present) *n_present = m->n_present;
  if (n_staged) *n_staged = m->dv_n ? m->dv_n : m->n_ops;
  return GWAOI_OK;
}

namespace {

// The view after the current accumulation's passes, from the view before them and their events
// (the replay sink maintained from the events instead of rebuilt from positions).
// Returns GWAOI_OK with *done = false when the events do not allow it (a row with too many
// changes): the caller rebuilds from the grid. Costs one small read-back (the flag).
int relation_delta(gwaoi_mgr* m, bool* done) {
  *done = false;
  hipStream_t st = m->stream;
  const uint64_t nev = m->tick_events;
  const uint64_t bound = m->rel_nnz + 2 * nev;  // every event an ENTER: the most the view can grow to
  m->rel_why = 6;
  if (bound > m->index_limit) return GWAOI_OK;
  const size_t n1 = (size_t)m->cap + 1;
  if (!m->rel_rp2) RCHK(dalloc(&m->rel_rp2, n1));
  if (!m->rel_dn) {  // one allocation, zeroed by one memset: change counts, row cursors, flags
    RCHK(dalloc(&m->rel_dn, 2 * n1 + 2));
    m->rel_dcur = m->rel_dn + n1;
    m->rel_flag = m->rel_dn + 2 * n1;  // [0] flag, [1] long rows
  }
  if (2 * nev > m->rel_dch_cap) {
    if (m->rel_dch) hipFree(m->rel_dch);
    m->rel_dch = nullptr;
    m->rel_dch_cap = 0;
    const uint64_t want = 2 * nev + nev / 2 + 4096;
    // changes, their rows, the sign prefixes of long rows, the long rows (at most want / 32 of them)
    RCHK(dalloc(&m->rel_dch, 3 * want + want / 32 + 1));
    m->rel_dch_cap = want;
  }
  if (bound > m->rel_tmp_cap) {
    if (m->rel_tmp) hipFree(m->rel_tmp);
    m->rel_tmp = nullptr;
    m->rel_tmp_cap = 0;
    const uint64_t want = bound + m->rel_nnz / 4 + 1024;
    RCHK(dalloc(&m->rel_tmp, want));
    m->rel_tmp_cap = want;
  }
  gw::RelDeltaArgs a{};
  a.ev = m->ev_out;
  a.nev = (uint32_t)nev;
  a.cap = m->cap;
  a.rp_old = m->rel_rp;
  a.cols_old = m->rel_cols;
  a.dn = m->rel_dn;
  a.dcur = m->rel_dcur;
  a.dch = m->rel_dch;
  a.dchrow = m->rel_dch + m->rel_dch_cap;
  a.rp_new = m->rel_rp2;
  a.cols_new = m->rel_tmp;
  a.cols_cap = m->rel_tmp_cap;
  a.flag = m->rel_flag;
  a.psum = reinterpret_cast<int32_t*>(m->rel_dch + 2 * m->rel_dch_cap);
  a.longrows = m->rel_dch + 3 * m->rel_dch_cap;
  a.nlong = m->rel_flag + 1;
  a.long_cap = (uint32_t)(m->rel_dch_cap / 32 + 1);
  HIPCHK(hipMemsetAsync(m->rel_dn, 0, (2 * n1 + 2) * sizeof(uint32_t), st));
  gw::launch_rel_delta_count(a, st);
  gw::launch_scan(m->scan, m->rel_dn, m->cap + 1, st);
  gw::launch_rel_delta_apply(a, m->scan, st);
  HIPCHK(hipGetLastError());
  uint32_t w[2] = {0, 0};
  RCHK(read_words(m, m->rel_flag, 1, m->rel_rp2 + m->cap, 1, w));
  const uint32_t flag = w[0], nnz_new = w[1];
  m->rel_why = 7;
  if (flag) return GWAOI_OK;
  m->rel_why = 8;
  // the events are exactly the relation's changes: the new size is the old one plus twice the net
  // enters (a mismatch would mean a broken event stream: rebuild rather than trust it)
  const int64_t expect = (int64_t)m->rel_nnz + 2 * ((int64_t)m->tick_enter - (int64_t)(nev - m->tick_enter));
  if (expect != (int64_t)nnz_new) return GWAOI_OK;
  std::swap(m->rel_rp, m->rel_rp2);
  std::swap(m->rel_cols, m->rel_tmp);
  std::swap(m->rel_cap, m->rel_tmp_cap);
  m->rel_nnz = nnz_new;
  *done = true;
  return GWAOI_OK;
}

}  // namespace

int gwaoi_relation_device(gwaoi_mgr* m, gwaoi_relation_view* out) {
  RCHK(check_mgr(m));
  if (!out) {
    set_err("relation_device: null argument");
    return GWAOI_ERR_INVALID;
  }
  RCHK(set_dev(m));
  bool flushed = false;
  if (m->n_ops || m->dv_n) {
    RCHK(run_pass(m, false));
    flushed = true;
  }
  // events of a batch flushed here are discarded (documented in gwaoi.h), after the view used them
  struct Discard {
    gwaoi_mgr* m;
    bool on;
    ~Discard() {
      if (on) {
        m->acc_open = false;
        reset_tick(m);
      }
    }
  } discard{m, flushed};
  if (m->rel_valid && m->rel_mode == 0 && m->rel_passes == m->passes_run) {  // nothing ran since the view
    out->row_ptr = m->rel_rp;
    out->cols = m->rel_cols;
    out->nnz = m->rel_nnz;
    return GWAOI_OK;
  }
  // Incremental when every pass since the view is in the open accumulation, none applied SILENT ops,
  // and the events are not many against the relation (the update copies the whole view once).
  m->rel_why = !m->rel_valid ? 1 : m->rel_mode ? 2 : m->acc_base != m->rel_passes ? 3 : m->acc_silent ? 4
               : m->tick_events > m->rel_nnz / 2 + 65536 ? 5 : 0;
  if (m->rel_why == 0) {
    bool done = false;
    RCHK(relation_delta(m, &done));
    if (done) {
      m->rel_passes = m->passes_run;
      m->rel_stat_incr++;
      // the slab serves only rebuilds: after a run of incremental updates it goes back to the device
      // (ADVICE r2), and the next rebuild allocates it again
      if (++m->rel_incr_streak >= kSlabIdleViews && m->rel_slab) {
        HIPCHK(hipStreamSynchronize(m->stream));
        hipFree(m->rel_slab);
        hipFree(m->rel_fix);
        m->rel_slab = nullptr;
        m->rel_fix = nullptr;
        m->rel_slab_recs = 0;
      }
      out->row_ptr = m->rel_rp;
      out->cols = m->rel_cols;
      out->nnz = m->rel_nnz;
      return GWAOI_OK;
    }
  }
  m->rel_valid = false;
  RCHK(ensure_grid_current(m));  // (after small passes the grid lags their ops: rebuilt from the slots)
  hipStream_t st = m->stream;
  if (!m->rel_rp) RCHK(dalloc(&m->rel_rp, (size_t)m->cap + 1));
  if (!m->rel_tot) RCHK(dalloc(&m->rel_tot, 3));  // [0] entries, [1] longest row, [2] rows to fix
  if (!m->rel_tstat) RCHK(dalloc(&m->rel_tstat, (size_t)m->max_cells / gw::kTileCells + 1));
  // The count pass also writes every row of up to kSlabS entries into a slab (by grid record), when
  // that fits; the rows then go from the slab to cols sorted, with no second walk. A longer row (crowds)
  // sends the call down the two-walk path: fill pass, sort in place. The slab holds the rows of the
  // current grid's records (+25% headroom, reallocated when a grid has more), within a fixed budget and
  // half of the device memory free at the time.
  constexpr uint32_t kSlabS = 128;
  constexpr uint64_t kSlabBudget = 4ull << 30;  // bytes
  m->rel_incr_streak = 0;
  const uint64_t recs = std::max<uint64_t>(m->h_ctr[gw::CTR_RECORDS], 1);
  if (m->rel_slab && recs > m->rel_slab_recs) {
    HIPCHK(hipStreamSynchronize(m->stream));
    hipFree(m->rel_slab);
    m->rel_slab = nullptr;
  }
  if (!m->rel_slab) {  // (retried at every rebuild: free memory changes)
    const uint64_t srecs = std::min<uint64_t>(2ull * m->cap, recs + recs / 4 + 64);
    const uint64_t slab_words = ((srecs + 63) / 64) * 64 * kSlabS;
    size_t free_b = 0, total_b = 0;
    const bool room = hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
                      slab_words * 4 <= std::min<uint64_t>(kSlabBudget, free_b / 2);
    if (!room || dalloc(&m->rel_slab, (size_t)slab_words) != GWAOI_OK ||
        (!m->rel_fix && dalloc(&m->rel_fix, 2 * (size_t)m->cap) != GWAOI_OK)) {
      if (m->rel_slab) hipFree(m->rel_slab);
      m->rel_slab = nullptr;
      m->rel_no_slab = true;
    } else {
      m->rel_slab_recs = srecs;
      m->rel_no_slab = false;
    }
  }
  const Grid& g = m->grid[m->cur];
  gw::RelArgs a{};
  a.g = {g.rec, g.cs, g.d_geom, g.d_tile_space};
  a.pos_x = m->pos_x;
  a.pos_z = m->pos_z;
  a.seq = m->seq;
  a.space_of = m->space_of;
  a.cap = m->cap;
  a.row_ptr = nullptr;
  a.row_cnt = m->rel_rp;
  a.cols = nullptr;
  a.ntiles = g.ncells ? g.ntiles : 0u;
  a.total64 = m->rel_tot;
  a.maxlen = reinterpret_cast<uint32_t*>(m->rel_tot + 1);
  a.tstat = m->rel_tstat;
  a.slab = m->rel_slab;
  a.slab_s = a.slab ? kSlabS : 0u;
  a.slab_recs = a.slab ? (uint32_t)std::min<uint64_t>(m->rel_slab_recs, 0xffffffffull) : 0u;
  // count pass, scan, then the row lengths' total is the one value the host must know (allocation)
  HIPCHK(hipMemsetAsync(m->rel_rp, 0, ((size_t)m->cap + 1) * sizeof(uint32_t), st));
  HIPCHK(hipMemsetAsync(m->rel_tot, 0, 3 * sizeof(unsigned long long), st));
  gw::launch_relation(a, st);
  unsigned long long tot[2] = {0, 0};
  RCHK(read_words(m, reinterpret_cast<const uint32_t*>(m->rel_tot), 4, nullptr, 0,
                  reinterpret_cast<uint32_t*>(tot)));
  const unsigned long long total64 = tot[0];
  const uint32_t maxlen = (uint32_t)tot[1];
  if (total64 > m->index_limit) {  // row_ptr is uint32: a scan past 2^32 - 1 would wrap
    set_err("relation_device: %llu directed entries exceed the view's uint32 row offsets (limit %llu)",
            (unsigned long long)total64, (unsigned long long)m->index_limit);
    return GWAOI_ERR_NOMEM;
  }
  gw::launch_scan(m->scan, m->rel_rp, m->cap + 1, st);
  const uint32_t total = (uint32_t)total64;
  const uint64_t want = (uint64_t)total + total / 4 + 1024;
  if (total > m->rel_cap) {
    if (m->rel_cols) hipFree(m->rel_cols);
    m->rel_cols = nullptr;
    m->rel_cap = 0;
    RCHK(dalloc(&m->rel_cols, want));
    m->rel_cap = want;
  }
  if (total > m->rel_tmp_cap) {
    if (m->rel_tmp) hipFree(m->rel_tmp);
    m->rel_tmp = nullptr;
    m->rel_tmp_cap = 0;
    RCHK(dalloc(&m->rel_tmp, want));
    m->rel_tmp_cap = want;
  }
  if (total == 0) {
    // empty relation: row_ptr is all zeros, nothing to sort
  } else if (a.slab && maxlen <= a.slab_s) {
    gw::launch_row_sort_slab(g.rec, g.cs + g.ncells, 2 * m->cap, m->rel_rp, a.slab, a.slab_s, m->rel_cols,
                             m->rel_tmp, m->rel_fix, reinterpret_cast<uint32_t*>(m->rel_tot + 2), st);
  } else {  // a row longer than the slab keeps: the fill pass walks again
    a.row_ptr = m->rel_rp;
    a.cols = m->rel_cols;
    a.slab = nullptr;
    a.slab_s = 0;
    gw::launch_relation(a, st);
    gw::launch_row_sort(m->rel_rp, m->cap, m->rel_cols, m->rel_tmp, st);
  }
  HIPCHK(hipGetLastError());
  m->rel_valid = true;
  m->rel_passes = m->passes_run;
  m->rel_nnz = total;
  m->rel_stat_full++;
  out->row_ptr = m->rel_rp;
  out->cols = m->rel_cols;
  out->nnz = total;
  return GWAOI_OK;
}

int gwaoi_debug_set_relation_mode(gwaoi_mgr* m, int mode, uint64_t* n_incremental, uint64_t* n_full,
                                  int* last_rebuild_reason) {
  RCHK(check_mgr(m));
  if (mode < -1 || mode > 1) return GWAOI_ERR_INVALID;
  if (mode >= 0) m->rel_mode = mode;
  if (n_incremental) *n_incremental = m->rel_stat_incr;
  if (n_full) *n_full = m->rel_stat_full;
  if (last_rebuild_reason) *last_rebuild_reason = m->rel_why;
  return GWAOI_OK;
}

int gwaoi_export_relation(gwaoi_mgr* m, uint32_t* row_ptr, uint32_t* cols, uint64_t cols_cap, uint64_t* nnz) {
  RCHK(check_mgr(m));
  if (!row_ptr || !nnz || (cols_cap && !cols)) {
    set_err("export_relation: null argument");
    return GWAOI_ERR_INVALID;
  }
  gwaoi_relation_view v;
  RCHK(gwaoi_relation_device(m, &v));
  *nnz = v.nnz;
  if (v.nnz > cols_cap) {
    set_err("export_relation: cols_cap %llu < nnz %llu", (unsigned long long)cols_cap, (unsigned long long)v.nnz);
    return GWAOI_ERR_INVALID;
  }
  hipStream_t st = m->stream;
  hipError_t e = hipMemcpyAsync(row_ptr, v.row_ptr, ((size_t)m->cap + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && v.nnz)
    e = hipMemcpyAsync(cols, v.cols, (size_t)v.nnz * sizeof(uint32_t), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    set_err("export_relation: %s", hipGetErrorString(e));
    return GWAOI_ERR_HIP;
  }
  return GWAOI_OK;
}

int gwaoi_export_relation_delta(gwaoi_mgr* m, gwaoi_event* out, uint64_t cap, uint64_t* n) {
  RCHK(check_mgr(m));
  if (!n || (cap && !out)) {
    set_err("export_relation_delta: null argument");
    return GWAOI_ERR_INVALID;
  }
  *n = 0;
  if (!m->dx_ready) {
    set_err("export_relation_delta: no tick to export (call it after gwaoi_tick, before the next pass runs)");
    return GWAOI_ERR_STATE;
  }
  if (m->dx_silent) {
    set_err("export_relation_delta: the tick applied SILENT ops, whose pairs are not in its events");
    return GWAOI_ERR_STATE;
  }
  const uint64_t nev = m->dx_events;
  if (!nev) return GWAOI_OK;
  if (nev > 0x7FFFFFFFull) {
    set_err("export_relation_delta: %llu events exceed the export's uint32 indices", (unsigned long long)nev);
    return GWAOI_ERR_NOMEM;
  }
  RCHK(set_dev(m));
  hipStream_t st = m->stream;
  uint64_t slots = 1024;
  while (slots < 2 * nev) slots <<= 1;
  if (slots > m->dx_slots) {
    for (void* p : {(void*)m->dx_keys, (void*)m->dx_cnt, (void*)m->dx_last})
      if (p) hipFree(p);
    m->dx_keys = nullptr, m->dx_cnt = m->dx_last = nullptr, m->dx_slots = 0;
    RCHK(dalloc(&m->dx_keys, slots));
    RCHK(dalloc(&m->dx_cnt, slots));
    RCHK(dalloc(&m->dx_last, slots));
    m->dx_slots = slots;
  }
  if (nev > m->dx_cap) {
    for (void* p : {(void*)m->dx_slot, (void*)m->dx_flags, (void*)m->dx_out, (void*)m->dx_part})
      if (p) hipFree(p);
    m->dx_slot = m->dx_flags = m->dx_part = nullptr, m->dx_out = nullptr, m->dx_cap = 0;
    const uint64_t want = nev + nev / 4 + 1024;
    RCHK(dalloc(&m->dx_slot, want));
    RCHK(dalloc(&m->dx_flags, want + 1));
    RCHK(dalloc(&m->dx_out, 2 * want));
    RCHK(dalloc(&m->dx_part, gw::scan_part_words((uint32_t)want + 1)));
    m->dx_cap = want;
  }
  HIPCHK(hipMemsetAsync(m->dx_keys, 0xFF, slots * sizeof(unsigned long long), st));
  HIPCHK(hipMemsetAsync(m->dx_cnt, 0, slots * sizeof(uint32_t), st));
  HIPCHK(hipMemsetAsync(m->dx_last, 0, slots * sizeof(uint32_t), st));
  gw::DeltaExportArgs a{};
  a.ev = m->ev_out;
  a.nev = (uint32_t)nev;
  a.mask = (uint32_t)(slots - 1);
  a.keys = m->dx_keys;
  a.cnt = m->dx_cnt;
  a.last = m->dx_last;
  a.slot_of = m->dx_slot;
  a.flags = m->dx_flags;
  a.out = m->dx_out;
  gw::ScanCtx sc;
  sc.status = m->dx_part;
  gw::launch_delta_export(a, sc, st);
  HIPCHK(hipGetLastError());
  uint32_t kept = 0;
  HIPCHK(hipMemcpyAsync(&kept, m->dx_flags + nev, sizeof kept, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  *n = 2ull * kept;
  if (*n > cap) {
    set_err("export_relation_delta: cap %llu < %llu changes", (unsigned long long)cap, (unsigned long long)*n);
    return GWAOI_ERR_INVALID;
  }
  if (*n) {
    HIPCHK(hipMemcpyAsync(out, m->dx_out, *n * sizeof(gwaoi_event), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return GWAOI_OK;
}

int gwaoi_set_timing(gwaoi_mgr* m, int enable) {
  if (!m) return GWAOI_ERR_INVALID;
  RCHK(set_dev(m));
  RCHK(collect_timing(m));
  m->timing = enable != 0;
  return GWAOI_OK;
}

int gwaoi_get_stats(const gwaoi_mgr* m, gwaoi_stats* out) {
  if (!m || !out) return GWAOI_ERR_INVALID;
  gwaoi_mgr* mm = const_cast<gwaoi_mgr*>(m);  // the last timed pass is folded in on demand
  RCHK(set_dev(mm));
  RCHK(collect_timing(mm));
  *out = m->stats;
  return GWAOI_OK;
}

int gwaoi_reset_stats(gwaoi_mgr* m) {
  if (!m) return GWAOI_ERR_INVALID;
  RCHK(set_dev(m));
  RCHK(collect_timing(m));
  m->stats = gwaoi_stats{};
  return GWAOI_OK;
}

// ---- tooling (include/gwaoi_tools.h) ----

int gwaoi_device_count(int* n) {
  if (!n) return GWAOI_ERR_INVALID;
  *n = 0;
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    set_err("hipGetDeviceCount: %s", hipGetErrorString(e));
    return GWAOI_ERR_HIP;
  }
  return GWAOI_OK;
}

int gwaoi_dev_malloc(int device, size_t bytes, void** out) {
  if (!out) return GWAOI_ERR_INVALID;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(out, bytes ? bytes : 1));
  return GWAOI_OK;
}

int gwaoi_dev_free(int device, void* p) {
  HIPCHK(hipSetDevice(device));
  if (p) HIPCHK(hipFree(p));
  return GWAOI_OK;
}

int gwaoi_dev_htod(int device, void* dst, const void* src, size_t bytes) {
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return GWAOI_OK;
}

int gwaoi_dev_dtoh(int device, void* dst, const void* src, size_t bytes) {
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return GWAOI_OK;
}

int gwaoi_dev_sync(int device) {
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipDeviceSynchronize());
  return GWAOI_OK;
}

int gwaoi_wl_init(int device, float* d_x, float* d_z, uint32_t n, uint64_t seed, float L) {
  HIPCHK(hipSetDevice(device));
  gw::launch_wl_init(d_x, d_z, n, seed, L, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  return GWAOI_OK;
}

int gwaoi_wl_step(int device, const float* d_xprev, const float* d_zprev, float* d_xout, float* d_zout, uint32_t n,
                  uint64_t seed, uint64_t tick, float L, float s) {
  HIPCHK(hipSetDevice(device));
  gw::launch_wl_step(d_xprev, d_zprev, d_xout, d_zout, n, seed, tick, L, s, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  return GWAOI_OK;
}

int gwaoi_wl_init_spaces(int device, float* d_x, float* d_z, uint32_t n_per, uint32_t nspaces, uint64_t seed0,
                         float L, uint32_t nhot, float sigma, uint32_t hot_every) {
  HIPCHK(hipSetDevice(device));
  gw::launch_wl_init_spaces(d_x, d_z, n_per, nspaces, seed0, L, nhot, sigma, hot_every, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  return GWAOI_OK;
}

int gwaoi_wl_step_spaces(int device, const float* d_xprev, const float* d_zprev, float* d_xout, float* d_zout,
                         uint32_t n_per, uint32_t nspaces, uint64_t seed0, uint64_t tick, float L, float s) {
  HIPCHK(hipSetDevice(device));
  gw::launch_wl_step_spaces(d_xprev, d_zprev, d_xout, d_zout, n_per, nspaces, seed0, tick, L, s, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  return GWAOI_OK;
}

int gwaoi_wl_iota(int device, uint32_t* d, uint32_t n) {
  HIPCHK(hipSetDevice(device));
  gw::launch_iota(d, n, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  return GWAOI_OK;
}

int gwaoi_debug_set_next_seq(gwaoi_mgr* m, uint32_t next_seq) {
  RCHK(check_mgr(m));
  if (next_seq < m->next_seq || next_seq >= kSeqLimit) {
    set_err("debug_set_next_seq: must be in [%u, %u)", m->next_seq, kSeqLimit);
    return GWAOI_ERR_INVALID;
  }
  m->next_seq = next_seq;
  return GWAOI_OK;
}


int gwaoi_debug_set_sweep_lds(gwaoi_mgr* m, int enable) {
  RCHK(check_mgr(m));
  // 0: every mover walks from global memory (k_sweep lists them all for k_sweep_dense); 1: the default;
  // 2: staging only (timing); 3: the default without the big sweep (grids built from now on)
  m->sweep_lds = enable < 0 ? 0 : (enable > 2 ? 1 : enable);
  if (enable == 3 || enable == 1) {
    m->big_sweep = enable == 1;
    m->geom_dirty = true;
  }
  return GWAOI_OK;
}

int gwaoi_debug_set_band(gwaoi_mgr* m, int mode, uint64_t* n_band_movers) {
  RCHK(check_mgr(m));
  if (mode > 2) {
    set_err("debug_set_band: mode %d (0 off: every dense mover walks its ring, 1 on, 2 every band plan)", mode);
    return GWAOI_ERR_INVALID;
  }
  if (mode >= 0) m->band_mode = mode;
  if (n_band_movers) *n_band_movers = m->band_movers;
  return GWAOI_OK;
}

int gwaoi_debug_sweep_sizes(gwaoi_mgr* m, int enable, uint64_t* tiles) {
  RCHK(check_mgr(m));
  RCHK(set_dev(m));
  if (enable > 0 && !m->d_size_tiles) {
    RCHK(dalloc(&m->d_size_tiles, 4));
    HIPCHK(hipMemsetAsync(m->d_size_tiles, 0, 4 * sizeof(uint32_t), m->stream));
  }
  uint32_t h[4] = {0, 0, 0, 0};
  if (m->d_size_tiles) {
    HIPCHK(hipStreamSynchronize(m->stream));
    HIPCHK(hipMemcpy(h, m->d_size_tiles, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  if (tiles)
    for (int k = 0; k < 3; ++k) tiles[k] = h[k];
  if (enable == 0 && m->d_size_tiles) {
    HIPCHK(hipFree(m->d_size_tiles));
    m->d_size_tiles = nullptr;
  }
  return GWAOI_OK;
}

int gwaoi_debug_set_small_pass(gwaoi_mgr* m, int mode, uint64_t* n_small) {
  RCHK(check_mgr(m));
  if (mode > 2) {
    set_err("debug_set_small_pass: mode %d (0 off, 1 auto, 2 whenever the overlay has room)", mode);
    return GWAOI_ERR_INVALID;
  }
  if (mode >= 0) m->small_mode = mode;
  if (n_small) *n_small = m->small_passes;
  return GWAOI_OK;
}

int gwaoi_debug_set_build_mode(gwaoi_mgr* m, int mode, uint64_t* n_fused, uint64_t* n_counting, uint64_t* n_reruns) {
  RCHK(check_mgr(m));
  if (mode > 1) {
    set_err("build mode %d (0 one-pass when possible, 1 counting)", mode);
    return GWAOI_ERR_INVALID;
  }
  if (mode >= 0) m->build_mode = mode;
  if (n_fused) *n_fused = m->builds_fused;
  if (n_counting) *n_counting = m->builds_counting;
  if (n_reruns) *n_reruns = m->build_reruns;
  return GWAOI_OK;
}

int gwaoi_debug_sweep_occupancy(int device, int* blocks_per_cu, int* lds_bytes) {
  if (!blocks_per_cu || !lds_bytes) return GWAOI_ERR_INVALID;
  HIPCHK(hipSetDevice(device));
  gw::sweep_init();
  *lds_bytes = (int)gw::sweep_lds_bytes();
  if (gw::sweep_occupancy(blocks_per_cu)) {
    set_err("hipOccupancyMaxActiveBlocksPerMultiprocessor failed");
    return GWAOI_ERR_HIP;
  }
  return GWAOI_OK;
}

int gwaoi_debug_read_stamps(void* host, size_t bytes) {
  if (!host) return GWAOI_ERR_INVALID;
  const int r = gw::read_stamps(host, bytes);
  if (r) set_err("debug_read_stamps: library not built with GW_STAMPS=1");
  return r;
}

int gwaoi_set_population_hint(gwaoi_mgr* m, uint32_t space, uint32_t expected) {
  RCHK(check_mgr(m));
  if (space >= m->nspaces) {
    set_err("set_population_hint: space %u >= %u", space, m->nspaces);
    return GWAOI_ERR_INVALID;
  }
  m->spaces[space].pop_hint = expected;
  m->geom_dirty = true;
  return GWAOI_OK;
}

int gwaoi_debug_set_index_limit(gwaoi_mgr* m, uint64_t limit) {
  RCHK(check_mgr(m));
  m->index_limit = std::min<uint64_t>(limit, 0xFFFFFFFFull);
  return GWAOI_OK;
}

int gwaoi_debug_set_cells_per_dist(gwaoi_mgr* m, float cpd) {
  RCHK(check_mgr(m));
  if (!(cpd > 0) || cpd > 64) return GWAOI_ERR_INVALID;
  m->cells_per_dist = cpd;
  m->density_cells = false;
  m->geom_dirty = true;
  return GWAOI_OK;
}

int gwaoi_debug_set_cell_side(gwaoi_mgr* m, float side) {
  RCHK(check_mgr(m));
  if (!(side >= 0) || !std::isfinite(side)) return GWAOI_ERR_INVALID;
  m->cell_side = side;
  m->density_cells = false;
  m->geom_dirty = true;
  return GWAOI_OK;
}

}  // extern "C"
