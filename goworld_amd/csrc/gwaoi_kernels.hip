// gwaoi_kernels.hip — gfx950 kernels of the tick-batched AOI pipeline.
//
// One pass applies a batch of ops (Enter/Leave/Moved, in staging order) and emits exactly the pair
// events go-aoi's XZListAOIManager would raise for the same calls one by one (include/gwaoi.h).
//
// Why no neighbour lists are stored: after any go-aoi call on m, m's neighbour set is exactly
// {o : in(m, o)} (adjust() keeps mark==2 neighbours, drops the rest, adds new mark==2 nodes), and a
// pair is only re-evaluated by a call on one of its two members. So the relation is a pure function
// of positions and of "who acted last": N(a,b) = in(L, F) with L the member whose last op is later
// and F the other, both at their current positions. Every entity carries seq = the global sequence
// number of its last op, and a pass needs, per mover m with op seq q:
//   before(m,o) = state just before m's op:  in(o_new, m_old) if o acted earlier in this pass,
//                                            else in(L, F) over the start-of-pass state,
//   after(m,o)  = in(m_new, o at that time) (o_new if o acted earlier, else o_old),
// and emits ENTER/LEAVE(m,o) where they differ. Old-pass positions come from the old grid (the
// previous pass's new grid), new ones from the new grid; both are cell-sorted snapshots.
//
// Float semantics: every bound is one binary32 add/sub (built with -ffp-contract=off, denormals
// preserved), compared inclusively — bit-exact with Go float32 arithmetic.
#include <hip/hip_runtime.h>

#include "gwaoi_internal.h"
#include "gwaoi_workload.h"

namespace gw {

constexpr int kBlock = 256;
// Query boxes are widened by (|c| + D) * 2^-20 before they are turned into cell ranges, so a
// candidate whose OWN box (rounded from its own coordinate) reaches the mover is never missed.
// Cell ranges are only a candidate filter; the exact predicate decides.
constexpr float kMargin = 9.5367431640625e-07f;

__device__ __forceinline__ int cellc(float v, float o, float inv, int n) {
  float f = (v - o) * inv;  // monotone in v, so cell(lo) <= cell(v) <= cell(hi) for lo <= v <= hi
  if (!(f >= 0.0f)) return 0;
  if (f >= (float)n) return n - 1;
  return (int)f;
}

// in(c, p): p inside the box of an entity at c (go-aoi Mark/GetClearMarkedNeighbors bounds).
__device__ __forceinline__ bool inbox(float cx, float cz, float D, float px, float pz) {
  const float lx = cx - D, hx = cx + D, lz = cz - D, hz = cz + D;
  return px >= lx && px <= hx && pz >= lz && pz <= hz;
}

struct Bounds {
  float lx, hx, lz, hz;
  __device__ __forceinline__ bool has(float px, float pz) const {
    return px >= lx && px <= hx && pz >= lz && pz <= hz;
  }
};

struct CellBox {
  int x0, x1, z0, z1;
};

__device__ __forceinline__ CellBox qbox(const Geom& g, float cx, float cz) {
  const float mx = (fabsf(cx) + g.D) * kMargin, mz = (fabsf(cz) + g.D) * kMargin;
  CellBox b;
  b.x0 = cellc((cx - g.D) - mx, g.x0, g.inv_c, g.ncx);
  b.x1 = cellc((cx + g.D) + mx, g.x0, g.inv_c, g.ncx);
  b.z0 = cellc((cz - g.D) - mz, g.z0, g.inv_c, g.ncz);
  b.z1 = cellc((cz + g.D) + mz, g.z0, g.inv_c, g.ncz);
  return b;
}

__device__ __forceinline__ uint32_t cell_key(const Geom& g, int cx, int cz) {
  return g.base + ((uint32_t)((cz >> kTileShift) * g.ntx + (cx >> kTileShift)) << kTileCellShift) +
         (uint32_t)(((cz & (kTile - 1)) << kTileShift) | (cx & (kTile - 1)));
}

// Row intervals of the union of box A (if va) and box B (if vb): one or two column intervals per
// row, so every cell is visited once.
template <class RowF>
__device__ __forceinline__ void for_each_row_interval(bool va, CellBox A, bool vb, CellBox B, RowF&& rf) {
  int r0 = va ? A.z0 : B.z0, r1 = va ? A.z1 : B.z1;
  if (va && vb) {
    r0 = min(A.z0, B.z0);
    r1 = max(A.z1, B.z1);
  }
  for (int r = r0; r <= r1; ++r) {
    const bool ia = va && r >= A.z0 && r <= A.z1;
    const bool ib = vb && r >= B.z0 && r <= B.z1;
    if (ia && ib) {
      if (B.x0 <= A.x1 + 1 && A.x0 <= B.x1 + 1) {
        rf(r, min(A.x0, B.x0), max(A.x1, B.x1));
      } else {
        rf(r, A.x0, A.x1);
        rf(r, B.x0, B.x1);
      }
    } else if (ia) {
      rf(r, A.x0, A.x1);
    } else if (ib) {
      rf(r, B.x0, B.x1);
    }
  }
}

// Global-memory path: entries of row r, columns [c0, c1]: one contiguous segment per tile crossed.
template <class F>
__device__ __forceinline__ void row_entries_global(const Geom& g, const uint32_t* __restrict__ cs, int r, int c0,
                                                   int c1, F&& f) {
  if (c0 > c1) return;
  const uint32_t rowbase = g.base + ((uint32_t)((r >> kTileShift) * g.ntx) << kTileCellShift) +
                           (uint32_t)((r & (kTile - 1)) << kTileShift);
  for (int tx = c0 >> kTileShift; tx <= (c1 >> kTileShift); ++tx) {
    const int lo = max(c0, tx << kTileShift), hi = min(c1, (tx << kTileShift) + kTile - 1);
    const uint32_t k = rowbase + ((uint32_t)tx << kTileCellShift) + (uint32_t)(lo & (kTile - 1));
    for (uint32_t j = cs[k], e = cs[k + (uint32_t)(hi - lo) + 1]; j < e; ++j) f(j);
  }
}

template <class F>
__device__ __forceinline__ void for_each_entry(const Geom& g, const uint32_t* __restrict__ cs, bool va,
                                               CellBox A, bool vb, CellBox B, F&& f) {
  for_each_row_interval(va, A, vb, B, [&](int r, int c0, int c1) { row_entries_global(g, cs, r, c0, c1, f); });
}

// ---------------------------------------------------------------------------------------------
// apply: one thread per op. Records each mover's start-of-pass state, stamps its old-grid entry
// with the op's seq, and writes the new state. Slots of one pass are distinct (the host guarantees
// it for host-staged ops; for device-staged batches k_slice_sort checks afterwards that every op's
// slot carries that op's seq — a duplicate leaves one of two ops without it).
__global__ void __launch_bounds__(kBlock) k_apply(ApplyArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n_ops) return;
  const uint32_t s = a.op_slot[i];
  const uint32_t q = a.base + i;
  if (i == 0) *a.rank_tail = 0u;
  const uint8_t kind = a.op_kind ? a.op_kind[i] : (uint8_t)OP_MOVE;
  if (a.check && s >= a.cap) {
    atomicOr(&a.ctr[CTR_ERR], ERR_BAD_SLOT);
    return;
  }
  const uint32_t q0 = a.seq[s];
  if (a.check && q0 == 0) {
    atomicOr(&a.ctr[CTR_ERR], ERR_ABSENT_SLOT);
    return;
  }
  a.old_x[s] = a.pos_x[s];
  a.old_z[s] = a.pos_z[s];
  a.old_seq[s] = q0;
  if (q0) a.old_side[a.old_gidx[s]] = q;
  if (kind == OP_LEAVE) {
    a.seq[s] = 0;
  } else {
    a.pos_x[s] = a.op_x[i];
    a.pos_z[s] = a.op_z[i];
    a.seq[s] = q;
    if (kind == OP_ENTER) a.space_of[s] = a.op_space[i];
  }
}

void launch_apply(const ApplyArgs& a, hipStream_t st) {
  if (!a.n_ops) return;
  hipLaunchKernelGGL(k_apply, dim3((a.n_ops + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
}

// ---------------------------------------------------------------------------------------------
// Counting sort of present entities by cell key: count (atomics give each entity its rank inside
// its cell), exclusive scan of the counts, scatter.
__global__ void __launch_bounds__(kBlock) k_bin_count(BinArgs a) {
  const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= a.cap) return;
  const uint32_t q = a.seq[s];
  if (!q) return;
  const Geom g = a.geom[a.space_of[s]];
  const uint32_t key = cell_key(g, cellc(a.pos_x[s], g.x0, g.inv_c, g.ncx), cellc(a.pos_z[s], g.z0, g.inv_c, g.ncz));
  a.key_of[s] = key;
  a.local_of[s] = atomicAdd(&a.cs[key], 1u);
}

__global__ void __launch_bounds__(kBlock) k_bin_scatter(BinArgs a) {
  const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= a.cap) return;
  const uint32_t q = a.seq[s];
  if (!q) return;
  const uint32_t j = a.cs[a.key_of[s]] + a.local_of[s];
  a.ent[j] = make_uint4(__float_as_uint(a.pos_x[s]), __float_as_uint(a.pos_z[s]), s, q);
  a.gidx[s] = j;
}

void launch_bin_count(const BinArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_bin_count, dim3((a.cap + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
}
void launch_bin_scatter(const BinArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_bin_scatter, dim3((a.cap + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
}

// ---------------------------------------------------------------------------------------------
// Exclusive scan (u32): per-block reduce, scan of block sums, block scan + offset. Wave64 prefix
// sums by __shfl_up; 256-thread blocks, 16 items per thread.
constexpr int kScanItems = 16;
constexpr uint32_t kScanChunk = kBlock * kScanItems;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// exclusive prefix of v over the block; *total = block sum. blockDim.x must be kBlock.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
  __shared__ uint32_t ws[kBlock / 64];
  const uint32_t inc = wave_incl_scan(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) ws[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kBlock / 64; ++k) {
    pre += k < w ? ws[k] : 0u;
    tot += ws[k];
  }
  __syncthreads();
  *total = tot;
  return pre + inc - v;
}

__global__ void __launch_bounds__(kBlock) k_scan_reduce(const uint32_t* __restrict__ d, uint32_t n,
                                                        uint32_t* __restrict__ part) {
  const uint32_t b0 = blockIdx.x * kScanChunk + threadIdx.x * kScanItems;
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) sum += (b0 + k < n) ? d[b0 + k] : 0u;
  uint32_t tot;
  block_excl_scan(sum, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kBlock) k_scan_part(uint32_t* part, uint32_t nb) {
  // single block; nb <= kScanChunk
  const uint32_t b0 = threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = (b0 + k < nb) ? part[b0 + k] : 0u;
    sum += v[k];
  }
  uint32_t tot;
  uint32_t pre = block_excl_scan(sum, &tot);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (b0 + k < nb) part[b0 + k] = pre;
    pre += v[k];
  }
}

__global__ void __launch_bounds__(kBlock) k_scan_down(uint32_t* __restrict__ d, uint32_t n,
                                                      const uint32_t* __restrict__ part) {
  const uint32_t b0 = blockIdx.x * kScanChunk + threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = (b0 + k < n) ? d[b0 + k] : 0u;
    sum += v[k];
  }
  uint32_t tot;
  uint32_t pre = block_excl_scan(sum, &tot) + (part ? part[blockIdx.x] : 0u);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (b0 + k < n) d[b0 + k] = pre;
    pre += v[k];
  }
}

uint32_t scan_part_words(uint32_t n) { return (n + kScanChunk - 1) / kScanChunk + 1; }

void launch_scan(uint32_t* d, uint32_t n, uint32_t* part, hipStream_t st) {
  if (!n) return;
  const uint32_t nb = (n + kScanChunk - 1) / kScanChunk;
  if (nb == 1) {
    hipLaunchKernelGGL(k_scan_down, dim3(1), dim3(kBlock), 0, st, d, n, (const uint32_t*)nullptr);
    return;
  }
  // nb <= kScanChunk: n <= 16.7M per level. Larger n would need a recursive level.
  hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(kBlock), 0, st, (const uint32_t*)d, n, part);
  hipLaunchKernelGGL(k_scan_part, dim3(1), dim3(kBlock), 0, st, part, nb);
  hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(kBlock), 0, st, d, n, (const uint32_t*)part);
}

// ---------------------------------------------------------------------------------------------
// Sweep. One 512-thread block per tile of the new grid (kTile x kTile cells); the block loops over
// the tile's movers, one thread per mover. The block first stages, for BOTH grids, every entry of
// the tile plus a halo of `reach` cells into LDS (entries, the old grid's side stamps, and a cell
// start table), laid out row by row so that any row interval of the region is one contiguous LDS
// range; each mover then walks its candidates in LDS. Movers whose query boxes leave the region
// (teleports), tiles whose region does not fit, and Leave ops take the global-memory path; both
// paths evaluate the same predicates.
//
// Ring walk: for a Moved op, a candidate strictly inside BOTH the old and the new box (shrunk by a
// margin far above float32 rounding) is inside from every perspective before and after, so it
// cannot raise an event. Cells whose every point is that deep (cell index strictly between the
// cells of the shrunken bounds; cellc is monotone, clamping included) are skipped: only the ring of
// border cells is read. Enter and Leave ops walk their whole box.
//
// Events are rare (~0.3 per mover per tick), but one global counter hit by every event serialises
// at the memory side, so each block stages its events in LDS and reserves its output range with ONE
// global atomic; a mover's events are numbered in a register (one thread per mover) and its count is
// stored once, without atomics.
constexpr int kSweepBlock = 512;
constexpr int kEvLds = 256;       // events staged per block before spilling to global atomics
constexpr int kRegCells = 2304;   // max cells of a staged region (48 x 48)
constexpr int kCap = 1088;        // max entries staged per grid
constexpr int kMaxRows = 48;
constexpr float kInner = 3.814697265625e-06f;  // 2^-18: ring margin, relative to |c| + D

struct SweepSmem {  // dynamic LDS (16-B aligned carve)
  uint32_t n, enter, base, flags;
  uint32_t ws[16];                  // block-scan scratch
  uint32_t gsp[2][kMaxRows * 3];    // global start of each (region row, tile part)
  uint4 ev[kEvLds];                 // event queue
  uint16_t lcs[2][kRegCells + 8];   // LDS start of each region cell (+ total)
  uint4 ent[2][kCap];  // old grid: {x, z, seq0, side}; new grid: {x, z, slot, seq}
  uint32_t slot_old[kCap];
};

size_t sweep_lds_bytes() { return sizeof(SweepSmem); }

template <class Q>
__device__ __forceinline__ void emit(const SweepArgs& a, Q& sm, uint32_t rank, uint32_t local, uint32_t mover,
                                     uint32_t other, bool enter) {
  const uint4 rec = make_uint4(rank, local, mover, other | (enter ? 0x80000000u : 0u));
  const uint32_t li = atomicAdd(&sm.n, 1u);
  if (li < (uint32_t)kEvLds) {
    sm.ev[li] = rec;
  } else {
    const uint32_t gi = atomicAdd(&a.ctr[CTR_EVENTS], 1u);
    if (gi < a.ev_cap) a.ev_tmp[gi] = rec;
  }
  if (enter) atomicAdd(&sm.enter, 1u);
}

struct Mover {
  uint32_t sm, q, q0, rank;
  bool valid0, valid1;
  float mx0, mz0, mx1, mz1, D;
};

__device__ __forceinline__ Mover make_mover(const SweepArgs& a, uint32_t sm, uint32_t q, bool valid1, float mx1,
                                            float mz1, float D) {
  Mover m;
  m.sm = sm;
  m.q = q;
  m.q0 = a.old_seq[sm];
  m.rank = q - a.base;
  m.valid0 = m.q0 != 0;
  m.valid1 = valid1;
  m.mx0 = a.old_x[sm];
  m.mz0 = a.old_z[sm];
  m.mx1 = mx1;
  m.mz1 = mz1;
  m.D = D;
  return m;
}

// The cells a mover must read: rows z0..z1 of the union of its old and new query boxes, and in each
// row at most two column intervals — the two boxes' intervals (merged when they touch), or, for a
// move whose boxes overlap, the two ring pieces left and right of the cells deep inside both boxes.
// The walk runs over rows RELATIVE to each lane's own window with a wave-uniform trip count, and
// always visits segment A then segment B (possibly empty), so lanes of a wave that sit in
// different cell rows still follow the same control flow.
struct Walk {
  int z0, z1;          // rows
  int ax0, ax1, az0, az1;  // box A columns / rows (old box, or the union for a ring walk)
  int bx0, bx1, bz0, bz1;  // box B (new box); for a ring walk: inner rows bz0..bz1, inner cols bx0..bx1
  bool ring;
};

__device__ __forceinline__ Walk make_walk(const Mover& m, const Geom& g) {
  const CellBox A0 = qbox(g, m.mx0, m.mz0), A1 = qbox(g, m.mx1, m.mz1);
  Walk w;
  w.ring = false;
  if (m.valid0 && m.valid1) {
    const int x0 = min(A0.x0, A1.x0), x1 = max(A0.x1, A1.x1);
    const int z0 = min(A0.z0, A1.z0), z1 = max(A0.z1, A1.z1);
    if (x1 - x0 <= (A1.x1 - A1.x0) + 2 && z1 - z0 <= (A1.z1 - A1.z0) + 2) {
      const float D = g.D;
      const float ex = (fmaxf(fabsf(m.mx0), fabsf(m.mx1)) + D) * kInner;
      const float ez = (fmaxf(fabsf(m.mz0), fabsf(m.mz1)) + D) * kInner;
      w.ring = true;
      w.z0 = w.az0 = z0;
      w.z1 = w.az1 = z1;
      w.ax0 = x0;
      w.ax1 = x1;
      w.bx0 = cellc((fmaxf(m.mx0, m.mx1) - D) + ex, g.x0, g.inv_c, g.ncx) + 1;
      w.bx1 = cellc((fminf(m.mx0, m.mx1) + D) - ex, g.x0, g.inv_c, g.ncx) - 1;
      w.bz0 = cellc((fmaxf(m.mz0, m.mz1) - D) + ez, g.z0, g.inv_c, g.ncz) + 1;
      w.bz1 = cellc((fminf(m.mz0, m.mz1) + D) - ez, g.z0, g.inv_c, g.ncz) - 1;
      if (w.bx0 > w.bx1) w.bz0 = 1, w.bz1 = 0;  // no inner cells: full rows
      return w;
    }
  }
  const CellBox A = m.valid0 ? A0 : A1, B = m.valid1 ? A1 : A0;
  w.ax0 = A.x0, w.ax1 = A.x1, w.az0 = A.z0, w.az1 = A.z1;
  w.bx0 = B.x0, w.bx1 = B.x1, w.bz0 = B.z0, w.bz1 = B.z1;
  w.z0 = min(A.z0, B.z0);
  w.z1 = max(A.z1, B.z1);
  return w;
}

// The two column segments of row r (empty segment: c0 > c1).
__device__ __forceinline__ void walk_row(const Walk& w, int r, int& a0, int& a1, int& b0, int& b1) {
  a0 = 1, a1 = 0, b0 = 1, b1 = 0;
  if (r < w.z0 || r > w.z1) return;
  if (w.ring) {
    if (r >= w.bz0 && r <= w.bz1) {
      a0 = w.ax0, a1 = w.bx0 - 1, b0 = w.bx1 + 1, b1 = w.ax1;
    } else {
      a0 = w.ax0, a1 = w.ax1;
    }
    return;
  }
  const bool ia = r >= w.az0 && r <= w.az1, ib = r >= w.bz0 && r <= w.bz1;
  if (ia) a0 = w.ax0, a1 = w.ax1;
  if (ib) b0 = w.bx0, b1 = w.bx1;
  if (ia && ib && w.bx0 <= w.ax1 + 1 && w.ax0 <= w.bx1 + 1) {  // touching: one merged interval
    a0 = min(w.ax0, w.bx0);
    a1 = max(w.ax1, w.bx1);
    b0 = 1, b1 = 0;
  }
}

// segf(r, c0, c1) for each non-empty segment, rows relative to the lane's window.
template <class SegF>
__device__ __forceinline__ void walk_cells(const Mover& m, const Geom& g, SegF&& segf) {
  const Walk w = make_walk(m, g);
  const int h = w.z1 - w.z0;
  for (int rel = 0; __any(rel <= h); ++rel) {  // vote over the ACTIVE lanes: wave-uniform trip count
    const int r = w.z0 + rel;
    int a0, a1, b0, b1;
    walk_row(w, r, a0, a1, b0, b1);
    segf(r, a0, a1);
    segf(r, b0, b1);
  }
}

// The per-mover evaluation over the candidates of a cell walk; `cand_old(j)` / `cand_new(j)`
// read entry j of the old / new grid through the caller's accessor.
//  (A) old grid: o at its start-of-pass position, skipped if it acted earlier in this pass;
//      before = in(L, F) over the start-of-pass state, after = in(m_new, o_old).
//  (B) new grid: only o that acted earlier in this pass (and are present after it);
//      before = in(o_new, m_old), after = in(m_new, o_new).
template <class Q, class Rows>
__device__ __forceinline__ uint32_t sweep_mover(const SweepArgs& a, Q& q, const Mover& m, Rows&& rows) {
  const float D = m.D;
  const Bounds b1 = {m.mx1 - D, m.mx1 + D, m.mz1 - D, m.mz1 + D};
  const Bounds b0 = {m.mx0 - D, m.mx0 + D, m.mz0 - D, m.mz0 + D};
  const uint32_t rq = m.q - a.base;  // o acted earlier in this pass <=> (seq_o - base) < rq
  uint32_t local = 0;
  rows(
      [&](const uint4 e, uint32_t qo) {  // old grid
        if (e.z == m.sm || qo - a.base < rq) return;
        const float ox = __uint_as_float(e.x), oz = __uint_as_float(e.y);
        const bool before = m.valid0 && ((e.w > m.q0) ? inbox(ox, oz, D, m.mx0, m.mz0) : b0.has(ox, oz));
        const bool after = m.valid1 && b1.has(ox, oz);
        if (before != after) emit(a, q, m.rank, local++, m.sm, e.z, after);
      },
      [&](const uint4 e) {  // new grid
        if (!(e.w - a.base < rq)) return;
        const float ox = __uint_as_float(e.x), oz = __uint_as_float(e.y);
        const bool before = m.valid0 && inbox(ox, oz, D, m.mx0, m.mz0);
        const bool after = m.valid1 && b1.has(ox, oz);
        if (before != after) emit(a, q, m.rank, local++, m.sm, e.z, after);
      });
  return local;
}

template <class Q>
__device__ __forceinline__ uint32_t sweep_global(const SweepArgs& a, Q& q, const Mover& m, const Geom& go,
                                                 const Geom& gn) {
  return sweep_mover(a, q, m, [&](auto&& fo, auto&& fn) {
    walk_cells(m, go, [&](int r, int c0, int c1) {
      row_entries_global(go, a.og.cs, r, c0, c1, [&](uint32_t j) { fo(a.og.ent[j], a.og.side[j]); });
    });
    walk_cells(m, gn, [&](int r, int c0, int c1) {
      row_entries_global(gn, a.ng.cs, r, c0, c1, [&](uint32_t j) { fn(a.ng.ent[j]); });
    });
  });
}

struct Region {
  int zr0, zr1, xr0, xr1, ncols, nrows, ncells;
  __device__ __forceinline__ bool holds(const CellBox& b) const {
    return b.z0 >= zr0 && b.z1 <= zr1 && b.x0 >= xr0 && b.x1 <= xr1;
  }
};

// LDS walk, written out for the hot loop: one 16-B LDS read per candidate, branch-free predicates,
// a branch only where an event is raised (rare), two candidates per iteration.
//  old-grid record {x, z, seq0, side}: skip o if (side - base) <= rank, i.e. o acted earlier in this
//  pass or o is m itself (m's own old entry carries m's op seq); the slot is read only on emit.
//  new-grid record {x, z, slot, seq}: o counts only if (seq - base) < rank (acted earlier).
__device__ __forceinline__ uint32_t sweep_lds(const SweepArgs& a, SweepSmem& sm, const Mover& m, const Region& R,
                                              const Geom& g) {
  const float D = m.D;
  const Bounds b1 = {m.mx1 - D, m.mx1 + D, m.mz1 - D, m.mz1 + D};
  const Bounds b0 = {m.mx0 - D, m.mx0 + D, m.mz0 - D, m.mz0 + D};
  const uint32_t base = a.base, rank = m.rank, q0 = m.q0;
  const bool v0 = m.valid0, v1 = m.valid1;
  const float mx0 = m.mx0, mz0 = m.mz0;
  uint32_t local = 0;
  // Predicates in VALU arithmetic: lo <= p <= hi  <=>  min(p - lo, hi - p) >= 0, exactly (the sign
  // of a binary32 difference of finite values is the sign of the exact difference when subnormals
  // are kept; x - x = +0). An invalid side is forced to -1 (false).
  const float sel0 = v0 ? 1.0f : -1.0f, sel1 = v1 ? 1.0f : -1.0f;
  auto margin = [](float px, float pz, float lx, float hx, float lz, float hz) {
    return fminf(fminf(px - lx, hx - px), fminf(pz - lz, hz - pz));
  };
  auto old_ev = [&](const uint4 c, uint32_t j) {
    const float ox = __uint_as_float(c.x), oz = __uint_as_float(c.y);
    const float am = margin(ox, oz, b0.lx, b0.hx, b0.lz, b0.hz);                 // m's perspective
    const float ao = margin(mx0, mz0, ox - D, ox + D, oz - D, oz + D);           // o's perspective
    const float bf = fminf(sel0, (c.z > q0) ? ao : am);                          // o acted last?
    const float af = fminf(sel1, margin(ox, oz, b1.lx, b1.hx, b1.lz, b1.hz));
    const bool before = bf >= 0.0f, after = af >= 0.0f;
    if ((c.w - base) > rank && before != after) emit(a, sm, rank, local++, m.sm, sm.slot_old[j], after);
  };
  auto new_ev = [&](const uint4 c) {
    const float ox = __uint_as_float(c.x), oz = __uint_as_float(c.y);
    const float bf = fminf(sel0, margin(mx0, mz0, ox - D, ox + D, oz - D, oz + D));
    const float af = fminf(sel1, margin(ox, oz, b1.lx, b1.hx, b1.lz, b1.hz));
    const bool before = bf >= 0.0f, after = af >= 0.0f;
    if ((c.w - base) < rank && before != after) emit(a, sm, rank, local++, m.sm, c.z, after);
  };
  walk_cells(m, g, [&](int r, int c0, int c1) {
    if (c0 > c1) return;
    const int b = (r - R.zr0) * R.ncols - R.xr0;
    uint32_t j = sm.lcs[0][b + c0];
    const uint32_t e = sm.lcs[0][b + c1 + 1];
    uint32_t k = sm.lcs[1][b + c0];
    const uint32_t f = sm.lcs[1][b + c1 + 1];
    for (; j + 1 < e; j += 2) {
      const uint4 c0v = sm.ent[0][j], c1v = sm.ent[0][j + 1];
      old_ev(c0v, j);
      old_ev(c1v, j + 1);
    }
    if (j < e) old_ev(sm.ent[0][j], j);
    for (; k + 1 < f; k += 2) {
      const uint4 c0v = sm.ent[1][k], c1v = sm.ent[1][k + 1];
      new_ev(c0v);
      new_ev(c1v);
    }
    if (k < f) new_ev(sm.ent[1][k]);
  });
  return local;
}

// exclusive scan of v over a kSweepBlock-thread block; *total = block sum (LDS scratch `ws`)
__device__ __forceinline__ uint32_t block_excl_scan_big(uint32_t v, uint32_t* ws, uint32_t* total) {
  constexpr int NW = kSweepBlock / 64;
  const uint32_t inc = wave_incl_scan(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) ws[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const uint32_t x = ws[k];
    pre += k < w ? x : 0u;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return pre + inc - v;
}

constexpr int kCellsPerThread = (kRegCells + kSweepBlock - 1) / kSweepBlock;

// Stage the region of grid `gi` (0 = old, 1 = new): per-cell counts from the cell starts, a block
// scan into the LDS cell-start table, then a flat copy (thread per entry: region row by binary
// search, tile part by two compares, one 16-B load). Returns the staged count (block-uniform); a
// count > kCap means "does not fit" and nothing was copied.
__device__ __forceinline__ uint32_t stage(const GridView& gv, const Geom& g, const Region& R, SweepSmem& sm, int gi) {
  uint16_t* lcs = sm.lcs[gi];
  uint32_t* gsp = sm.gsp[gi];
  const int pt0 = R.xr0 >> kTileShift;  // tile column of the region's first column
  uint32_t n[kCellsPerThread];
  uint32_t sum = 0;
  const int c0 = threadIdx.x * kCellsPerThread;
#pragma unroll
  for (int k = 0; k < kCellsPerThread; ++k) {
    const int c = c0 + k;
    n[k] = 0;
    if (c < R.ncells) {
      const int rr = c / R.ncols, col = R.xr0 + (c - rr * R.ncols);
      const uint32_t key = cell_key(g, col, R.zr0 + rr);
      const uint32_t s0 = gv.cs[key];
      n[k] = gv.cs[key + 1] - s0;
      if (col == R.xr0 || (col & (kTile - 1)) == 0) gsp[rr * 3 + ((col >> kTileShift) - pt0)] = s0;
    }
    sum += n[k];
  }
  uint32_t total;
  uint32_t pre = block_excl_scan_big(sum, sm.ws, &total);
  if (total > (uint32_t)kCap) return total;
#pragma unroll
  for (int k = 0; k < kCellsPerThread; ++k) {
    if (c0 + k < R.ncells) lcs[c0 + k] = (uint16_t)pre;
    pre += n[k];
  }
  if (threadIdx.x == 0) lcs[R.ncells] = (uint16_t)total;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < total; i += kSweepBlock) {
    int lo = 0, hi = R.nrows;  // find rr with lcs[rr * ncols] <= i < lcs[(rr + 1) * ncols]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (lcs[mid * R.ncols] <= i) lo = mid;
      else hi = mid;
    }
    const int rb = lo * R.ncols;
    // tile parts of the row start at region columns 0, then each multiple of kTile
    const int p1c = ((pt0 + 1) << kTileShift) - R.xr0, p2c = p1c + kTile;
    int p = 0, pc = 0;
    if (p1c < R.ncols && lcs[rb + p1c] <= i) {
      p = 1;
      pc = p1c;
      if (p2c < R.ncols && lcs[rb + p2c] <= i) {
        p = 2;
        pc = p2c;
      }
    }
    const uint32_t src = gsp[lo * 3 + p] + (i - lcs[rb + pc]);
    const uint4 e = gv.ent[src];
    if (gi == 0) {
      sm.ent[0][i] = make_uint4(e.x, e.y, e.w, gv.side[src]);
      sm.slot_old[i] = e.z;
    } else {
      sm.ent[1][i] = e;
    }
  }
  return total;
}

__device__ __forceinline__ bool same_geom(const Geom& a, const Geom& b) {
  return a.x0 == b.x0 && a.z0 == b.z0 && a.inv_c == b.inv_c && a.ncx == b.ncx && a.ncz == b.ncz && a.base == b.base;
}

__global__ void __launch_bounds__(kSweepBlock, 6) k_sweep(SweepArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  SweepSmem& sm = *reinterpret_cast<SweepSmem*>(smem_raw);
  if (threadIdx.x == 0) {
    sm.n = 0;
    sm.enter = 0;
  }
  if (blockIdx.x < a.ntiles) {
    const uint32_t t = blockIdx.x;
    const uint32_t e0 = a.ng.cs[t << kTileCellShift], e1 = a.ng.cs[(t + 1) << kTileCellShift];
    // does the tile hold a mover of this pass? (block-uniform exit otherwise)
    bool mine = false;
    for (uint32_t j = e0 + threadIdx.x; j < e1 && !mine; j += kSweepBlock) mine = a.ng.ent[j].w >= a.base;
    if (!__syncthreads_or(mine)) return;
    const uint32_t sp = a.ng.tile_space[t];
    const Geom gn = a.ng.geom[sp];
    const Geom go = a.og.geom[sp];
    bool lds = a.use_lds && gn.reach > 0 && same_geom(go, gn);
    Region R;
    if (lds) {
      const uint32_t tl = t - gn.tile_base;
      const int tz = (int)(tl / (uint32_t)gn.ntx), tx = (int)(tl - (uint32_t)tz * (uint32_t)gn.ntx);
      R.zr0 = max(0, tz * kTile - gn.reach);
      R.zr1 = min(gn.ncz - 1, tz * kTile + kTile - 1 + gn.reach);
      R.xr0 = max(0, tx * kTile - gn.reach);
      R.xr1 = min(gn.ncx - 1, tx * kTile + kTile - 1 + gn.reach);
      R.ncols = R.xr1 - R.xr0 + 1;
      R.nrows = R.zr1 - R.zr0 + 1;
      R.ncells = R.nrows * R.ncols;
      lds = R.ncells <= kRegCells && R.nrows <= kMaxRows && R.ncols <= kTile + 2 * kTile;
    }
    if (lds) {
      const uint32_t n_old = stage(a.og, go, R, sm, 0);
      __syncthreads();
      const uint32_t n_new = stage(a.ng, gn, R, sm, 1);
      lds = n_old <= (uint32_t)kCap && n_new <= (uint32_t)kCap;  // block-uniform
      __syncthreads();
    }
    if (a.use_lds == 2) {  // ablation (timing only): staging without the candidate walk
      for (uint32_t j = e0 + threadIdx.x; j < e1; j += kSweepBlock)
        if (a.ng.ent[j].w >= a.base) a.rank_cnt[a.ng.ent[j].w - a.base] = 0;
    } else {
      for (uint32_t j = e0 + threadIdx.x; j < e1; j += kSweepBlock) {
        const uint4 e = a.ng.ent[j];
        if (e.w < a.base) continue;  // did not act in this pass
        const Mover m = make_mover(a, e.z, e.w, true, __uint_as_float(e.x), __uint_as_float(e.y), gn.D);
        uint32_t cnt;
        if (lds && R.holds(qbox(gn, m.mx1, m.mz1)) && (!m.valid0 || R.holds(qbox(gn, m.mx0, m.mz0))))
          cnt = sweep_lds(a, sm, m, R, gn);
        else
          cnt = sweep_global(a, sm, m, go, gn);
        a.rank_cnt[m.rank] = cnt;
      }
    }
  } else {
    __syncthreads();
    const uint32_t t = (blockIdx.x - a.ntiles) * kSweepBlock + threadIdx.x;
    if (t < a.n_leaves) {
      const uint32_t i = a.leave_ops[t];
      const uint32_t smv = a.op_slot[i];
      const uint32_t sp = a.space_of[smv];
      const Geom go = a.og.geom[sp], gn = a.ng.geom[sp];
      const Mover m = make_mover(a, smv, a.base + i, false, 0.0f, 0.0f, go.D);
      a.rank_cnt[i] = sweep_global(a, sm, m, go, gn);
    }
  }
  // flush the block's events with one global atomic
  __syncthreads();
  const uint32_t nq = min(sm.n, (uint32_t)kEvLds);
  if (threadIdx.x == 0) {
    sm.base = nq ? atomicAdd(&a.ctr[CTR_EVENTS], nq) : 0u;
    if (sm.enter) atomicAdd(&a.ctr[CTR_ENTER], sm.enter);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nq; i += kSweepBlock) {
    const uint32_t gi = sm.base + i;
    if (gi < a.ev_cap) a.ev_tmp[gi] = sm.ev[i];
  }
}

void sweep_init() {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sweep), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(SweepSmem));
}

// Flat variant (use_lds == 0): one thread per new-grid entry in key (tile-major) order, 256-thread
// blocks and only the event queue in LDS, i.e. full occupancy; candidates come through L1/L2.
struct FlatQ {
  uint32_t n, enter, base, flags;
  uint4 ev[kEvLds];
};

__global__ void __launch_bounds__(kBlock) k_sweep_flat(SweepArgs a) {
  __shared__ FlatQ q;
  if (threadIdx.x == 0) {
    q.n = 0;
    q.enter = 0;
  }
  __syncthreads();
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t < a.n_new) {
    const uint4 e = a.ng.ent[t];
    if (e.w >= a.base) {
      const uint32_t sp = a.space_of[e.z];
      const Geom go = a.og.geom[sp], gn = a.ng.geom[sp];
      const Mover m = make_mover(a, e.z, e.w, true, __uint_as_float(e.x), __uint_as_float(e.y), gn.D);
      a.rank_cnt[m.rank] = sweep_global(a, q, m, go, gn);
    }
  } else if (t < a.n_new + a.n_leaves) {
    const uint32_t i = a.leave_ops[t - a.n_new];
    const uint32_t smv = a.op_slot[i];
    const uint32_t sp = a.space_of[smv];
    const Geom go = a.og.geom[sp], gn = a.ng.geom[sp];
    const Mover m = make_mover(a, smv, a.base + i, false, 0.0f, 0.0f, go.D);
    a.rank_cnt[i] = sweep_global(a, q, m, go, gn);
  }
  __syncthreads();
  const uint32_t nq = min(q.n, (uint32_t)kEvLds);
  if (threadIdx.x == 0) {
    q.base = nq ? atomicAdd(&a.ctr[CTR_EVENTS], nq) : 0u;
    if (q.enter) atomicAdd(&a.ctr[CTR_ENTER], q.enter);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nq; i += kBlock) {
    const uint32_t gi = q.base + i;
    if (gi < a.ev_cap) a.ev_tmp[gi] = q.ev[i];
  }
}

void launch_sweep(const SweepArgs& a, hipStream_t st) {
  if (a.use_lds == 0) {
    const uint32_t n = a.n_new + a.n_leaves;
    if (n) hipLaunchKernelGGL(k_sweep_flat, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
    return;
  }
  const uint32_t nb = a.ntiles + (a.n_leaves + kSweepBlock - 1) / kSweepBlock;
  if (!nb) return;
  hipLaunchKernelGGL(k_sweep, dim3(nb), dim3(kSweepBlock), sizeof(SweepSmem), st, a);
}

// ---------------------------------------------------------------------------------------------
// Canonical order: events bucketed by the mover's op rank (scan of per-rank counts), then each
// rank's slice sorted by other|kind (LEAVE = bit31 clear sorts first). Every step checks on the
// device that the sweep's events fit the buffers (else it writes nothing; the host grows them and
// re-runs), so the host synchronises once per pass. Two side jobs ride along: k_place zeroes the
// cell counts of the grid the NEXT pass builds and the next pass's counter block; k_slice_sort
// validates device-staged batches (every op's slot must carry that op's seq).
__device__ __forceinline__ bool ev_fits(const EvGuard& g, uint32_t* n) {
  *n = g.ctr[CTR_EVENTS];
  return *n <= g.tmp_cap && g.keep + *n <= g.out_cap;
}

__global__ void __launch_bounds__(kBlock) k_place(OrderArgs o) {
  const uint32_t tid = blockIdx.x * kBlock + threadIdx.x, nth = gridDim.x * kBlock;
  uint32_t n;
  // An overflowing pass is re-run from the sweep, which still reads the old grid: side jobs only
  // once the pass is final.
  if (!ev_fits(o.g, &n)) return;
  for (uint32_t i = tid; i < o.zero_n; i += nth) o.zero_cs[i] = 0u;
  if (tid < CTR_N) o.ctr_next[tid] = 0u;
  for (uint32_t i = tid; i < n; i += nth) {
    const uint4 e = o.ev_tmp[i];
    o.ev_out[o.rank_off[e.x] + e.y] = make_uint2(e.z, e.w);
  }
}

__global__ void __launch_bounds__(kBlock) k_slice_sort(OrderArgs o) {
  const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= o.n_ops) return;
  if (o.check_ops) {
    const uint32_t s = o.op_slot[r];
    if (s < o.cap && o.seq[s] != o.base + r) atomicOr(const_cast<uint32_t*>(&o.g.ctr[CTR_ERR]), ERR_DUP_SLOT);
  }
  uint32_t n;
  if (!ev_fits(o.g, &n)) return;
  const uint32_t b = o.rank_off[r], e = o.rank_off[r + 1];
  uint2* ev = o.ev_out;
  for (uint32_t i = b + 1; i < e; ++i) {
    const uint2 v = ev[i];
    uint32_t k = i;
    while (k > b && ev[k - 1].y > v.y) {
      ev[k] = ev[k - 1];
      --k;
    }
    ev[k] = v;
  }
}

// Deliver the ordered events to mapped pinned host memory (GPU-initiated PCIe writes), so the host
// needs no second round trip to learn the count before a copy.
__global__ void __launch_bounds__(kBlock) k_copy_out(OrderArgs o) {
  uint32_t n;
  if (!ev_fits(o.g, &n)) return;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) o.host_out[i] = o.ev_out[i];
}

void launch_order(const OrderArgs& o, hipStream_t st) {
  hipLaunchKernelGGL(k_place, dim3(1024), dim3(kBlock), 0, st, o);
  if (o.n_ops)
    hipLaunchKernelGGL(k_slice_sort, dim3((o.n_ops + kBlock - 1) / kBlock), dim3(kBlock), 0, st, o);
  if (o.host_out) hipLaunchKernelGGL(k_copy_out, dim3(512), dim3(kBlock), 0, st, o);
}

// ---------------------------------------------------------------------------------------------
// Relation export: row s = {o : N(s,o)} = {o : in(L, F)}, L = later actor. Count pass (row_ptr null)
// then fill pass; rows sorted afterwards.
__global__ void __launch_bounds__(kBlock) k_relation(RelArgs a) {
  const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= a.cap) return;
  const uint32_t qs = a.seq[s];
  if (!qs) {
    if (!a.row_ptr) a.row_cnt[s] = 0;
    return;
  }
  const Geom g = a.g.geom[a.space_of[s]];
  const float sx = a.pos_x[s], sz = a.pos_z[s];
  const float D = g.D;
  const Bounds bs = {sx - D, sx + D, sz - D, sz + D};
  const CellBox B = qbox(g, sx, sz);
  uint32_t n = 0;
  uint32_t w = a.row_ptr ? a.row_ptr[s] : 0u;
  for_each_entry(g, a.g.cs, true, B, false, B, [&](uint32_t j) {
    const uint4 e = a.g.ent[j];
    if (e.z == s) return;
    const float ox = __uint_as_float(e.x), oz = __uint_as_float(e.y);
    const bool in = (e.w > qs) ? inbox(ox, oz, D, sx, sz) : bs.has(ox, oz);
    if (in) {
      if (a.row_ptr) a.cols[w++] = e.z;
      ++n;
    }
  });
  if (!a.row_ptr) a.row_cnt[s] = n;
}

void launch_relation(const RelArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_relation, dim3((a.cap + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
}

__global__ void __launch_bounds__(kBlock) k_row_sort(const uint32_t* __restrict__ row_ptr, uint32_t cap,
                                                     uint32_t* __restrict__ cols) {
  const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= cap) return;
  const uint32_t b = row_ptr[s], e = row_ptr[s + 1];
  for (uint32_t i = b + 1; i < e; ++i) {
    const uint32_t v = cols[i];
    uint32_t k = i;
    while (k > b && cols[k - 1] > v) {
      cols[k] = cols[k - 1];
      --k;
    }
    cols[k] = v;
  }
}

void launch_row_sort(const uint32_t* row_ptr, uint32_t cap, uint32_t* cols, hipStream_t st) {
  hipLaunchKernelGGL(k_row_sort, dim3((cap + kBlock - 1) / kBlock), dim3(kBlock), 0, st, row_ptr, cap, cols);
}

// ---------------------------------------------------------------------------------------------
// Workload generator (bench/test tooling), bit-identical to include/gwaoi_workload.h on the host.
__global__ void __launch_bounds__(kBlock) k_wl_init(float* x, float* z, uint32_t n, uint64_t seed, float L) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  x[i] = gww_init_coord(seed, n, i, 0, L);
  z[i] = gww_init_coord(seed, n, i, 1, L);
}

__global__ void __launch_bounds__(kBlock) k_wl_step(const float* xp, const float* zp, float* xo, float* zo,
                                                    uint32_t n, uint64_t seed, uint64_t tick, float L, float s) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const float x = gww_step_coord(xp[i], seed, tick, n, i, 0, L, s);
  const float z = gww_step_coord(zp[i], seed, tick, n, i, 1, L, s);
  xo[i] = x;
  zo[i] = z;
}

__global__ void __launch_bounds__(kBlock) k_iota(uint32_t* d, uint32_t n) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) d[i] = i;
}

void launch_wl_init(float* x, float* z, uint32_t n, uint64_t seed, float L, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_wl_init, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, x, z, n, seed, L);
}
void launch_wl_step(const float* xp, const float* zp, float* xo, float* zo, uint32_t n, uint64_t seed,
                    uint64_t tick, float L, float s, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_wl_step, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, xp, zp, xo, zo, n, seed,
                       tick, L, s);
}
void launch_iota(uint32_t* d, uint32_t n, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_iota, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, d, n);
}

}  // namespace gw
