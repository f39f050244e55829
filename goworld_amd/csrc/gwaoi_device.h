// gwaoi_device.h — device helpers shared by the gfx950 kernels (gwaoi_kernels.hip: pipeline and
// relation; gwaoi_sync.hip: tick-end sync fan-out and position ingest): cell mapping, the exact
// float32 box predicate of go-aoi's XZListAOIManager, and the global-memory row walk over the grid.
#pragma once

#include <hip/hip_runtime.h>

#include "gwaoi_internal.h"

namespace gw {

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

// cellc for the UPPER bound of a range: a NaN bound (from an infinite coordinate; the ABI rejects
// non-finite coordinates, so only a corrupted state gets here) widens to the last cell instead of
// collapsing to cell 0, so a cell range is never narrower than the exact predicate needs.
__device__ __forceinline__ int cellc_hi(float v, float o, float inv, int n) {
  float f = (v - o) * inv;
  if (!(f < (float)n)) return n - 1;
  if (!(f >= 0.0f)) return 0;
  return (int)f;
}

// in(c, p): p inside the box of an entity at c (go-aoi Mark/GetClearMarkedNeighbors bounds).
__device__ __forceinline__ bool inbox(float cx, float cz, float D, float px, float pz) {
  const float lx = cx - D, hx = cx + D, lz = cz - D, hz = cz + D;
  return px >= lx && px <= hx && pz >= lz && pz <= hz;
}

struct CellBox {
  int x0, x1, z0, z1;
};

__device__ __forceinline__ CellBox qbox(const Geom& g, float cx, float cz) {
  const float mx = (fabsf(cx) + g.D) * kMargin, mz = (fabsf(cz) + g.D) * kMargin;
  CellBox b;
  b.x0 = cellc((cx - g.D) - mx, g.x0, g.inv_c, g.ncx);
  b.x1 = cellc_hi((cx + g.D) + mx, g.x0, g.inv_c, g.ncx);
  b.z0 = cellc((cz - g.D) - mz, g.z0, g.inv_c, g.ncz);
  b.z1 = cellc_hi((cz + g.D) + mz, g.z0, g.inv_c, g.ncz);
  return b;
}

__device__ __forceinline__ uint32_t cell_key(const Geom& g, int cx, int cz) {
  return g.base + ((uint32_t)((cz >> kTileShift) * g.ntx + (cx >> kTileShift)) << kTileCellShift) +
         (uint32_t)(((cz & (kTile - 1)) << kTileShift) | (cx & (kTile - 1)));
}

__device__ __forceinline__ uint32_t cell_key_of(const Geom& g, float x, float z) {
  return cell_key(g, cellc(x, g.x0, g.inv_c, g.ncx), cellc(z, g.z0, g.inv_c, g.ncz));
}

// Global-memory path: records of row r, columns [c0, c1]: one contiguous segment per tile crossed.
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

// Stage the records of a tile's region (cells [cx0, cx0 + W) x [cz0, cz0 + ncell / W), row-major) into
// LDS in row-major cell order, so the cells [x0, x1] of region row r are ONE contiguous LDS range
// [cst[r W + x0], cst[r W + x1 + 1]). load(q) gives the staged form of global record q. Every thread of
// the block calls it; it ends with a barrier. Returns false (block-uniform, nothing staged) when the
// region holds more than `cap` records. red: kThreads / 64 words of LDS scratch.
template <int kThreads, int kMaxCells, class Load>
__device__ bool stage_region(const Geom& g, const uint32_t* __restrict__ cs, int cx0, int cz0, int W, int ncell,
                             uint16_t* cst, uint4* out, uint32_t cap, uint32_t* red, uint32_t* tot_sh, Load&& load) {
  constexpr int kPer = (kMaxCells + kThreads - 1) / kThreads;
  const int c0 = threadIdx.x * kPer, c1 = min(c0 + kPer, ncell);
  uint32_t sum = 0;
  for (int i = c0; i < c1; ++i) {
    const uint32_t k = cell_key(g, cx0 + i % W, cz0 + i / W);
    sum += cs[k + 1] - cs[k];
  }
  const int lane = threadIdx.x & 63;
  uint32_t inc = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  if (lane == 63) red[threadIdx.x >> 6] = inc;
  __syncthreads();
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) inc += red[w];
  if (threadIdx.x == kThreads - 1) *tot_sh = inc;
  __syncthreads();
  const uint32_t tot = *tot_sh;
  const bool fits = tot <= cap;
  if (fits) {
    uint32_t p = inc - sum;
    for (int i = c0; i < c1; ++i) {
      const uint32_t k = cell_key(g, cx0 + i % W, cz0 + i / W);
      cst[i] = (uint16_t)p;
      for (uint32_t q = cs[k], e = cs[k + 1]; q < e; ++q, ++p) out[p] = load(q);
    }
    if (threadIdx.x == 0) cst[ncell] = (uint16_t)tot;
  }
  __syncthreads();
  return fits;
}

}  // namespace gw
