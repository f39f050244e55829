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

// The same rows as [begin, end) record ranges: f(b, e) once per tile crossed.
template <class F>
__device__ __forceinline__ void row_entries_ranges(const Geom& g, const uint32_t* __restrict__ cs, int r, int c0,
                                                   int c1, F&& f) {
  if (c0 > c1) return;
  const uint32_t rowbase = g.base + ((uint32_t)((r >> kTileShift) * g.ntx) << kTileCellShift) +
                           (uint32_t)((r & (kTile - 1)) << kTileShift);
  for (int tx = c0 >> kTileShift; tx <= (c1 >> kTileShift); ++tx) {
    const int lo = max(c0, tx << kTileShift), hi = min(c1, (tx << kTileShift) + kTile - 1);
    const uint32_t k = rowbase + ((uint32_t)tx << kTileCellShift) + (uint32_t)(lo & (kTile - 1));
    f(cs[k], cs[k + (uint32_t)(hi - lo) + 1]);
  }
}

// A Space's geometry as block-uniform values: every field read through readfirstlane, so the
// compiler keeps them (and what is derived from them) in scalar registers. The loads themselves are
// vector loads (the kernels also store to global memory, so the compiler does not use the scalar
// cache for them), and without this the fields stay in VGPRs.
__device__ __forceinline__ Geom uniform_geom(const Geom* p) {
  const Geom v = *p;
  Geom g;
  g.x0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.x0)));
  g.z0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.z0)));
  g.inv_c = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.inv_c)));
  g.D = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.D)));
  g.ncx = __builtin_amdgcn_readfirstlane(v.ncx);
  g.ncz = __builtin_amdgcn_readfirstlane(v.ncz);
  g.ntx = __builtin_amdgcn_readfirstlane(v.ntx);
  g.ntz = __builtin_amdgcn_readfirstlane(v.ntz);
  g.base = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.base);
  g.tile_base = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.tile_base);
  g.reach = __builtin_amdgcn_readfirstlane(v.reach);
  g.pad = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.pad);
  return g;
}

// Inclusive wave64 scan through DPP lane moves (row_shr 1/2/4/8 inside rows of 16 lanes, then
// row_bcast 15/31 across rows: gfx9 wave64 DPP), i.e. VALU ops instead of the six LDS-crossbar round
// trips of __shfl_up (dense walk: skew 3.07 -> 2.90 ms; k_sweep's staging scans: 95.1 -> 93.8 us).
// Every lane of the wave must be active.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63, rl = lane & 15;
  int t;
  t = __builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  if (rl >= 1) v += (uint32_t)t;
  t = __builtin_amdgcn_mov_dpp((int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  if (rl >= 2) v += (uint32_t)t;
  t = __builtin_amdgcn_mov_dpp((int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  if (rl >= 4) v += (uint32_t)t;
  t = __builtin_amdgcn_mov_dpp((int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  if (rl >= 8) v += (uint32_t)t;
  t = __builtin_amdgcn_mov_dpp((int)v, 0x142, 0xf, 0xf, false);  // row_bcast:15
  if ((lane & 31) >= 16) v += (uint32_t)t;
  t = __builtin_amdgcn_mov_dpp((int)v, 0x143, 0xf, 0xf, false);  // row_bcast:31
  if (lane >= 32) v += (uint32_t)t;
  return v;
}

// Inclusive wave64 max-scan (the same DPP lane moves as wave_incl_scan). Every lane must be active.
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  const int lane = threadIdx.x & 63, rl = lane & 15;
  int t;
  t = __builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  if (rl >= 1) v = max(v, (uint32_t)t);
  t = __builtin_amdgcn_mov_dpp((int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  if (rl >= 2) v = max(v, (uint32_t)t);
  t = __builtin_amdgcn_mov_dpp((int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  if (rl >= 4) v = max(v, (uint32_t)t);
  t = __builtin_amdgcn_mov_dpp((int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  if (rl >= 8) v = max(v, (uint32_t)t);
  t = __builtin_amdgcn_mov_dpp((int)v, 0x142, 0xf, 0xf, false);  // row_bcast:15
  if ((lane & 31) >= 16) v = max(v, (uint32_t)t);
  t = __builtin_amdgcn_mov_dpp((int)v, 0x143, 0xf, 0xf, false);  // row_bcast:31
  if (lane >= 32) v = max(v, (uint32_t)t);
  return v;
}

// Owners of positions w0 + lane and w0 + 64 + lane of a stream that the lanes' ranges [excl, excl + cnt)
// concatenate in lane order (positions past the stream get the last lane with a range): each lane whose
// range starts inside the window marks its start in the wave's LDS row (128 words), then a max-scan over
// the marks in lane order; positions before the first mark belong to the lane holding position w0. Two LDS
// writes, two reads and two DPP scans instead of two binary searches of six dependent lane moves.
// Every lane must be active.
__device__ __forceinline__ void stream_owners(uint32_t* row, uint32_t excl, uint32_t cnt, uint32_t w0, int& o0,
                                              int& o1) {
  const int lane = threadIdx.x & 63;
  row[lane] = 0u;
  row[64 + lane] = 0u;
  __builtin_amdgcn_wave_barrier();
  if (cnt && excl >= w0 && excl < w0 + 128u) row[excl - w0] = (uint32_t)lane + 1u;  // (starts are distinct)
  __builtin_amdgcn_wave_barrier();
  const unsigned long long before = __ballot(cnt != 0u && excl <= w0);
  const uint32_t carry = before ? (uint32_t)(64 - __clzll((long long)before)) : 1u;  // lane + 1
  const uint32_t s0 = wave_incl_max(row[lane]), s1 = wave_incl_max(row[64 + lane]);
  const uint32_t m0 = (uint32_t)__builtin_amdgcn_readlane((int)s0, 63);
  o0 = (int)max(carry, s0) - 1;
  o1 = (int)max(max(carry, m0), s1) - 1;
  __builtin_amdgcn_wave_barrier();  // the row's reads before its next writes
}

// q = n / d for 0 <= n < 2^20, 1 <= d < 2^11 (region cell indices): float reciprocal, then one
// correction step each way (exact; avoids the ~30-instruction integer division sequence)
__device__ __forceinline__ int small_div(int n, int d) {
  int q = (int)(((float)n + 0.5f) * (1.0f / (float)d));
  q -= (q * d > n) ? 1 : 0;
  q += ((q + 1) * d <= n) ? 1 : 0;
  return q;
}

// Stage the records of a tile's region (cells [cx0, cx0 + W) x [cz0, cz0 + ncell / W), row-major) into
// LDS in row-major cell order, so the cells [x0, x1] of region row r are ONE contiguous LDS range
// [cst[r W + x0], cst[r W + x1 + 1]). load(q) gives the staged form of global record q. Every thread of
// the block calls it; it ends with a barrier. Returns false (block-uniform, nothing staged) when the
// region holds more than `cap` records. red: kThreads / 64 words of LDS scratch.
// Each thread takes kPer consecutive cells; every cell-start load is issued up front, and the
// records are then gathered by a flat pass (thread per staged record, its loads issued together), so
// the staging costs a few memory round trips instead of one per cell and per record.
template <int kThreads, int kMaxCells, int kMaxRecs, class Load>
__device__ bool stage_region(const Geom& g, const uint32_t* __restrict__ cs, int cx0, int cz0, int W, int ncell,
                             uint16_t* cst, uint4* out, uint32_t* red, uint32_t* tot_sh, Load&& load) {
  constexpr int kPer = (kMaxCells + kThreads - 1) / kThreads;
  constexpr int kIters = (kMaxRecs + kThreads - 1) / kThreads;
  const int c0 = threadIdx.x * kPer;
  uint32_t s0[kPer], n[kPer];
  uint32_t sum = 0;
  const int rr0 = small_div(c0, W), col0 = c0 - rr0 * W;
  {
    int rr = rr0, col = col0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      s0[k] = 0;
      n[k] = 0;
      if (c0 + k < ncell) {
        const uint32_t key = cell_key(g, cx0 + col, cz0 + rr);
        s0[k] = cs[key];
        n[k] = cs[key + 1] - s0[k];
      }
      sum += n[k];
      if (++col == W) col = 0, ++rr;
    }
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
  const bool fits = tot <= (uint32_t)kMaxRecs;
  if (!fits) return false;  // block-uniform
  uint32_t p = inc - sum;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    if (c0 + k < ncell) cst[c0 + k] = (uint16_t)p;
    for (uint32_t q = 0; q < n[k]; ++q) out[p + q].x = s0[k] + q;  // source map, gathered below
    p += n[k];
  }
  if (threadIdx.x == 0) cst[ncell] = (uint16_t)tot;
  __syncthreads();
  uint32_t src[kIters];
#pragma unroll
  for (int k = 0; k < kIters; ++k) {
    const uint32_t i = threadIdx.x + k * kThreads;
    src[k] = i < tot ? out[i].x : 0u;
  }
  uint4 v[kIters];
#pragma unroll
  for (int k = 0; k < kIters; ++k) {
    const uint32_t i = threadIdx.x + k * kThreads;
    if (i < tot) v[k] = load(src[k]);
  }
#pragma unroll
  for (int k = 0; k < kIters; ++k) {
    const uint32_t i = threadIdx.x + k * kThreads;
    if (i < tot) out[i] = v[k];
  }
  __syncthreads();
  return true;
}

}  // namespace gw
