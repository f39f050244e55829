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

// Visit the entries of the cells covered by the union of box A (if va) and box B (if vb), each
// entry once: one or two contiguous segments per cell row.
template <class F>
__device__ __forceinline__ void for_each_entry(const Geom& g, const uint32_t* __restrict__ cs, bool va,
                                               CellBox A, bool vb, CellBox B, F&& f) {
  int r0 = va ? A.z0 : B.z0, r1 = va ? A.z1 : B.z1;
  if (va && vb) {
    r0 = min(A.z0, B.z0);
    r1 = max(A.z1, B.z1);
  }
  for (int r = r0; r <= r1; ++r) {
    const bool ia = va && r >= A.z0 && r <= A.z1;
    const bool ib = vb && r >= B.z0 && r <= B.z1;
    int s0, s1, t0 = 0, t1 = -1;
    if (ia && ib) {
      if (B.x0 <= A.x1 + 1 && A.x0 <= B.x1 + 1) {
        s0 = min(A.x0, B.x0);
        s1 = max(A.x1, B.x1);
      } else {
        s0 = A.x0;
        s1 = A.x1;
        t0 = B.x0;
        t1 = B.x1;
      }
    } else if (ia) {
      s0 = A.x0;
      s1 = A.x1;
    } else if (ib) {
      s0 = B.x0;
      s1 = B.x1;
    } else {
      continue;
    }
    const uint32_t row = g.base + (uint32_t)r * (uint32_t)g.ncx;
    for (uint32_t j = cs[row + s0], e = cs[row + s1 + 1]; j < e; ++j) f(j);
    if (t1 >= t0)
      for (uint32_t j = cs[row + t0], e = cs[row + t1 + 1]; j < e; ++j) f(j);
  }
}

// ---------------------------------------------------------------------------------------------
// apply: one thread per op. Records each mover's start-of-pass state, stamps its old-grid entry
// with the op's seq, and writes the new state. Slots of one pass are distinct (host guarantees it;
// device-staged batches are checked here).
__global__ void __launch_bounds__(kBlock) k_apply(ApplyArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n_ops) return;
  const uint32_t s = a.op_slot[i];
  const uint32_t q = a.base + i;
  if (i == 0) *a.rank_tail = 0u;
  const uint8_t kind = a.op_kind ? a.op_kind[i] : (uint8_t)OP_MOVE;
  if (a.check) {
    if (s >= a.cap) {
      atomicOr(&a.ctr[CTR_ERR], ERR_BAD_SLOT);
      return;
    }
    if (atomicExch(&a.stamp[s], a.batch) == a.batch) {
      atomicOr(&a.ctr[CTR_ERR], ERR_DUP_SLOT);
      return;
    }
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
  const uint32_t key = g.base + (uint32_t)cellc(a.pos_z[s], g.z0, g.inv_c, g.ncz) * (uint32_t)g.ncx +
                       (uint32_t)cellc(a.pos_x[s], g.x0, g.inv_c, g.ncx);
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
// Sweep: one thread per mover. Events are rare (~0.3 per mover per tick) but a single global counter
// hit by every event serialises at the memory side, so each block stages its events in LDS and
// reserves its output range with ONE global atomic; a mover's events are numbered in a register
// (one thread per mover), and its count is stored once, without atomics.
constexpr int kEvLds = 1024;  // events staged per block (16 KiB); overflow goes straight to global

struct EvQueue {
  uint4 ev[kEvLds];
  uint32_t n;
  uint32_t enter;
  uint32_t base;
};

__device__ __forceinline__ void emit(const SweepArgs& a, EvQueue& q, uint32_t rank, uint32_t local,
                                     uint32_t mover, uint32_t other, bool enter) {
  const uint4 rec = make_uint4(rank, local, mover, other | (enter ? 0x80000000u : 0u));
  const uint32_t li = atomicAdd(&q.n, 1u);
  if (li < (uint32_t)kEvLds) {
    q.ev[li] = rec;
  } else {
    const uint32_t gi = atomicAdd(&a.ctr[CTR_EVENTS], 1u);
    if (gi < a.ev_cap) a.ev_tmp[gi] = rec;
  }
  if (enter) atomicAdd(&q.enter, 1u);
}

// valid1: m is present after its op (not a Leave); (mx1, mz1) its new position. Returns the number
// of events m raised.
__device__ __forceinline__ uint32_t sweep_mover(const SweepArgs& a, EvQueue& eq, uint32_t sm, uint32_t q,
                                                bool valid1, float mx1, float mz1) {
  const uint32_t sp = a.space_of[sm];
  const uint32_t q0 = a.old_seq[sm];
  const bool valid0 = q0 != 0;
  const float mx0 = a.old_x[sm], mz0 = a.old_z[sm];
  const Geom go = a.og.geom[sp];
  const Geom gn = a.ng.geom[sp];
  const float D = go.D;
  const uint32_t rank = q - a.base;
  const Bounds b1 = {mx1 - D, mx1 + D, mz1 - D, mz1 + D};
  const Bounds b0 = {mx0 - D, mx0 + D, mz0 - D, mz0 + D};
  uint32_t local = 0;

  // (A) old grid: candidates o at their start-of-pass position that have not acted yet in this pass
  //     (no op, or a later op). before = in(L, F) at the start of the pass; after = in(m_new, o_old).
  {
    const CellBox A0 = qbox(go, mx0, mz0), A1 = qbox(go, mx1, mz1);
    const uint4* __restrict__ ent = a.og.ent;
    const uint32_t* __restrict__ side = a.og.side;
    for_each_entry(go, a.og.cs, valid0, A0, valid1, A1, [&](uint32_t j) {
      const uint4 e = ent[j];
      if (e.z == sm) return;
      const uint32_t qo = side[j];
      if (qo >= a.base && qo < q) return;  // o acted earlier in this pass: handled in (B)
      const float ox = __uint_as_float(e.x), oz = __uint_as_float(e.y);
      bool before = false;
      if (valid0) before = (e.w > q0) ? inbox(ox, oz, D, mx0, mz0) : b0.has(ox, oz);
      const bool after = valid1 && b1.has(ox, oz);
      if (before != after) emit(a, eq, rank, local++, sm, e.z, after);
    });
  }
  // (B) new grid: candidates o that acted earlier in this pass and are present after it.
  //     before = in(o_new, m_old) (o's op set the pair); after = in(m_new, o_new).
  {
    const CellBox B0 = qbox(gn, mx0, mz0), B1 = qbox(gn, mx1, mz1);
    const uint4* __restrict__ ent = a.ng.ent;
    for_each_entry(gn, a.ng.cs, valid0, B0, valid1, B1, [&](uint32_t j) {
      const uint4 e = ent[j];
      if (!(e.w >= a.base && e.w < q)) return;
      const float ox = __uint_as_float(e.x), oz = __uint_as_float(e.y);
      const bool before = valid0 && inbox(ox, oz, D, mx0, mz0);
      const bool after = valid1 && b1.has(ox, oz);
      if (before != after) emit(a, eq, rank, local++, sm, e.z, after);
    });
  }
  return local;
}

// Threads [0, n_new): new-grid entries (movers present after the pass are those whose seq belongs
// to this pass). Threads [n_new, n_new + n_leaves): Leave ops (absent after the pass).
__global__ void __launch_bounds__(kBlock) k_sweep(SweepArgs a) {
  __shared__ EvQueue eq;
  if (threadIdx.x == 0) {
    eq.n = 0;
    eq.enter = 0;
  }
  __syncthreads();
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t < a.n_new) {
    const uint4 e = a.ng.ent[t];
    if (e.w >= a.base) a.rank_cnt[e.w - a.base] = sweep_mover(a, eq, e.z, e.w, true, __uint_as_float(e.x),
                                                             __uint_as_float(e.y));
  } else if (t < a.n_new + a.n_leaves) {
    const uint32_t i = a.leave_ops[t - a.n_new];
    a.rank_cnt[i] = sweep_mover(a, eq, a.op_slot[i], a.base + i, false, 0.0f, 0.0f);
  }
  __syncthreads();
  const uint32_t nq = min(eq.n, (uint32_t)kEvLds);
  if (threadIdx.x == 0) {
    eq.base = nq ? atomicAdd(&a.ctr[CTR_EVENTS], nq) : 0u;
    if (eq.enter) atomicAdd(&a.ctr[CTR_ENTER], eq.enter);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nq; i += kBlock) {
    const uint32_t gi = eq.base + i;
    if (gi < a.ev_cap) a.ev_tmp[gi] = eq.ev[i];
  }
}

void launch_sweep(const SweepArgs& a, hipStream_t st) {
  const uint32_t n = a.n_new + a.n_leaves;
  if (!n) return;
  hipLaunchKernelGGL(k_sweep, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
}

// ---------------------------------------------------------------------------------------------
// Canonical order: events bucketed by the mover's op rank (scan of per-rank counts), then each
// rank's slice sorted by other|kind (LEAVE = bit31 clear sorts first).
__device__ __forceinline__ bool ev_fits(const EvGuard& g, uint32_t* n) {
  *n = g.ctr[CTR_EVENTS];
  return *n <= g.tmp_cap && g.keep + *n <= g.out_cap;
}

__global__ void __launch_bounds__(kBlock) k_place(const uint4* __restrict__ ev_tmp, EvGuard g,
                                                  const uint32_t* __restrict__ rank_off, uint2* __restrict__ ev_out) {
  uint32_t n;
  if (!ev_fits(g, &n)) return;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint4 e = ev_tmp[i];
    ev_out[rank_off[e.x] + e.y] = make_uint2(e.z, e.w);
  }
}

void launch_place(const uint4* ev_tmp, const EvGuard& g, const uint32_t* rank_off, uint2* ev_out, hipStream_t st) {
  hipLaunchKernelGGL(k_place, dim3(1024), dim3(kBlock), 0, st, ev_tmp, g, rank_off, ev_out);
}

__global__ void __launch_bounds__(kBlock) k_slice_sort(const uint32_t* __restrict__ rank_off, uint32_t n_ops,
                                                       EvGuard g, uint2* __restrict__ ev) {
  const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
  uint32_t n;
  if (r >= n_ops || !ev_fits(g, &n)) return;
  const uint32_t b = rank_off[r], e = rank_off[r + 1];
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

void launch_slice_sort(const uint32_t* rank_off, uint32_t n_ops, const EvGuard& g, uint2* ev_out, hipStream_t st) {
  if (!n_ops) return;
  hipLaunchKernelGGL(k_slice_sort, dim3((n_ops + kBlock - 1) / kBlock), dim3(kBlock), 0, st, rank_off, n_ops, g,
                     ev_out);
}

// Deliver the ordered events to mapped pinned host memory (GPU-initiated PCIe writes), so the host
// needs no second round trip to learn the count before a copy.
__global__ void __launch_bounds__(kBlock) k_copy_out(const uint2* __restrict__ ev, EvGuard g, uint2* host) {
  uint32_t n;
  if (!ev_fits(g, &n)) return;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) host[i] = ev[i];
}

void launch_copy_out(const uint2* ev_out, const EvGuard& g, uint2* host_mapped, hipStream_t st) {
  hipLaunchKernelGGL(k_copy_out, dim3(512), dim3(kBlock), 0, st, ev_out, g, host_mapped);
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
