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
// and emits ENTER/LEAVE(m,o) where they differ.
//
// One cell-sorted grid per pass holds, for every entity, a record binned at its END-of-pass cell
// carrying both its start- and end-of-pass state; an entity whose start cell differs (or that left)
// also gets a "ghost" record at its start cell. Every candidate is then met once, in the cell of
// the position that matters for the pair (start position if it has not acted yet, end position
// if it has).
//
// Float semantics: every bound is one binary32 add/sub (built with -ffp-contract=off, denormals
// preserved), compared inclusively — bit-exact with Go float32 arithmetic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <type_traits>

#include "gwaoi_device.h"
#include "gwaoi_internal.h"
#include "gwaoi_workload.h"

namespace gw {

constexpr int kBlock = 256;
// ---------------------------------------------------------------------------------------------
// apply: one thread per op. Records the slot's start-of-pass state and this pass's op seq, then
// writes the end-of-pass state. Slots of one pass are distinct (the host guarantees it for
// host-staged ops; for device-staged batches k_slice_sort checks afterwards that every op's slot
// carries that op's seq — a duplicate leaves one of two ops without it).
// lane-aggregated append: one atomic per wave for the lanes with `pred`; returns this lane's slot
__device__ __forceinline__ uint32_t wave_append(uint32_t* ctr, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (!m) return 0u;
  const int leader = __ffsll((long long)m) - 1;
  const int lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// An op's event count for the canonical order: only non-zero counts are stored (k_apply zeroed them).
// (Also adding each count to its scan chunk's sum here, so the order's scan needs no reduce pass:
// k_sweep 90 -> 107 us at config 2, the device-scope atomics cost more than the pass they save.)
__device__ __forceinline__ void put_count(uint32_t* rank_cnt, uint32_t rank, uint32_t cnt) {
  if (cnt) rank_cnt[rank] = cnt;
}

// Small pass: slot s's overlay record after its op (seq q; q0 = its seq before, 0 = absent): the main
// record a grid build would write at its end position (start state in .b), or for a Leave its ghost at
// the start position. The slot joins the overlay the first time it has an op since the grid was built.
__device__ __forceinline__ void overlay_put(const ApplyArgs& a, uint32_t s, uint8_t kind, uint32_t q, uint32_t q0,
                                            float x0, float z0, float x1, float z1) {
  uint32_t e;
  if (a.ov_tag[s] == a.gen) {
    e = a.ov_idx[s];
  } else {
    e = atomicAdd(a.ov_count, 1u);  // (small passes only: a few ops)
    a.ov_tag[s] = a.gen;
    a.ov_idx[s] = e;
  }
  if (e >= a.ov_cap) return;  // (the host bounds the overlay below ov_cap)
  const bool leave = kind == OP_LEAVE;
  const uint4 ra = make_uint4(__float_as_uint(leave ? x0 : x1), __float_as_uint(leave ? z0 : z1),
                              s | (leave ? REC_GHOST : 0u), q);
  const uint4 rb = make_uint4(__float_as_uint(q0 ? x0 : x1), __float_as_uint(q0 ? z0 : z1), q0, leave ? 0u : q);
  a.ov_rec[e] = Rec{ra, rb};
}

__global__ void __launch_bounds__(kBlock) k_apply(ApplyArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t n_real = a.n_dev ? *a.n_dev : a.n_ops;
  const bool live = i < a.n_ops && i < n_real;
  if (i == 0) {
    a.ctr[CTR_NOPS] = min(n_real, a.n_ops);
    if (n_real > a.n_ops) atomicOr(&a.ctr[CTR_ERR], ERR_BAD_COUNT);
    a.rank_cnt[a.n_ops] = 0u;
  }
  if (i < a.n_ops) a.rank_cnt[i] = 0u;  // the sweep stores only non-zero event counts
  uint32_t s = 0, q0 = 0;
  uint8_t kind = OP_MOVE;
  bool ok = live;
  if (live) {
    s = a.op_slot[i];
    const uint8_t raw = a.op_kind ? a.op_kind[i] : (uint8_t)OP_MOVE;
    kind = (uint8_t)(raw & OP_KIND);
    if (a.cp_slot) {  // host ops read over PCIe: device copies for the kernels after this one
      a.cp_slot[i] = s;
      a.cp_kind[i] = raw;
    }
    if (a.check && s >= a.cap) {
      atomicOr(&a.ctr[CTR_ERR], ERR_BAD_SLOT);
      ok = false;
    } else {
      q0 = a.seq[s];
      if (a.check && kind == OP_ENTER && q0 != 0) {
        atomicOr(&a.ctr[CTR_ERR], ERR_PRESENT_SLOT);
        ok = false;
      } else if (a.check && kind != OP_ENTER && q0 == 0) {
        atomicOr(&a.ctr[CTR_ERR], ERR_ABSENT_SLOT);
        ok = false;
      } else if (a.check && kind == OP_ENTER && a.op_space && a.op_space[i] >= a.nspaces) {
        atomicOr(&a.ctr[CTR_ERR], ERR_BAD_SPACE);
        ok = false;
      } else if (a.check && kind != OP_LEAVE &&
                 !(finite_bits(__float_as_uint(a.op_x[i])) && finite_bits(__float_as_uint(a.op_z[i])))) {
        atomicOr(&a.ctr[CTR_ERR], ERR_BAD_COORD);
        ok = false;
      }
    }
  }
  if (a.leaves) {  // device-staged mixed batch: Leave list and presence delta on the device (wave-uniform)
    const bool lv = ok && kind == OP_LEAVE;
    const uint32_t j = wave_append(&a.ctr[CTR_LEAVES], lv);
    if (lv) a.leaves[j] = i;
    const unsigned long long ent = __ballot(ok && kind == OP_ENTER), lea = __ballot(lv);
    if ((threadIdx.x & 63) == 0 && (ent | lea))
      atomicAdd(&a.ctr[CTR_PRESENT], (uint32_t)__popcll(ent) - (uint32_t)__popcll(lea));
  }
  if (!ok) return;
  const uint32_t q = a.base + i;
  const float x0 = a.pos_x[s], z0 = a.pos_z[s];
  a.old_x[s] = x0;
  a.old_z[s] = z0;
  a.old_seq[s] = q0;
  a.opq[s] = q;
  if (kind == OP_LEAVE) {
    a.seq[s] = 0;
  } else {
    a.pos_x[s] = a.op_x[i];
    a.pos_z[s] = a.op_z[i];
    a.seq[s] = q;
    if (kind == OP_ENTER) a.space_of[s] = a.op_space ? a.op_space[i] : 0u;
  }
  if (a.ov_rec) overlay_put(a, s, kind, q, q0, x0, z0, kind == OP_LEAVE ? x0 : a.op_x[i], kind == OP_LEAVE ? z0 : a.op_z[i]);
}

// Moved-only batches (no kinds, no Leave list) with 16-B aligned op arrays: four ops per thread. A
// group whose slots are four consecutive slots from a multiple of 4 (a batch in slot order) moves every
// per-slot array with 16-B accesses; any other group, or one failing a check, takes the per-op path
// (which raises the error flags).
__device__ __forceinline__ void apply_move(const ApplyArgs& a, uint32_t i) {
  const uint32_t s = a.op_slot[i];
  if (a.check && s >= a.cap) {
    atomicOr(&a.ctr[CTR_ERR], ERR_BAD_SLOT);
    return;
  }
  const uint32_t q0 = a.seq[s];
  const float x = a.op_x[i], z = a.op_z[i];
  if (a.check && q0 == 0) {
    atomicOr(&a.ctr[CTR_ERR], ERR_ABSENT_SLOT);
    return;
  }
  if (a.check && !(finite_bits(__float_as_uint(x)) && finite_bits(__float_as_uint(z)))) {
    atomicOr(&a.ctr[CTR_ERR], ERR_BAD_COORD);
    return;
  }
  const uint32_t q = a.base + i;
  a.old_x[s] = a.pos_x[s];
  a.old_z[s] = a.pos_z[s];
  a.old_seq[s] = q0;
  a.opq[s] = q;
  a.pos_x[s] = x;
  a.pos_z[s] = z;
  a.seq[s] = q;
}

__global__ void __launch_bounds__(kBlock) k_apply_moves4(ApplyArgs a) {
  const uint32_t i0 = 4u * (blockIdx.x * kBlock + threadIdx.x);
  const uint32_t n_real = a.n_dev ? *a.n_dev : a.n_ops;
  const uint32_t n = min(n_real, a.n_ops);
  if (i0 == 0) {
    a.ctr[CTR_NOPS] = n;
    if (n_real > a.n_ops) atomicOr(&a.ctr[CTR_ERR], ERR_BAD_COUNT);
    a.rank_cnt[a.n_ops] = 0u;
  }
  if (i0 >= a.n_ops) return;
  if (i0 + 4 <= a.n_ops) {  // the sweep stores only non-zero event counts
    *reinterpret_cast<uint4*>(&a.rank_cnt[i0]) = make_uint4(0u, 0u, 0u, 0u);
  } else {
    for (uint32_t i = i0; i < a.n_ops; ++i) a.rank_cnt[i] = 0u;
  }
  if (i0 + 4 <= n) {
    const uint4 sl = *reinterpret_cast<const uint4*>(&a.op_slot[i0]);
    if ((sl.x & 3u) == 0 && sl.y == sl.x + 1 && sl.z == sl.x + 2 && sl.w == sl.x + 3 && sl.w < a.cap) {
      const uint32_t s = sl.x;
      const uint4 q0 = *reinterpret_cast<const uint4*>(&a.seq[s]);
      const float4 px = *reinterpret_cast<const float4*>(&a.pos_x[s]);
      const float4 pz = *reinterpret_cast<const float4*>(&a.pos_z[s]);
      const float4 ox = *reinterpret_cast<const float4*>(&a.op_x[i0]);
      const float4 oz = *reinterpret_cast<const float4*>(&a.op_z[i0]);
      auto fin = [](float v) { return finite_bits(__float_as_uint(v)); };
      const bool ok = !a.check || (q0.x && q0.y && q0.z && q0.w && fin(ox.x) && fin(ox.y) && fin(ox.z) && fin(ox.w) &&
                                   fin(oz.x) && fin(oz.y) && fin(oz.z) && fin(oz.w));
      if (ok) {
        const uint32_t q = a.base + i0;
        const uint4 qn = make_uint4(q, q + 1, q + 2, q + 3);
        *reinterpret_cast<float4*>(&a.old_x[s]) = px;
        *reinterpret_cast<float4*>(&a.old_z[s]) = pz;
        *reinterpret_cast<uint4*>(&a.old_seq[s]) = q0;
        *reinterpret_cast<uint4*>(&a.opq[s]) = qn;
        *reinterpret_cast<float4*>(&a.pos_x[s]) = ox;
        *reinterpret_cast<float4*>(&a.pos_z[s]) = oz;
        *reinterpret_cast<uint4*>(&a.seq[s]) = qn;
        return;
      }
    }
  }
  for (uint32_t i = i0; i < i0 + 4 && i < n; ++i) apply_move(a, i);
}

void launch_apply(const ApplyArgs& a, hipStream_t st) {
  if (!a.n_ops) return;
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  if (!a.op_kind && !a.leaves && !a.ov_rec && al16(a.op_slot) && al16(a.op_x) && al16(a.op_z)) {
    const uint32_t groups = (a.n_ops + 3) / 4;
    hipLaunchKernelGGL(k_apply_moves4, dim3((groups + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
    return;
  }
  hipLaunchKernelGGL(k_apply, dim3((a.n_ops + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
}

// ---------------------------------------------------------------------------------------------
// The pass's grid: counting sort of records by cell key. Per slot: a main record at its end cell
// (if present at the end) and a ghost record at its start cell (if present at the start and its
// start cell differs, or it left). Count (atomics rank records inside a cell), scan, scatter.
//   ra = {x_bin, z_bin, slot | flags, opq}     rb = {x_start, z_start, seq_start, seq_end}
struct SlotState {
  bool acted, p_start, p_end;
  float x0, z0, x1, z1;
  uint32_t q0, q1, oq;
};

// (the start-of-pass fields are loaded whatever opq says, so all seven loads of a slot are in flight
// together instead of waiting for opq first)
__device__ __forceinline__ SlotState slot_state(const BinArgs& a, uint32_t s) {
  SlotState t;
  t.oq = a.opq[s];
  t.q1 = a.seq[s];
  t.x1 = a.pos_x[s];
  t.z1 = a.pos_z[s];
  const uint32_t q0 = a.old_seq[s];
  const float x0 = a.old_x[s], z0 = a.old_z[s];
  t.acted = (t.oq - a.base) < a.n_ops;
  t.p_end = t.q1 != 0;
  t.q0 = t.acted ? q0 : t.q1;
  t.x0 = t.acted ? x0 : t.x1;
  t.z0 = t.acted ? z0 : t.z1;
  t.p_start = t.q0 != 0;
  return t;
}

__global__ void __launch_bounds__(kBlock) k_bin_count(BinArgs a) {
  const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= a.cap) return;
  const SlotState t = slot_state(a, s);
  uint32_t k1 = kNoKey, k0 = kNoKey;
  if (t.p_end || t.p_start) {
    const Geom g = a.geom[a.space_of[s]];
    if (t.p_end) k1 = cell_key_of(g, t.x1, t.z1);
    if (t.p_start) k0 = cell_key_of(g, t.x0, t.z0);
    if (k0 == k1) k0 = kNoKey;  // no ghost: the main record's cell is the start cell
    if (k1 != kNoKey) a.local_of[2 * s] = atomicAdd(&a.cs[k1], 1u);
    if (k0 != kNoKey) a.local_of[2 * s + 1] = atomicAdd(&a.cs[k0], 1u);
  }
  a.key_of[2 * s] = k1;
  a.key_of[2 * s + 1] = k0;
}

__global__ void __launch_bounds__(kBlock) k_bin_scatter(BinArgs a) {
  const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= a.cap) return;
  const uint32_t k1 = a.key_of[2 * s], k0 = a.key_of[2 * s + 1];
  if (k1 == kNoKey && k0 == kNoKey) return;
  const SlotState t = slot_state(a, s);
  const uint4 rb = make_uint4(__float_as_uint(t.x0), __float_as_uint(t.z0), t.q0, t.q1);
  if (k1 != kNoKey) {
    const uint32_t j = a.cs[k1] + a.local_of[2 * s];
    a.rec[j] = Rec{make_uint4(__float_as_uint(t.x1), __float_as_uint(t.z1), s | (k0 != kNoKey ? REC_HASG : 0u), t.oq), rb};
  }
  if (k0 != kNoKey) {
    const uint32_t j = a.cs[k0] + a.local_of[2 * s + 1];
    a.rec[j] = Rec{make_uint4(__float_as_uint(t.x0), __float_as_uint(t.z0), s | REC_GHOST, t.oq), rb};
  }
}

void launch_bin_count(const BinArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_bin_count, dim3((a.cap + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
}
void launch_bin_scatter(const BinArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_bin_scatter, dim3((a.cap + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
}

// ---------------------------------------------------------------------------------------------
// Exclusive scan (u32) building blocks: wave64 prefix sums, block scan over 256 threads.

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

// Two-kernel scan: k_scan_reduce writes each chunk's sum to part[]; k_scan_apply has every block sum
// the part[] entries before its chunk itself (at most kScanMaxChunks plain loads from L2, one or a
// few per thread) and scan its chunk. (A single-pass version that waits on published chunk
// aggregates through agent-scope atomics measured 3-6x slower here.) IPT items per thread keep the
// chunk count <= kScanMaxChunks up to 16.7M items.
constexpr uint32_t kScanMaxChunks = 1024;

template <int IPT>
__device__ __forceinline__ void scan_load(const uint32_t* __restrict__ d, uint32_t n, uint32_t b0, uint32_t (&v)[IPT]) {
  if (b0 + IPT <= n) {
#pragma unroll
    for (int k = 0; k < IPT; k += 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(d + b0 + k);
      v[k] = q.x, v[k + 1] = q.y, v[k + 2] = q.z, v[k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < IPT; ++k) v[k] = (b0 + k < n) ? d[b0 + k] : 0u;
  }
}

template <int IPT>
__global__ void __launch_bounds__(kBlock) k_scan_reduce(const uint32_t* __restrict__ d, uint32_t n,
                                                        uint32_t* __restrict__ part) {
  uint32_t v[IPT];
  scan_load<IPT>(d, n, (blockIdx.x * kBlock + threadIdx.x) * IPT, v);
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) sum += v[k];
  uint32_t tot;
  block_excl_scan(sum, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

template <int IPT>
__global__ void __launch_bounds__(kBlock) k_scan_apply(uint32_t* __restrict__ d, uint32_t n,
                                                       const uint32_t* __restrict__ part) {
  uint32_t before = 0;
  for (uint32_t p = threadIdx.x; p < blockIdx.x; p += kBlock) before += part[p];
  const uint32_t b0 = (blockIdx.x * kBlock + threadIdx.x) * IPT;
  uint32_t v[IPT];
  scan_load<IPT>(d, n, b0, v);
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) sum += v[k];
  uint32_t tot_before, tot;
  block_excl_scan(before, &tot_before);
  uint32_t pre = block_excl_scan(sum, &tot) + tot_before;
  if (b0 + IPT <= n) {
#pragma unroll
    for (int k = 0; k < IPT; k += 4) {
      uint4 q;
      q.x = pre, pre += v[k];
      q.y = pre, pre += v[k + 1];
      q.z = pre, pre += v[k + 2];
      q.w = pre, pre += v[k + 3];
      *reinterpret_cast<uint4*>(d + b0 + k) = q;
    }
  } else {
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      if (b0 + k < n) d[b0 + k] = pre;
      pre += v[k];
    }
  }
}

// Short arrays (n <= kScanOneMax: tile totals, block counts) in ONE kernel of one 1024-thread block,
// 32 items per thread: a launch less than the two-kernel scan, whose second kernel alone costs a
// dispatch (~4.7 us of a tick's stream time each, r04_c24 kernel stats).
#ifndef GW_SCAN_ONE_MAX
#define GW_SCAN_ONE_MAX 8192  // (32768, i.e. the fan-out's tile totals too: count stage +2.5 us, r04_c27)
#endif
constexpr int kScanOneThreads = 1024, kScanOneIpt = 32;
constexpr uint32_t kScanOneMax = GW_SCAN_ONE_MAX;
static_assert(kScanOneMax <= (uint32_t)kScanOneThreads * kScanOneIpt, "one block's items");

__global__ void __launch_bounds__(kScanOneThreads) k_scan_one(uint32_t* __restrict__ d, uint32_t n) {
  __shared__ uint32_t ws[kScanOneThreads / 64];
  const uint32_t b0 = threadIdx.x * kScanOneIpt;
  uint32_t v[kScanOneIpt];
  scan_load<kScanOneIpt>(d, n, b0, v);
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < kScanOneIpt; ++k) sum += v[k];
  const uint32_t inc = wave_incl_scan(sum);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) ws[w] = inc;
  __syncthreads();
  uint32_t pre = inc - sum;
  for (int k = 0; k < w; ++k) pre += ws[k];
  if (b0 + kScanOneIpt <= n) {
#pragma unroll
    for (int k = 0; k < kScanOneIpt; k += 4) {
      uint4 q;
      q.x = pre, pre += v[k];
      q.y = pre, pre += v[k + 1];
      q.z = pre, pre += v[k + 2];
      q.w = pre, pre += v[k + 3];
      *reinterpret_cast<uint4*>(d + b0 + k) = q;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kScanOneIpt; ++k) {
      if (b0 + k < n) d[b0 + k] = pre;
      pre += v[k];
    }
  }
}

static uint32_t scan_ipt(uint32_t n) {
  for (uint32_t ipt : {4u, 16u})
    if ((n + kBlock * ipt - 1) / (kBlock * ipt) <= kScanMaxChunks) return ipt;
  return 64u;
}

uint32_t scan_part_words(uint32_t n) {
  const uint32_t ipt = scan_ipt(n);
  return (n + kBlock * ipt - 1) / (kBlock * ipt) + 1;
}

template <int IPT>
static void scan_ipt_launch(ScanCtx& c, uint32_t* d, uint32_t n, uint32_t nb, hipStream_t st) {
  if (nb > 1) hipLaunchKernelGGL(k_scan_reduce<IPT>, dim3(nb), dim3(kBlock), 0, st, (const uint32_t*)d, n, c.status);
  hipLaunchKernelGGL(k_scan_apply<IPT>, dim3(nb), dim3(kBlock), 0, st, d, n, (const uint32_t*)c.status);
}

void launch_scan(ScanCtx& c, uint32_t* d, uint32_t n, hipStream_t st) {
  if (!n) return;
  if (n <= kScanOneMax) {
    hipLaunchKernelGGL(k_scan_one, dim3(1), dim3(kScanOneThreads), 0, st, d, n);
    return;
  }
  const uint32_t ipt = scan_ipt(n);
  const uint32_t nb = (n + kBlock * ipt - 1) / (kBlock * ipt);
  if (ipt == 4)
    scan_ipt_launch<4>(c, d, n, nb, st);
  else if (ipt == 16)
    scan_ipt_launch<16>(c, d, n, nb, st);
  else
    scan_ipt_launch<64>(c, d, n, nb, st);
}

// ---- tile-bucketed build -------------------------------------------------------------------------
// (1) k_bin_tcount: block b takes the slots of chunk c(b) (kBinChunk consecutive slots); an LDS tile
//     histogram counts the chunk's records per tile, and each non-zero count is added to its tile's
//     total by ONE returning atomic, whose return value is the (tile, chunk) bucket's offset inside
//     the tile (any order of a tile's buckets will do: k_bin_tsort orders by cell), kept in
//     thist[tile * nblk + c]. (2) k_bin_tscatter: every block scans the tile totals in LDS (tile
//     starts; each block stores its share for k_bin_tsort and zeroes its share of the next build's
//     totals), then scatters its chunk's records to their buckets, the rank inside a bucket from an LDS
//     atomic on the bucket cursor. (3) k_bin_tsort: one block per tile counts its records per cell
//     (LDS), scans the 1024 counts, writes the tile's cell starts and places every record (LDS atomic
//     rank within its cell). The cell of a record is recomputed from its binned position with the
//     same cell_key_of as (1).
#ifndef GW_BIN_THREADS
#define GW_BIN_THREADS 1024
#endif
constexpr int kBinThreads = GW_BIN_THREADS;  // 16 waves: one block per CU at 1M slots, latency hidden by width
constexpr int kBinItems = kBinChunk / kBinThreads;

// the chunk a block takes: XCD x (block b runs on XCD b % 8) takes a contiguous run of chunks, so the
// adjacent (tile, chunk) buckets a tile's scatter writes meet in one L2
__device__ __forceinline__ uint32_t bin_chunk_of(uint32_t b, uint32_t nblk) {
  const uint32_t x = b % 8u, per = nblk / 8u, rem = nblk % 8u;
  return x * per + min(x, rem) + b / 8u;
}

// The Spaces' geometry in LDS for the build kernels when there are few Spaces (one load chain less per
// slot: space_of -> geometry becomes space_of -> LDS); more Spaces read it from global memory. The two
// cases are two instantiations of the slot loop (bin_slots), so every access has a known address
// space (a pointer that may be either is a FLAT access, slower for both).
constexpr uint32_t kLdsGeoms = 64;

// keys of slot s's main (k1) and ghost (k0) records, kNoKey for none; geom_of(space) gives a Geom
template <class GeomOf>
__device__ __forceinline__ void bin_keys(const BinArgs& a, GeomOf&& geom_of, uint32_t s, const SlotState& t,
                                         uint32_t& k1, uint32_t& k0) {
  k1 = kNoKey, k0 = kNoKey;
  if (t.p_end || t.p_start) {
    const Geom g = geom_of(a.space_of[s]);
    if (t.p_end) k1 = cell_key_of(g, t.x1, t.z1);
    if (t.p_start) k0 = cell_key_of(g, t.x0, t.z0);
    if (k0 == k1) k0 = kNoKey;
  }
}

template <class Body>
__device__ __forceinline__ void bin_chunk_loop(const BinArgs& a, uint32_t c, Body&& body) {
  const uint32_t s0 = c * a.chunk;
  if (a.chunk == kBinChunk) {  // the common size: unrolled, every item's loads in flight together
#pragma unroll
    for (int k = 0; k < kBinItems; ++k) {
      const uint32_t s = s0 + k * kBinThreads + threadIdx.x;
      if (s >= a.cap) break;
      body(s);
    }
  } else {
    const uint32_t s1 = min(s0 + a.chunk, a.cap);
    for (uint32_t s = s0 + threadIdx.x; s < s1; s += kBinThreads) body(s);
  }
}

// body(s, t, k1, k0) for every slot of chunk c, with the Spaces' geometry from gs (LDS, filled here
// when there are few Spaces; the caller's barrier follows before the first use) or global memory
template <class Body>
__device__ __forceinline__ void bin_slots(const BinArgs& a, uint32_t c, Geom* gs, Body&& body) {
  auto run = [&](auto&& geom_of) {
    bin_chunk_loop(a, c, [&](uint32_t s) {
      const SlotState t = slot_state(a, s);
      uint32_t k1, k0;
      bin_keys(a, geom_of, s, t, k1, k0);
      body(s, t, k1, k0);
    });
  };
  if (a.nspaces <= kLdsGeoms)  // block-uniform
    run([&](uint32_t sp) { return gs[sp]; });
  else
    run([&](uint32_t sp) { return a.geom[sp]; });
}

__device__ __forceinline__ void bin_load_geoms(const BinArgs& a, Geom* gs) {
  if (a.nspaces <= kLdsGeoms)
    for (uint32_t i = threadIdx.x; i < a.nspaces; i += blockDim.x) gs[i] = a.geom[i];
}

__global__ void __launch_bounds__(kBinThreads) k_bin_tcount(BinArgs a) {
  extern __shared__ uint32_t th[];
  __shared__ Geom gs[kLdsGeoms];
  bin_load_geoms(a, gs);
  for (uint32_t i = threadIdx.x; i < a.ntiles; i += kBinThreads) th[i] = 0u;
  __syncthreads();
  const uint32_t c = bin_chunk_of(blockIdx.x, a.nblk);
  bin_slots(a, c, gs, [&](uint32_t, const SlotState&, uint32_t k1, uint32_t k0) {
    if (k1 != kNoKey) atomicAdd(&th[k1 >> kTileCellShift], 1u);
    if (k0 != kNoKey) atomicAdd(&th[k0 >> kTileCellShift], 1u);
  });
  __syncthreads();
  // every returning atomic of the thread in flight together (a loop would wait for each in turn)
  constexpr uint32_t kPer = (kMaxLdsTiles + kBinThreads - 1) / kBinThreads;
  uint32_t cnt[kPer], off[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = threadIdx.x + k * kBinThreads;
    cnt[k] = i < a.ntiles ? th[i] : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k)
    if (cnt[k]) off[k] = atomicAdd(&a.ttot[threadIdx.x + k * kBinThreads], cnt[k]);
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k)
    if (cnt[k]) a.thist[(threadIdx.x + k * kBinThreads) * a.nblk + c] = off[k];
}

__global__ void __launch_bounds__(kBinThreads) k_bin_tscatter(BinArgs a) {
  extern __shared__ uint32_t th[];  // [ntiles]: tile starts, then this chunk's bucket cursors
  __shared__ uint32_t ws[kBinThreads / 64];
  __shared__ Geom gs[kLdsGeoms];
  bin_load_geoms(a, gs);  // (visible after the scan's barriers below)
  constexpr uint32_t kPer = (kMaxLdsTiles + kBinThreads - 1) / kBinThreads;
  const uint32_t n = a.ntiles, i0 = threadIdx.x * kPer;
  const uint32_t c = bin_chunk_of(blockIdx.x, a.nblk);
  // this chunk's bucket offsets inside the tiles (strided: tile threadIdx.x + k kBinThreads) and the tile
  // totals (blocked, for the scan), every load in flight together
  uint32_t h[kPer], v[kPer], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = threadIdx.x + k * kBinThreads;
    h[k] = i < n ? a.thist[i * a.nblk + c] : 0u;  // (stale for tiles this chunk has no record of)
    v[k] = i0 + k < n ? a.ttot[i0 + k] : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) sum += v[k];
  const uint32_t inc = wave_incl_scan(sum);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) ws[w] = inc;
  __syncthreads();
  uint32_t pre = inc - sum, tot = 0;
#pragma unroll
  for (int k = 0; k < kBinThreads / 64; ++k) {
    pre += k < w ? ws[k] : 0u;
    tot += ws[k];
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    if (i0 + k < n) th[i0 + k] = pre;
    pre += v[k];
  }
  __syncthreads();
  const uint32_t gt = blockIdx.x * kBinThreads + threadIdx.x, gn = gridDim.x * kBinThreads;
  for (uint32_t i = gt; i < n; i += gn) a.tstart[i] = th[i];
  if (gt == 0) a.tstart[n] = tot;
  for (uint32_t i = gt; i < kMaxLdsTiles; i += gn) a.ttot_next[i] = 0u;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = threadIdx.x + k * kBinThreads;
    if (i < n) th[i] += h[k];
  }
  __syncthreads();
  bin_slots(a, c, gs, [&](uint32_t s, const SlotState& t, uint32_t k1, uint32_t k0) {
    if (k1 == kNoKey && k0 == kNoKey) return;
    uint32_t j1 = 0, j0 = 0;
    if (k1 != kNoKey) j1 = atomicAdd(&th[k1 >> kTileCellShift], 1u);
    if (k0 != kNoKey) j0 = atomicAdd(&th[k0 >> kTileCellShift], 1u);
    const uint4 rb = make_uint4(__float_as_uint(t.x0), __float_as_uint(t.z0), t.q0, t.q1);
    if (k1 != kNoKey)
      a.trec[j1] = Rec{make_uint4(__float_as_uint(t.x1), __float_as_uint(t.z1), s | (k0 != kNoKey ? REC_HASG : 0u), t.oq),
                       rb};
    if (k0 != kNoKey) a.trec[j0] = Rec{make_uint4(__float_as_uint(t.x0), __float_as_uint(t.z0), s | REC_GHOST, t.oq), rb};
  });
}

// ---- one-pass tile build (the steady state) -------------------------------------------------------
// Bucket layout planned from the PREVIOUS tile build's starts: tile i's records go to
// [plan_start(i), plan_start(i + 1)), which leaves every tile 25% + 15 records of room over its previous
// count. A block can then place its chunk's records as soon as its tile histogram has been added to
// the tile totals (the returning atomic gives the bucket's offset inside the tile): no count pass
// over the slots before the scatter, and no scan between them. A bucket that passes its tile's room
// (a tile that grew by more than that since the previous build: mass Enter, teleports) raises
// CTR_BOVF, and the host re-runs the pass with the counting build (k_bin_tcount / k_bin_tscatter);
// every write stays inside trec whatever the plan. The last block to finish scans the exact tile
// totals into this build's (compact) tile starts, which k_bin_tsort writes the cells at.
__device__ __forceinline__ uint32_t plan_start(const uint32_t* __restrict__ prev, uint32_t i) {
  return (uint32_t)min<uint64_t>((uint64_t)prev[i] * 5u / 4u + 16ull * i, 0xffffffffull);
}

// Chunks of kBinChunk slots (capacities up to 256 kBinChunk) keep each slot's state in registers between
// the histogram and the scatter; larger chunks load it again for the scatter.
constexpr int kFusedItems = kBinItems;

template <bool HOLD>
__global__ void __launch_bounds__(kBinThreads) k_bin_tfused(BinArgs a) {
  extern __shared__ uint32_t th[];  // [ntiles]: this chunk's tile counts, then its bucket cursors
  __shared__ Geom gs[kLdsGeoms];
  __shared__ uint32_t ws[kBinThreads / 64];
  __shared__ uint32_t is_last;
  bin_load_geoms(a, gs);
  const uint32_t n = a.ntiles;
  for (uint32_t i = threadIdx.x; i < n; i += kBinThreads) th[i] = 0u;
  {
    const uint32_t gt = blockIdx.x * kBinThreads + threadIdx.x, gn = gridDim.x * kBinThreads;
    for (uint32_t i = gt; i < kMaxLdsTiles; i += gn) a.ttot_next[i] = 0u;
  }
  __syncthreads();
  const uint32_t c = bin_chunk_of(blockIdx.x, a.nblk);
  // scatter of one slot's records through the chunk's bucket cursors
  auto place = [&](uint32_t s, const SlotState& t, uint32_t k1, uint32_t k0) {
    if (k1 == kNoKey && k0 == kNoKey) return;
    uint32_t j1 = 0, j0 = 0;
    if (k1 != kNoKey) j1 = atomicAdd(&th[k1 >> kTileCellShift], 1u);
    if (k0 != kNoKey) j0 = atomicAdd(&th[k0 >> kTileCellShift], 1u);
    const uint4 rb = make_uint4(__float_as_uint(t.x0), __float_as_uint(t.z0), t.q0, t.q1);
    if (k1 != kNoKey && j1 < a.trec_cap)
      a.trec[j1] = Rec{make_uint4(__float_as_uint(t.x1), __float_as_uint(t.z1), s | (k0 != kNoKey ? REC_HASG : 0u), t.oq),
                       rb};
    if (k0 != kNoKey && j0 < a.trec_cap)
      a.trec[j0] = Rec{make_uint4(__float_as_uint(t.x0), __float_as_uint(t.z0), s | REC_GHOST, t.oq), rb};
  };
  SlotState t[HOLD ? kFusedItems : 1];
  uint32_t k1[HOLD ? kFusedItems : 1], k0[HOLD ? kFusedItems : 1];
  if constexpr (HOLD) {  // a.chunk == kBinChunk
    const uint32_t s0 = c * kBinChunk;
    auto load = [&](auto&& geom_of) {
#pragma unroll
      for (int k = 0; k < kFusedItems; ++k) {
        const uint32_t s = s0 + k * kBinThreads + threadIdx.x;
        k1[k] = k0[k] = kNoKey;
        if (s < a.cap) {
          t[k] = slot_state(a, s);
          bin_keys(a, geom_of, s, t[k], k1[k], k0[k]);
        }
      }
    };
    if (a.nspaces <= kLdsGeoms)  // block-uniform; two code paths, so no access goes through a FLAT pointer
      load([&](uint32_t sp) { return gs[sp]; });
    else
      load([&](uint32_t sp) { return a.geom[sp]; });
#pragma unroll
    for (int k = 0; k < kFusedItems; ++k) {
      if (k1[k] != kNoKey) atomicAdd(&th[k1[k] >> kTileCellShift], 1u);
      if (k0[k] != kNoKey) atomicAdd(&th[k0[k] >> kTileCellShift], 1u);
    }
  } else {
    bin_slots(a, c, gs, [&](uint32_t, const SlotState&, uint32_t q1, uint32_t q0) {
      if (q1 != kNoKey) atomicAdd(&th[q1 >> kTileCellShift], 1u);
      if (q0 != kNoKey) atomicAdd(&th[q0 >> kTileCellShift], 1u);
    });
  }
  __syncthreads();
  constexpr uint32_t kPer = (kMaxLdsTiles + kBinThreads - 1) / kBinThreads;
  {
    uint32_t cnt[kPer], off[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t i = threadIdx.x + k * kBinThreads;
      cnt[k] = i < n ? th[i] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k)
      if (cnt[k]) off[k] = atomicAdd(&a.ttot[threadIdx.x + k * kBinThreads], cnt[k]);
    bool ovf = false;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t i = threadIdx.x + k * kBinThreads;
      if (cnt[k]) {
        const uint64_t pe = (uint64_t)plan_start(a.tprev, i) + off[k] + cnt[k];
        const bool fits = pe <= a.trec_cap;
        ovf |= !fits || pe > plan_start(a.tprev, i + 1);
        th[i] = fits ? (uint32_t)(pe - cnt[k]) : a.trec_cap;  // (past trec: nothing written)
      }
    }
    if (ovf) a.ctr[CTR_BOVF] = 1u;
  }
  __syncthreads();
  if constexpr (HOLD) {
#pragma unroll
    for (int k = 0; k < kFusedItems; ++k) place(c * kBinChunk + k * kBinThreads + threadIdx.x, t[k], k1[k], k0[k]);
  } else {
    bin_slots(a, c, gs, place);
  }
  // The last block to finish scans the tile totals. No fence: a fence here (L2 write-back by every wave,
  // with the scatter's records dirty in it) made the build 3.6x slower. Every block's total atomics
  // have returned before its barrier and its ticket, and the last block reads the totals by atomics
  // too, all at the point device-scope atomics meet from every XCD.
  __syncthreads();
  if (threadIdx.x == 0) is_last = atomicAdd(&a.ctr[CTR_BDONE], 1u) == gridDim.x - 1;
  __syncthreads();
  if (!is_last) return;
  const uint32_t i0 = threadIdx.x * kPer;
  uint32_t v[kPer], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) v[k] = i0 + k < n ? atomicAdd(&a.ttot[i0 + k], 0u) : 0u;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) sum += v[k];
  const uint32_t inc = wave_incl_scan(sum);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) ws[w] = inc;
  __syncthreads();
  uint32_t pre = inc - sum, tot = 0;
#pragma unroll
  for (int k = 0; k < kBinThreads / 64; ++k) {
    pre += k < w ? ws[k] : 0u;
    tot += ws[k];
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    if (i0 + k < n) a.tstart[i0 + k] = pre;
    pre += v[k];
  }
  if (threadIdx.x == 0) a.tstart[n] = tot;
}

// Tiles of up to 4 * kBlock records (all of config 2's) keep their records in registers between the
// count and the placement (one read); larger tiles stream them twice.
// cell index inside its tile, with the Space's geometry fields read as scalars (a local Geom copy
// here gets demoted to scratch/LDS by the compiler)
struct TileMap {
  float x0, z0, inv_c;
  int ncx, ncz;
};

__device__ __forceinline__ TileMap tile_map(const Geom* __restrict__ gp) {
  TileMap m;
  m.x0 = gp->x0;
  m.z0 = gp->z0;
  m.inv_c = gp->inv_c;
  m.ncx = gp->ncx;
  m.ncz = gp->ncz;
  return m;
}

__device__ __forceinline__ uint32_t tile_cell(const TileMap& m, float x, float z) {
  const int cx = cellc(x, m.x0, m.inv_c, m.ncx), cz = cellc(z, m.z0, m.inv_c, m.ncz);
  return (uint32_t)(((cz & (kTile - 1)) << kTileShift) | (cx & (kTile - 1)));
}

// a main record of this pass's op that is not OP_SILENT (k_sweep walks exactly these; cf. is_walker)
__device__ __forceinline__ bool bin_walker(const BinArgs& a, const uint4 ra) {
  const uint32_t r = ra.w - a.base;
  return !(ra.z & REC_GHOST) && r < a.n_ops && !(a.op_kind && (a.op_kind[r] & OP_SILENT));
}

// a record that stands for a slot with an op in this pass, once per slot: its main record, or, for a
// slot that left (absent at the end: seq_end 0), its ghost. k_place compares the sum with the op count:
// two ops on one slot (a device batch's duplicate) leave one acted slot for two ops.
__device__ __forceinline__ uint32_t bin_acted(const BinArgs& a, const uint4 ra, const uint4 rb) {
  return ((ra.w - a.base) < a.n_ops && (!(ra.z & REC_GHOST) || rb.w == 0u)) ? 1u : 0u;
}

__global__ void __launch_bounds__(kBlock) k_bin_tsort(BinArgs a) {
  __shared__ uint32_t cnt[kTileCells];
  __shared__ uint32_t ws[kBlock / 64];
  const uint32_t t = blockIdx.x;
  // (every load of the block's start issued together: the overflow flag, the tile's starts, its plan)
  const uint32_t ovf = a.fused ? a.ctr[CTR_BOVF] : 0u;
  const uint32_t ob = a.tstart[t], oe = a.tstart[t + 1];  // the tile's cells, in rec
  const uint32_t pb = a.fused ? plan_start(a.tprev, t) : ob;
  if (ovf) {  // the plan did not hold: an empty grid (nothing walks), the pass re-runs
    for (int c = threadIdx.x; c < kTileCells; c += kBlock) a.cs[(t << kTileCellShift) + c] = 0u;
    if (threadIdx.x == 0) a.tile_walk[t] = 0u, a.tile_acted[t] = 0u;
    if (t + 1 == a.ntiles && threadIdx.x == 0) a.cs[a.ntiles << kTileCellShift] = 0u;
    return;
  }
  const uint32_t b = pb, e = b + (oe - ob);  // the tile's bucket, in trec
  for (int c = threadIdx.x; c < kTileCells; c += kBlock) cnt[c] = 0u;
  const TileMap g = tile_map(&a.geom[a.tile_space[t]]);
  const bool small = e - b <= 4u * kBlock;
  // small tiles: four records per thread held in registers (loads clamped into [b, e) instead of
  // conditional, so the compiler keeps them in VGPRs)
  const uint32_t j0 = b + threadIdx.x, j1 = j0 + kBlock, j2 = j1 + kBlock, j3 = j2 + kBlock;
  const uint32_t last = e > b ? e - 1 : b;
  const bool on0 = small && j0 < e, on1 = small && j1 < e, on2 = small && j2 < e, on3 = small && j3 < e;
  uint4 a0, b0, a1, b1, a2, b2, a3, b3;
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  if (small && e > b) {
    a0 = a.trec[min(j0, last)].a, b0 = a.trec[min(j0, last)].b;
    a1 = a.trec[min(j1, last)].a, b1 = a.trec[min(j1, last)].b;
    a2 = a.trec[min(j2, last)].a, b2 = a.trec[min(j2, last)].b;
    a3 = a.trec[min(j3, last)].a, b3 = a.trec[min(j3, last)].b;
    c0 = tile_cell(g, __uint_as_float(a0.x), __uint_as_float(a0.y));
    c1 = tile_cell(g, __uint_as_float(a1.x), __uint_as_float(a1.y));
    c2 = tile_cell(g, __uint_as_float(a2.x), __uint_as_float(a2.y));
    c3 = tile_cell(g, __uint_as_float(a3.x), __uint_as_float(a3.y));
  }
  __syncthreads();
  bool walk = false;  // the tile holds a mover whose events are reported (k_sweep skips the others)
  uint32_t acted = 0;  // slots of this pass's ops, each counted once (bin_acted)
  if (small) {
    if (on0) atomicAdd(&cnt[c0], 1u), walk |= bin_walker(a, a0), acted += bin_acted(a, a0, b0);
    if (on1) atomicAdd(&cnt[c1], 1u), walk |= bin_walker(a, a1), acted += bin_acted(a, a1, b1);
    if (on2) atomicAdd(&cnt[c2], 1u), walk |= bin_walker(a, a2), acted += bin_acted(a, a2, b2);
    if (on3) atomicAdd(&cnt[c3], 1u), walk |= bin_walker(a, a3), acted += bin_acted(a, a3, b3);
  } else {
    // crowded tiles (a config-5 hotspot: thousands of records): four records per thread and round, all
    // loads issued before any is used (one round trip per round instead of one per record: these
    // blocks set the kernel's tail)
    // (the small path's registers a0..a3 / b0..b3 are reused: separate arrays spilled)
    for (uint32_t j = b + threadIdx.x; j < e; j += 4u * kBlock) {
      a0 = a.trec[j].a;
      a1 = a.trec[min(j + kBlock, last)].a;
      a2 = a.trec[min(j + 2u * kBlock, last)].a;
      a3 = a.trec[min(j + 3u * kBlock, last)].a;
      auto one = [&](const uint4& ra, uint32_t jj) {
        if (jj >= e) return;
        atomicAdd(&cnt[tile_cell(g, __uint_as_float(ra.x), __uint_as_float(ra.y))], 1u);
        walk |= bin_walker(a, ra);
        // (bin_acted; the end seq is read only for a ghost of this pass's op)
        if ((ra.w - a.base) < a.n_ops) acted += (!(ra.z & REC_GHOST) || a.trec[jj].b.w == 0u) ? 1u : 0u;
      };
      one(a0, j), one(a1, j + kBlock), one(a2, j + 2u * kBlock), one(a3, j + 3u * kBlock);
    }
  }
  const int any_walker = __syncthreads_or(walk);
  if (threadIdx.x == 0) a.tile_walk[t] = any_walker ? 1u : 0u;
  {
    const uint32_t wa = __builtin_amdgcn_readlane(wave_incl_scan(acted), 63);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = wa;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tot = 0;
      for (int k = 0; k < kBlock / 64; ++k) tot += ws[k];
      a.tile_acted[t] = tot;
    }
    __syncthreads();  // ws is reused by the scan below
  }
  // exclusive scan of the 1024 counts (4 per thread, consecutive)
  constexpr int kPer = kTileCells / kBlock;
  static_assert(kPer == 4, "one uint4 of counts per thread");
  const uint4 cv = *reinterpret_cast<const uint4*>(&cnt[threadIdx.x * kPer]);
  const uint32_t sum = cv.x + cv.y + cv.z + cv.w;
  const uint32_t inc = wave_incl_scan(sum);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) ws[w] = inc;
  __syncthreads();
  uint32_t pre = ob + inc - sum;
  for (int k = 0; k < w; ++k) pre += ws[k];
  const uint4 cso = make_uint4(pre, pre + cv.x, pre + cv.x + cv.y, pre + cv.x + cv.y + cv.z);
  *reinterpret_cast<uint4*>(&cnt[threadIdx.x * kPer]) = cso;
  *reinterpret_cast<uint4*>(&a.cs[(t << kTileCellShift) + threadIdx.x * kPer]) = cso;
  if (t + 1 == a.ntiles && threadIdx.x == 0) a.cs[a.ntiles << kTileCellShift] = oe;
  __syncthreads();
  if (small) {
    if (on0) {
      Rec* o = &a.rec[atomicAdd(&cnt[c0], 1u)];
      o->a = a0, o->b = b0;
    }
    if (on1) {
      Rec* o = &a.rec[atomicAdd(&cnt[c1], 1u)];
      o->a = a1, o->b = b1;
    }
    if (on2) {
      Rec* o = &a.rec[atomicAdd(&cnt[c2], 1u)];
      o->a = a2, o->b = b2;
    }
    if (on3) {
      Rec* o = &a.rec[atomicAdd(&cnt[c3], 1u)];
      o->a = a3, o->b = b3;
    }
  } else {
    for (uint32_t j = b + threadIdx.x; j < e; j += 4u * kBlock) {
      a0 = a.trec[j].a, b0 = a.trec[j].b;
      a1 = a.trec[min(j + kBlock, last)].a, b1 = a.trec[min(j + kBlock, last)].b;
      a2 = a.trec[min(j + 2u * kBlock, last)].a, b2 = a.trec[min(j + 2u * kBlock, last)].b;
      a3 = a.trec[min(j + 3u * kBlock, last)].a, b3 = a.trec[min(j + 3u * kBlock, last)].b;
      auto put = [&](const uint4& ra, const uint4& rb, uint32_t jj) {
        if (jj >= e) return;
        Rec* o = &a.rec[atomicAdd(&cnt[tile_cell(g, __uint_as_float(ra.x), __uint_as_float(ra.y))], 1u)];
        o->a = ra, o->b = rb;
      };
      put(a0, b0, j), put(a1, b1, j + kBlock), put(a2, b2, j + 2u * kBlock), put(a3, b3, j + 3u * kBlock);
    }
  }
}

void launch_bin_tiles(const BinArgs& a, hipStream_t st) {
  if (!a.ntiles) return;
  const size_t lds = a.ntiles * sizeof(uint32_t);
  if (a.fused && a.chunk == kBinChunk) {
    hipLaunchKernelGGL(k_bin_tfused<true>, dim3(a.nblk), dim3(kBinThreads), lds, st, a);
  } else if (a.fused) {
    hipLaunchKernelGGL(k_bin_tfused<false>, dim3(a.nblk), dim3(kBinThreads), lds, st, a);
  } else {
    hipLaunchKernelGGL(k_bin_tcount, dim3(a.nblk), dim3(kBinThreads), lds, st, a);
    hipLaunchKernelGGL(k_bin_tscatter, dim3(a.nblk), dim3(kBinThreads), lds, st, a);
  }
  hipLaunchKernelGGL(k_bin_tsort, dim3(a.ntiles), dim3(kBlock), 0, st, a);
}


// ---------------------------------------------------------------------------------------------
// Sweep. One block per tile of the pass's grid (kTile x kTile cells, ~520 entities at config-2
// density); the block loops over the tile's movers, one thread per mover. The block first stages every
// record of the tile plus a halo of `reach` cells into LDS (both record halves), with two cell-start
// tables over the staged region: row-major (the records' own order, so a row interval of cells is one
// contiguous LDS range) and column-major (through an index array, so a column interval of cells is one
// contiguous range too). Each mover then walks its candidates in LDS. Movers whose query boxes leave
// the region (teleports), tiles whose region does not fit, and Leave ops take the global-memory path;
// every path evaluates the same predicates.
//
// Ring walk: for a Moved op, a candidate strictly inside BOTH the old and the new box (shrunk by a
// margin far above float32 rounding) is inside from every perspective before and after, so it
// cannot raise an event. Cells whose every point is that deep (cell index strictly between the
// cells of the shrunken bounds; cellc is monotone, clamping included) are skipped: only the ring of
// border cells is read. For an ordinary move the ring is 1-2 full rows at the top and bottom of the
// union box (row-major segments) and 1-2 columns left and right over the rows between them
// (column-major segments): at most 8 contiguous LDS ranges, walked as ONE flat candidate stream per
// lane, so the lanes of a wave stay converged for max-over-lanes(candidates) iterations instead of a
// per-row loop whose trip count is the max over lanes row by row. Enter and Leave ops, and moves
// whose ring is wider, walk the box row by row.
//
// Events are rare (~0.3 per mover per tick), but atomics on one global counter serialise at the
// memory side (even one per block: 2 x 2,304 per launch cost 10 us), so each block stages its events in
// LDS and copies them into its tile's own region of ev_tmp, storing the count; only a queue overflow
// takes slots of the shared region by atomics. A mover's events are numbered in a register (one thread
// per mover) and its count is stored once, without atomics.
#ifndef GW_SWEEP_BLOCK
#define GW_SWEEP_BLOCK 512
#endif
#ifndef GW_SWEEP_WAVES_PER_EU
#define GW_SWEEP_WAVES_PER_EU 6
#endif
constexpr int kSweepBlock = GW_SWEEP_BLOCK;  // 8 waves: a config-2 tile holds ~520 movers (one round, a few twice)
#ifndef GW_EV_LDS
#define GW_EV_LDS 256
#endif
constexpr int kEvLds = GW_EV_LDS;      // events staged per block before spilling to global atomics
#ifndef GW_CAP
#define GW_CAP 1200
#endif
// GW_CAP: records the small sweep stages at most (config 2: ~1030 +- 32 in a 44 x 44 region)
constexpr int kMaxRows = 48;
// The LDS sweep in two sizes: the small one (three 512-thread blocks per CU, a region of 48 x 48 cells and
// 1,200 records: config 2's tiles) and the big one for Spaces whose region needs more (large D at fine
// cells: config 5's D = 200 / 400 Spaces, ~1,300 / ~2,200 records in 50 x 50 / 66 x 66 cells): one
// 1024-thread block per CU. A Space takes one of them (Geom.reach: small, Geom.pad: big) or neither.
template <int kB, int kCapT, int kCellsT, int kRowsT, int kWpeT>
struct SwCfg {
  static constexpr int kBlk = kB, kCap = kCapT, kCells = kCellsT, kRows = kRowsT, kWpe = kWpeT;
  static constexpr int kCellsPT = (kCells + kB - 1) / kB;  // region cells per thread (staging)
  static constexpr int kIters = (kCap + kB - 1) / kB;      // staged records per thread
  static constexpr bool kBig = kB > 512 || kCapT > 1600;  // the big or the mid sweep (Geom.pad)
  static constexpr bool kMid = kB == 512 && kCapT > 1600;  // the mid sweep (Geom.pad & kPadMid)
};
using SwSmall = SwCfg<kSweepBlock, GW_CAP, kSweepRegCells, kMaxRows, GW_SWEEP_WAVES_PER_EU>;
using SwBig = SwCfg<1024, kSweepBigCap, kSweepBigCells, kSweepBigRows, 4>;
using SwMid = SwCfg<512, kSweepMidCap, kSweepMidCells, kSweepMidRows, 4>;
constexpr float kInner = 3.814697265625e-06f;  // 2^-18: ring margin, relative to |c| + D

template <class C>
struct SweepSmemT {  // dynamic LDS (16-B aligned carve)
  static constexpr uint32_t kEv = kEvLds;  // event queue entries
  uint32_t n, enter, base, item;
  uint32_t nmv, unsorted, pad1, pad2;  // nmv: movers in mv; unsorted: a mover's events left unsorted
  uint32_t ws[16];                 // block-scan scratch
  uint4 ev[kEvLds];             // event queue
  uint16_t lcs[C::kCells + 8];  // row-major: LDS start of each region cell (+ total)
  uint16_t ccs[C::kCells + 8];  // column-major: start in cidx of each region cell (+ total)
  uint16_t cidx[C::kCap];          // column-major order of the staged records (LDS record indices)
  uint16_t mv[C::kCap];            // the tile's movers (LDS record indices)
  uint4 rp[C::kCap];      // staged record, LDS form: {x_start, z_start, x_end, z_end} (float bits)
  uint2 rm[C::kCap];      // {r | G, seq_start | A}: op rank (kNoRank: no op) and the validity mode (lds_record)
  uint32_t rslot[C::kCap];  // slot (read only when an event is emitted); while staging: grid index | kCoreBit
};
using SweepSmem = SweepSmemT<SwSmall>;
// 24 waves per CU (160 KiB of LDS): three 512-thread blocks, or four 384-thread blocks
#ifndef GW_SWEEP_BLOCKS_PER_CU
#define GW_SWEEP_BLOCKS_PER_CU 3
#endif
static_assert(sizeof(SweepSmem) <= 163840 / GW_SWEEP_BLOCKS_PER_CU - 512, "sweep LDS budget per block");
static_assert(sizeof(SweepSmemT<SwBig>) <= 163840 - 512, "big sweep: one block per CU");
static_assert(sizeof(SweepSmemT<SwMid>) <= 163840 / 2 - 512, "mid sweep: two blocks per CU");

size_t sweep_lds_bytes() { return sizeof(SweepSmem); }
uint32_t sweep_block() { return kSweepBlock; }

// Queue one event in the block's LDS queue (one LDS atomic; the file is built without the atomic
// optimizer, so this is a single ds_add_rtn rather than a wave reduction around every call). Enter
// events are counted in a register (`nent`) and added to the block total once per thread.
template <class Q>
__device__ __forceinline__ void emit(const SweepArgs& a, Q& sm, uint32_t rank, uint32_t local, uint32_t mover,
                                     uint32_t other, bool enter, uint32_t& nent) {
#if GW_ABL_NOEMIT  // ablation (timing only): events counted, not queued
  nent += enter ? 1u : 0u;
  return;
#endif
  const uint4 rec = make_uint4(rank, local, mover, other | (enter ? 0x80000000u : 0u));
  const uint32_t li = atomicAdd(&sm.n, 1u);
  if (li < (uint32_t)kEvLds) {
    sm.ev[li] = rec;
  } else {
    // queue full (crowded tiles): one global atomic per wave for the lanes that overflow together,
    // not one per event on the single counter every block shares
    const uint32_t gi = wave_append(&a.ctr[CTR_EVENTS], true);
    if (gi < a.ev_cap) a.ev_tmp[gi] = rec;
    asm volatile("" ::: "memory");  // two stores, not one FLAT store (emit_masks)
  }
  nent += enter ? 1u : 0u;
}

struct Mover {
  uint32_t slot, q, q0, rank;
  bool valid0, valid1;
  float mx0, mz0, mx1, mz1, D;
};

// The cells a mover must read: rows z0..z1 of the union of its old and new query boxes, and in each
// row at most two column intervals — the two boxes' intervals (merged when they touch), or, for a
// move whose boxes overlap, the two ring pieces left and right of the cells deep inside both boxes.
// The walk runs over rows RELATIVE to each lane's own window with a wave-uniform trip count, and
// always visits segment A then segment B (possibly empty), so lanes of a wave that sit in
// different cell rows still follow the same control flow.
struct Walk {
  int z0, z1;
  int ax0, ax1, az0, az1;  // box A (old box, or the union for a ring walk)
  int bx0, bx1, bz0, bz1;  // box B (new box); for a ring walk: the inner rows / columns
  bool ring;
};

__device__ __forceinline__ Walk make_walk(const Mover& m, const Geom& g, const CellBox& A0, const CellBox& A1) {
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

__device__ __forceinline__ Walk make_walk(const Mover& m, const Geom& g) {
  return make_walk(m, g, qbox(g, m.mx0, m.mz0), qbox(g, m.mx1, m.mz1));
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

// segf(r, c0, c1) for each segment (possibly empty), rows relative to the lane's window.
template <class SegF>
__device__ __forceinline__ void walk_cells(const Walk& w, SegF&& segf) {
  const int h = w.z1 - w.z0;
  for (int rel = 0; __any(rel <= h); ++rel) {  // vote over the ACTIVE lanes: wave-uniform trip count
    const int r = w.z0 + rel;
    int a0, a1, b0, b1;
    walk_row(w, r, a0, a1, b0, b1);
    segf(r, a0, a1);
    segf(r, b0, b1);
  }
}

// The pair logic for one candidate record (ra, rb) of the pass's grid, evaluated for mover m.
//   acted earlier in this pass (opq in [base, q)): o is met at its END position (main record);
//     before = in(o_new, m_old), after = in(m_new, o_new).
//   otherwise: o is met at its START position (ghost record, or the main record when the start cell
//     is the same and o was present at the start); before = in(L, F) over the start-of-pass state
//     (o's perspective iff o's start seq > m's), after = in(m_new, o_start).
// "before" is one box test whose centre and test point are selected per candidate (m's old box
// around o, or o's box around m's old position), so both perspectives cost one set of compares.
// Every bound is one binary32 add/sub and every comparison inclusive, exactly as go-aoi's
// `lo <= p && p <= hi` on float32 (a NaN coordinate compares false, as in Go).
struct Judge {
  float lx1, hx1, lz1, hz1;  // m's new box
  float mx0, mz0, mx1, mz1, D;
  float eps;                 // judge_lds: distances within eps of D take the exact test
  bool v0, v1;               // m present before / after its op
  uint32_t base, rank, q, q0;
};

__device__ __forceinline__ Judge make_judge(const Mover& m, uint32_t base) {
  Judge j;
  const float D = m.D;
  j.lx1 = m.mx1 - D, j.hx1 = m.mx1 + D, j.lz1 = m.mz1 - D, j.hz1 = m.mz1 + D;
  j.mx0 = m.mx0, j.mz0 = m.mz0, j.mx1 = m.mx1, j.mz1 = m.mz1, j.D = D;
  // Every bound fl(c +- D) is within 2^-23 (|c| + D) of c +- D and fl(t - c) within 2^-24 |t - c| of
  // t - c; candidates whose box could be decided differently lie within 2D + a cell of the mover, so
  // |c| <= max|m| + 3D. A Chebyshev distance farther than eps from D is therefore decided exactly by
  // the symmetric test (the rest, ~1e-4 of the candidates, by the exact one).
  j.eps = (fmaxf(fmaxf(fabsf(m.mx0), fabsf(m.mz0)), fmaxf(fabsf(m.mx1), fabsf(m.mz1))) + 4.0f * D) *
          4.76837158203125e-07f;  // 2^-21
  j.v0 = m.valid0;
  j.v1 = m.valid1;
  j.base = base, j.rank = m.rank, j.q = m.q, j.q0 = m.q0;
  return j;
}

#ifndef GW_JUDGE_EXACT  // A/B knob: 1 = the exact tests for every candidate
#define GW_JUDGE_EXACT 0
#endif
// 0: no event; otherwise 1 = LEAVE, 2 = ENTER
__device__ __forceinline__ int judge(const Judge& J, const uint4 ra, const uint4 rb) {
  const uint32_t opq = ra.w;
  const bool ae = (opq - J.base) < J.rank;  // acted earlier in this pass
  const bool ghost = ra.z >= REC_GHOST, hasg = (ra.z & REC_HASG) != 0;
  const uint32_t seq0 = rb.z;
  const bool valid = (opq != J.q) & (ghost ? !ae : (ae | (!hasg & (seq0 != 0u))));
  const float px = ae ? __uint_as_float(ra.x) : __uint_as_float(rb.x);
  const float pz = ae ? __uint_as_float(ra.y) : __uint_as_float(rb.y);
  const float D = J.D;
  // Chebyshev distances first; the exact asymmetric tests only near the bound (cf. make_judge)
  const float b = fmaxf(fabsf(px - J.mx0), fabsf(pz - J.mz0));
  const float f = fmaxf(fabsf(px - J.mx1), fabsf(pz - J.mz1));
  bool before = J.v0 & (b <= D);
  bool after = J.v1 & (f <= D);
  if (GW_JUDGE_EXACT || __builtin_expect((int)(fabsf(b - D) <= J.eps) | (int)(fabsf(f - D) <= J.eps), 0)) {
    const bool useo = ae | (seq0 > J.q0);  // o's box (o acted last) or m's old box
    const float cx = useo ? px : J.mx0, cz = useo ? pz : J.mz0;  // box centre
    const float tx = useo ? J.mx0 : px, tz = useo ? J.mz0 : pz;  // point tested
    before = J.v0 & (tx >= cx - D) & (tx <= cx + D) & (tz >= cz - D) & (tz <= cz + D);
    after = J.v1 & (px >= J.lx1) & (px <= J.hx1) & (pz >= J.lz1) & (pz <= J.hz1);
  }
  return (valid & (before != after)) ? (after ? 2 : 1) : 0;
}

// The LDS form of a grid record, precomputing what judge() derives per candidate: position quad
// rp = {x_start, z_start, x_end, z_end} and rm = {r | G, seq_start | A}, r = the record's op rank in
// this pass (kNoRank if its entity has no op; ranks < capacity <= 2^31 - 1, seqs < 2^31). The record
// is a valid candidate for the mover of rank k iff r != k and
//   G (ghost: start cell, met only if not acted earlier):                      k < r
//   A (main with a ghost, or absent at the start: met only if acted earlier):  k > r
//   neither (main alone, present at the start):                                any k
// which is judge()'s `valid` term case by case; positions: start always, end = the binned position
// (for a ghost the binned position is its start, and a ghost is never used "acted earlier").
constexpr uint32_t kNoRank = 0x7FFFFFFFu, kTopBit = 0x80000000u;

__device__ __forceinline__ void lds_record(const uint4 ra, const uint4 rb, uint32_t base, uint32_t n_ops, uint4& rp,
                                           uint2& rm, uint32_t& rslot) {
  const uint32_t q = ra.w - base;
  const uint32_t r = q < n_ops ? q : kNoRank;
  const bool ghost = ra.z >= REC_GHOST, hasg = (ra.z & REC_HASG) != 0;
  const bool after = !ghost && (hasg || rb.z == 0u) && r != kNoRank;
  rp = make_uint4(rb.x, rb.y, ra.x, ra.y);
  rm = make_uint2(r | (ghost ? kTopBit : 0u), rb.z | (after ? kTopBit : 0u));
  rslot = ra.z & REC_SLOT;
}

// judge() on the LDS form. Both box tests first as Chebyshev distances (|dx|, |dz| <= D: symmetric,
// no centre/test-point selection, no bound arithmetic); a distance within J.eps of D, where float
// rounding of the bounds could matter, is re-decided by judge()'s exact asymmetric tests.
__device__ __forceinline__ int judge_lds(const Judge& J, const uint4 rp, const uint2 rm) {
  const uint32_t r = rm.x & ~kTopBit;
  const bool ae = r < J.rank;  // acted earlier in this pass
  const bool valid = (r != J.rank) & (!(rm.x & kTopBit) | !ae) & (!(rm.y & kTopBit) | ae);
  const float px = __uint_as_float(ae ? rp.z : rp.x);
  const float pz = __uint_as_float(ae ? rp.w : rp.y);
  const float D = J.D;
  const float b = fmaxf(fabsf(px - J.mx0), fabsf(pz - J.mz0));
  const float f = fmaxf(fabsf(px - J.mx1), fabsf(pz - J.mz1));
  bool before = J.v0 & (b <= D);
  bool after = J.v1 & (f <= D);
  if (GW_JUDGE_EXACT || __builtin_expect((int)(fabsf(b - D) <= J.eps) | (int)(fabsf(f - D) <= J.eps), 0)) {
    const uint32_t seq0 = rm.y & ~kTopBit;
    const bool useo = ae | (seq0 > J.q0);  // o's box (o acted last) or m's old box
    const float cx = useo ? px : J.mx0, cz = useo ? pz : J.mz0;  // box centre
    const float tx = useo ? J.mx0 : px, tz = useo ? J.mz0 : pz;  // point tested
    before = J.v0 & (tx >= cx - D) & (tx <= cx + D) & (tz >= cz - D) & (tz <= cz + D);
    after = J.v1 & (px >= J.lx1) & (px <= J.hx1) & (pz >= J.lz1) & (pz <= J.hz1);
  }
  return (valid & (before != after)) ? (after ? 2 : 1) : 0;
}

// judge_lds without the exact path, for the candidate loop: true for an event (its kind is re-derived
// at emission, where events are rare), near = a distance within J.eps of D (the caller re-decides those
// candidates with judge_lds).
__device__ __forceinline__ bool judge_fast(const Judge& J, const uint4 rp, const uint2 rm, bool& near) {
  const uint32_t r = rm.x & ~kTopBit;
  const bool ae = r < J.rank;
  const bool valid = (r != J.rank) & (!(rm.x & kTopBit) | !ae) & (!(rm.y & kTopBit) | ae);
  const float px = __uint_as_float(ae ? rp.z : rp.x);
  const float pz = __uint_as_float(ae ? rp.w : rp.y);
  const float b = fmaxf(fabsf(px - J.mx0), fabsf(pz - J.mz0));
  const float f = fmaxf(fabsf(px - J.mx1), fabsf(pz - J.mz1));
  near = fminf(fabsf(b - J.D), fabsf(f - J.D)) <= J.eps;
  return valid & ((J.v0 & (b <= J.D)) != (J.v1 & (f <= J.D)));
}

template <class Q>
__device__ __forceinline__ uint32_t sweep_global(const SweepArgs& a, Q& q, const Mover& m, const Geom& g,
                                                 uint32_t& nent) {
  const Judge J = make_judge(m, a.base);
  uint32_t local = 0;
  walk_cells(make_walk(m, g), [&](int r, int c0, int c1) {
    row_entries_global(g, a.g.cs, r, c0, c1, [&](uint32_t j) {
      const uint4 ra = a.g.rec[j].a;
      const int ev = judge(J, ra, a.g.rec[j].b);
      if (ev) emit(a, q, m.rank, local++, m.slot, ra.z & REC_SLOT, ev == 2, nent);
    });
  });
  return local;
}

struct Region {
  int zr0, zr1, xr0, xr1, ncols, nrows, ncells;
  __device__ __forceinline__ bool holds(const CellBox& b) const {
    return b.z0 >= zr0 && b.z1 <= zr1 && b.x0 >= xr0 && b.x1 <= xr1;
  }
};

// The ring of an ordinary move as at most 8 contiguous LDS ranges in two streams: the row stream
// (row-major: top rows z0, z0+1 and bottom rows z1, z1-1 over the union's columns) and the column
// stream (column-major: columns x0, x0+1, x1, x1-1 over the inner rows bz0..bz1). Returns false when
// the move has no such ring (no inner cells, or a ring side wider than 2 cells): the row walk handles
// it.
struct RingStream {
  uint32_t p1, p2, p3;      // exclusive prefix of the 4 segment lengths (p0 = 0)
  uint32_t d0, d1, d2, d3;  // d0 = start of segment 0; ds = offset(s) - offset(s-1), offset = start - p
  uint32_t total;
};

__device__ __forceinline__ void make_stream(RingStream& S, const uint32_t st[4], const uint32_t en[4]) {
  const uint32_t l0 = en[0] - st[0], l1 = en[1] - st[1], l2 = en[2] - st[2], l3 = en[3] - st[3];
  S.p1 = l0;
  S.p2 = l0 + l1;
  S.p3 = l0 + l1 + l2;
  S.total = S.p3 + l3;
  const uint32_t o0 = st[0], o1 = st[1] - S.p1, o2 = st[2] - S.p2, o3 = st[3] - S.p3;
  S.d0 = o0;
  S.d1 = o1 - o0;
  S.d2 = o2 - o1;
  S.d3 = o3 - o2;
}

// index of candidate k of a stream: k + the offset of the segment holding k (value selects only: an
// indexed pick from a register array would go through scratch)
__device__ __forceinline__ uint32_t stream_at(const RingStream& S, uint32_t k) {
  return k + S.d0 + (k >= S.p1 ? S.d1 : 0u) + (k >= S.p2 ? S.d2 : 0u) + (k >= S.p3 ? S.d3 : 0u);
}

template <class S>
__device__ __forceinline__ bool ring_plan(const Walk& w, const Region& R, const S& sm, RingStream& Rs,
                                          RingStream& Cs) {
  if (!w.ring || w.bz0 > w.bz1 || w.bx0 > w.bx1) return false;
  if (w.bz0 - w.z0 > 2 || w.z1 - w.bz1 > 2 || w.bx0 - w.ax0 > 2 || w.ax1 - w.bx1 > 2) return false;
  uint32_t st[4], en[4];
  const int xa = w.ax0 - R.xr0, xb = w.ax1 - R.xr0 + 1;
  auto row = [&](int slot, int r, bool on) {
    const int b = (r - R.zr0) * R.ncols;
    st[slot] = on ? sm.lcs[b + xa] : 0u;
    en[slot] = on ? sm.lcs[b + xb] : 0u;
  };
  row(0, w.z0, true);
  row(1, w.z1, true);
  row(2, w.z0 + 1, w.z0 + 1 < w.bz0);
  row(3, w.z1 - 1, w.z1 - 1 > w.bz1);
  make_stream(Rs, st, en);
  const int za = w.bz0 - R.zr0, zb = w.bz1 - R.zr0 + 1;
  auto col = [&](int slot, int c, bool on) {
    const int b = (c - R.xr0) * R.nrows;
    st[slot] = on ? sm.ccs[b + za] : 0u;
    en[slot] = on ? sm.ccs[b + zb] : 0u;
  };
  col(0, w.ax0, true);
  col(1, w.ax1, true);
  col(2, w.ax0 + 1, w.ax0 + 1 < w.bx0);
  col(3, w.ax1 - 1, w.ax1 - 1 > w.bx1);
  make_stream(Cs, st, en);
  return true;
}

// Judge candidates b..b+63 of one stream (idx(k) = LDS record index of candidate k): the hot loop
// only records which candidates raise an event (bit k - b of a per-lane mask; the kind is re-derived
// when the event is queued). Two candidates per iteration, both LDS reads in flight, their two bits
// merged before the 64-bit shift, and one (rarely taken) branch per pair for the exact tests. No
// atomic or LDS write sits in the candidate loop itself. (32-candidate chunks with 32-bit masks: the
// register allocator spills 5x more in this kernel, measured slower; the next pair's LDS reads issued
// before the current pair is judged: 94.9 -> 96.3 us at config 2.)
template <class S, class IdxF>
__device__ __forceinline__ unsigned long long judge_chunk(const S& sm, const Judge& J, uint32_t b, uint32_t total,
                                                          IdxF&& idx) {
  const uint32_t n = b < total ? min(total - b, 64u) : 0u;
  unsigned long long hit = 0;
  uint32_t k = 0;
  for (; k + 1 < n; k += 2) {
    const uint32_t j0 = idx(b + k), j1 = idx(b + k + 1);
    const uint4 p0 = sm.rp[j0], p1 = sm.rp[j1];
    const uint2 q0 = sm.rm[j0], q1 = sm.rm[j1];
    bool n0, n1;
    bool h0 = judge_fast(J, p0, q0, n0), h1 = judge_fast(J, p1, q1, n1);
    if (GW_JUDGE_EXACT || __builtin_expect(n0 | n1, 0)) {
      h0 = judge_lds(J, p0, q0) != 0;
      h1 = judge_lds(J, p1, q1) != 0;
    }
    hit |= (unsigned long long)((uint32_t)h0 | ((uint32_t)h1 << 1)) << k;
  }
  if (k < n) {
    const uint32_t j0 = idx(b + k);
    hit |= (unsigned long long)(judge_lds(J, sm.rp[j0], sm.rm[j0]) != 0) << k;
  }
  return hit;
}

// Queue the events marked in two hit masks (hA: candidates ia(bit), hB: ib(bit); each event's kind
// re-derived by judge_lds from the candidate's LDS record) for every
// lane of the wave at once: each lane's event count c, the wave's exclusive prefix and total by one
// ballot per bit of c (no LDS round trip), ONE LDS atomic per wave for the queue range, one global
// atomic per wave when the range runs past the queue; then each lane writes its own events in mask
// order (its `local` numbering). Every lane that reached the call takes part (the masks of a lane
// without events are zero).
// kSortLocal (a mover's whole walk in this one call): each event's `local` index is its rank in the
// canonical order of the mover's events (LEAVE first, then other slot ascending: the key other | ENTER),
// so k_place writes the op's slice already sorted and k_slice_sort has nothing to do: the lane renumbers
// its own queue entries after writing them (no keys held in registers: the walk sits at the kernel's
// VGPR limit). A lane with more than kSortMax events, or with events past the queue, flags the block
// (sm.unsorted) instead.
constexpr uint32_t kSortMax = 8;
// A mover whose events are numbered in walk order: its op's bit in the unsorted bitmask, for k_slice_sort
// (the caller's block or wave then sets CTR_UNS_SOME). Only those ops' slices are sorted.
__device__ __forceinline__ void flag_op(const SweepArgs& a, uint32_t rank) {
  atomicOr(&a.uns[rank >> 5], 1u << (rank & 31u));
}
template <bool kSortLocal, class S, class IdxA, class IdxB>
__device__ __forceinline__ void emit_masks(const SweepArgs& a, S& sm, const Mover& m, const Judge& J,
                                           unsigned long long hA, IdxA&& ia, unsigned long long hB, IdxB&& ib,
                                           uint32_t& local, uint32_t& nent) {
  const uint32_t c = (uint32_t)(__popcll(hA) + __popcll(hB));
#if GW_ABL_NOEMIT  // ablation (timing only): events queued nowhere (enter count not kept)
  local += c;
  return;
#endif
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  uint32_t pre = 0, tot = 0;
  for (int bit = 0; __any((c >> bit) != 0u); ++bit) {  // wave-uniform: the bits of the largest count
    const unsigned long long mb = __ballot((c >> bit) & 1u);
    pre += (uint32_t)__popcll(mb & below) << bit;
    tot += (uint32_t)__popcll(mb) << bit;
  }
  if (tot == 0u) return;  // wave-uniform
  const int leader = __ffsll((long long)__ballot(1)) - 1;
  uint32_t q0 = 0;
  if (lane == leader) q0 = atomicAdd(&sm.n, tot);
  q0 = __builtin_amdgcn_readfirstlane(q0);  // the first active lane is the leader
  const uint32_t qs = max(q0, S::kEv);  // first queue position that spills
  uint32_t g0 = 0;
  if (q0 + tot > qs) {  // wave-uniform
    if (lane == leader) g0 = atomicAdd(&a.ctr[CTR_EVENTS], q0 + tot - qs);
    g0 = __builtin_amdgcn_readfirstlane(g0);
  }
  uint32_t p = q0 + pre;
  const uint32_t l0 = local;
  auto put = [&](unsigned long long& h, auto&& idx) {
    while (h) {
      const int bit = __ffsll((long long)h) - 1;
      const uint32_t j = idx((uint32_t)bit);
      const bool enter = judge_lds(J, sm.rp[j], sm.rm[j]) == 2;
      const uint32_t eb = enter ? 0x80000000u : 0u;
      nent += enter ? 1u : 0u;
      if (p < S::kEv) {
        sm.ev[p] = make_uint4(m.rank, local, m.slot, sm.rslot[j] | eb);
      } else {
        const uint32_t gi = g0 + (p - qs);
        if (gi < a.ev_cap) a.ev_tmp[gi] = make_uint4(m.rank, local, m.slot, sm.rslot[j] | eb);
        // (keeps the two stores apart: merged into one store through a pointer that may be LDS or
        // global, they become a FLAT store, which also counts on lgkmcnt and so holds up every later
        // LDS wait of the wave; the ring walks spent 71% of their time in this emission that way)
        asm volatile("" ::: "memory");
      }
      ++local;
      ++p;
      h &= h - 1ull;
    }
  };
  put(hA, ia);
  put(hB, ib);
  if (kSortLocal && c >= 2u) {
    // renumber the lane's own queue entries by canonical rank (keys other | ENTER are distinct: one
    // event per other entity); entries that spilled past the queue, or too many, are left to k_slice_sort
    const uint32_t p0 = q0 + pre;
    if (c <= kSortMax && p0 + c <= S::kEv) {
      for (uint32_t i = 0; i < c; ++i) {
        const uint32_t ki = sm.ev[p0 + i].w;
        uint32_t rk = 0;
        for (uint32_t j = 0; j < c; ++j) rk += sm.ev[p0 + j].w < ki ? 1u : 0u;
        sm.ev[p0 + i].y = l0 + rk;
      }
    } else {
      flag_op(a, m.rank);
      sm.unsorted = 1u;
    }
  }
}

// Judge candidates 0..total-1 of one stream, 64 at a time, queueing each chunk's events.
template <class S, class IdxF>
__device__ __forceinline__ void judge_stream(const SweepArgs& a, S& sm, const Judge& J, const Mover& m,
                                             uint32_t total, IdxF&& idx, uint32_t& local, uint32_t& nent) {
  for (uint32_t b = 0; __any(b < total); b += 64) {
    const unsigned long long hit = judge_chunk(sm, J, b, total, idx);
    emit_masks<false>(a, sm, m, J, hit, [&](uint32_t k) { return idx(b + k); }, 0ull, [&](uint32_t k) { return k; },
                      local, nent);
  }
}

// Diagnostic build only (GW_STAMPS=1, scripts/variants.py): per-block timestamps of the sweep's
// phases, read back with gwaoi_debug_read_stamps. The product build compiles none of this.
#ifndef GW_STAMPS
#define GW_STAMPS 0
#endif
#if GW_STAMPS
constexpr int kStampWords = 16;
__device__ unsigned long long gw_stamps[kStampWords * 16384];
#define GW_STAMP(k, v)                                                              \
  do {                                                                              \
    if (threadIdx.x == 0 && sm.item < 16384) gw_stamps[sm.item * kStampWords + (k)] = (v); \
  } while (0)
#else
#define GW_STAMP(k, v) \
  do {                 \
  } while (0)
#endif

// Diagnostic build only (GW_STAMPS=1): the ring walk's phases per wave, summed into words 16 * 16382 + k
// of gw_stamps: [0] judge setup + ring plan, [1] row stream, [2] column stream, [3] emission, [4] waves
#if GW_STAMPS
#define GW_SPH(k)                                                                            \
  do {                                                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                              \
    if ((threadIdx.x & 63) == __builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63)))       \
      atomicAdd(&gw_stamps[kStampWords * 16382 + (k)], t_ - st0);                           \
    st0 = t_;                                                                                \
  } while (0)
#else
#define GW_SPH(k) \
  do {            \
  } while (0)
#endif
template <class S>
__device__ __forceinline__ uint32_t sweep_lds(const SweepArgs& a, S& sm, const Mover& m, const Walk& w,
                                              const Region& R, const Geom& g, uint32_t& nent) {
#if GW_STAMPS
  unsigned long long st0 = __builtin_amdgcn_s_memtime();
#endif
  const Judge J = make_judge(m, a.base);
  uint32_t local = 0;
  RingStream Rs, Cs;
  if (ring_plan(w, R, sm, Rs, Cs)) {
    // row stream: LDS record indices directly; column stream: through the column-major index
    auto ri = [&](uint32_t k) { return stream_at(Rs, k); };
    auto ci = [&](uint32_t k) { return (uint32_t)sm.cidx[stream_at(Cs, k)]; };
    if (__all(Rs.total <= 64u && Cs.total <= 64u)) {  // the usual ring: both streams in one chunk, one emission
      GW_SPH(0);
      const unsigned long long hR = judge_chunk(sm, J, 0, Rs.total, ri);
      GW_SPH(1);
      const unsigned long long hC = judge_chunk(sm, J, 0, Cs.total, ci);
      GW_SPH(2);
      emit_masks<true>(a, sm, m, J, hR, ri, hC, ci, local, nent);
      GW_SPH(3);
#if GW_STAMPS
      if ((threadIdx.x & 63) == __builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63)))
        atomicAdd(&gw_stamps[kStampWords * 16382 + 4], 1ull);
#endif
      return local;
    }
    judge_stream(a, sm, J, m, Rs.total, ri, local, nent);
    judge_stream(a, sm, J, m, Cs.total, ci, local, nent);
    if (local > 1u) flag_op(a, m.rank), sm.unsorted = 1u;  // numbered in walk order
    return local;
  }
  walk_cells(w, [&](int r, int c0, int c1) {
    const int b = (r - R.zr0) * R.ncols - R.xr0;
    const uint32_t j = sm.lcs[b + c0];
    const uint32_t e = (c0 <= c1) ? (uint32_t)sm.lcs[b + c1 + 1] : j;
    judge_stream(a, sm, J, m, e - j, [&](uint32_t k) { return j + k; }, local, nent);
  });
  if (local > 1u) flag_op(a, m.rank), sm.unsorted = 1u;
  return local;
}

// exclusive scan of v over a kB-thread block; *total = block sum (LDS scratch `ws`)
template <int kB = kSweepBlock>
__device__ __forceinline__ uint32_t block_excl_scan_big(uint32_t v, uint32_t* ws, uint32_t* total) {
  constexpr int NW = kB / 64;
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


constexpr uint32_t kCoreBit = 0x80000000u;  // staging map: the record lies in the tile itself, not its halo

__device__ __forceinline__ bool is_walker(const SweepArgs& a, const uint4 ra);


// Stage the region of tile (tcx, tcz: the tile's first column / row inside the region). Per cell
// (kCellsPerThread consecutive cells per thread, every cell-start load issued up front): counts, a
// block scan into the row-major LDS cell-start table, and per record its grid index, written into
// rslot by the cell's thread (kCoreBit: the cell is the tile's own). Then the column-major tables,
// then a flat copy: thread per record, grid index from LDS, one 32-B gather each (a thread's gathers
// issued together), LDS form. The tile's reported movers are listed in mv (unordered), or, when
// their boxes leave the region, appended to the dense list (k_sweep_dense). Returns the staged count
// (block-uniform); a count > kCap means "does not fit" and nothing was staged.
template <class C>
__device__ __forceinline__ uint32_t stage(const SweepArgs& a, const Geom& g, const Region& R, int tcx, int tcz,
                                          SweepSmemT<C>& sm) {
  constexpr int kCellsPerThread = C::kCellsPT, kStageIters = C::kIters, kSweepBlock = C::kBlk, kCap = C::kCap;
  uint32_t n[kCellsPerThread], s0[kCellsPerThread];
  uint32_t sum = 0;
  const int c0 = threadIdx.x * kCellsPerThread;
  // this thread's cells are consecutive in row-major order: one division, then a carry (ncols >= kTile)
  const int rr0 = small_div(c0, R.ncols), col0 = c0 - rr0 * R.ncols;
  {
    int rr = rr0, col = col0;
#pragma unroll
    for (int k = 0; k < kCellsPerThread; ++k) {
      n[k] = 0;
      s0[k] = 0;
      if (c0 + k < R.ncells) {
        const uint32_t key = cell_key(g, R.xr0 + col, R.zr0 + rr);
        s0[k] = a.g.cs[key];
        n[k] = a.g.cs[key + 1] - s0[k];
      }
      sum += n[k];
      if (++col == R.ncols) col = 0, ++rr;
    }
  }
  uint32_t total;
  uint32_t pre = block_excl_scan_big<kSweepBlock>(sum, sm.ws, &total);
  GW_STAMP(8, __builtin_amdgcn_s_memrealtime());  // cell starts loaded and scanned
  if (total > (uint32_t)kCap) return total;
  {
    int rr = rr0, col = col0;
#pragma unroll
    for (int k = 0; k < kCellsPerThread; ++k) {
      const int c = c0 + k;
      if (c < R.ncells) {
        sm.lcs[c] = (uint16_t)pre;
        const uint32_t core =
            ((uint32_t)(rr - tcz) < (uint32_t)kTile && (uint32_t)(col - tcx) < (uint32_t)kTile) ? kCoreBit : 0u;
        for (uint32_t q = 0; q < n[k]; ++q) {
          sm.rslot[pre + q] = (s0[k] + q) | core;
          sm.mv[pre + q] = (uint16_t)(rr << 7 | col);  // the record's region cell (read by the column pass)
        }
      }
      pre += n[k];
      if (++col == R.ncols) col = 0, ++rr;
    }
  }
  if (threadIdx.x == 0) {
    sm.lcs[R.ncells] = (uint16_t)total;
    sm.nmv = 0;
  }
  __syncthreads();
  GW_STAMP(9, __builtin_amdgcn_s_memrealtime());  // row-major table and source map written
  uint32_t src[kStageIters];
  Rec r[kStageIters];
  // column-major cell starts (cell counts from the row-major table; cell (rr, cc) is column-major
  // cell cc * nrows + rr), then the column-major index array by one scatter per record: record i of
  // region cell (rr, cc) goes to ccs[cc * nrows + rr] + (i - lcs[rr * ncols + cc])
  {
    uint32_t cn[kCellsPerThread];
    uint32_t sum2 = 0;
    int cc = small_div(c0, R.nrows), rr = c0 - cc * R.nrows;
#pragma unroll
    for (int k = 0; k < kCellsPerThread; ++k) {
      cn[k] = 0;
      if (c0 + k < R.ncells) {
        const int c = rr * R.ncols + cc;
        cn[k] = sm.lcs[c + 1] - sm.lcs[c];
      }
      sum2 += cn[k];
      if (++rr == R.nrows) rr = 0, ++cc;
    }
    uint32_t tot2;
    uint32_t pre2 = block_excl_scan_big<kSweepBlock>(sum2, sm.ws, &tot2);
#pragma unroll
    for (int k = 0; k < kCellsPerThread; ++k) {
      if (c0 + k < R.ncells) sm.ccs[c0 + k] = (uint16_t)pre2;
      pre2 += cn[k];
    }
    if (threadIdx.x == 0) sm.ccs[R.ncells] = (uint16_t)total;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kStageIters; ++k) {
      const uint32_t i = threadIdx.x + k * kSweepBlock;
      if (i < total) {
        const uint32_t cell = sm.mv[i], r = cell >> 7, c = cell & 127u;
        sm.cidx[sm.ccs[c * R.nrows + r] + (i - sm.lcs[r * R.ncols + c])] = (uint16_t)i;
      }
    }
    __syncthreads();  // mv is reused for the mover list below
  }
  GW_STAMP(10, __builtin_amdgcn_s_memrealtime());  // column-major tables
  // (issuing these gathers before the column-major pass instead, to overlap the two: 93.8 -> 94.2 us)
#pragma unroll
  for (int k = 0; k < kStageIters; ++k) {
    const uint32_t i = threadIdx.x + k * kSweepBlock;
    src[k] = i < total ? sm.rslot[i] : 0u;
  }
#pragma unroll
  for (int k = 0; k < kStageIters; ++k) {
    const uint32_t i = threadIdx.x + k * kSweepBlock;
    if (i < total) r[k] = a.g.rec[src[k] & ~kCoreBit];
  }
#pragma unroll
  for (int k = 0; k < kStageIters; ++k) {
    const uint32_t i = threadIdx.x + k * kSweepBlock;
    bool lm = false;
    if (i < total) {
      lds_record(r[k].a, r[k].b, a.base, a.n_ops, sm.rp[i], sm.rm[i], sm.rslot[i]);
      lm = (src[k] & kCoreBit) && is_walker(a, r[k].a);
    }
    const uint32_t li = wave_append(&sm.nmv, lm);  // wave-uniform call: the trip count is a constant
    if (lm) sm.mv[li] = (uint16_t)i;
  }
  GW_STAMP(11, __builtin_amdgcn_s_memrealtime());  // records gathered and staged (thread 0)
  return total;
}

__device__ __forceinline__ Mover mover_of(const uint4 ra, const uint4 rb, uint32_t base, float D) {
  Mover m;
  m.slot = ra.z & REC_SLOT;
  m.q = ra.w;
  m.q0 = rb.z;
  m.rank = m.q - base;
  m.valid0 = m.q0 != 0;
  m.valid1 = true;
  m.mx0 = __uint_as_float(rb.x);
  m.mz0 = __uint_as_float(rb.y);
  m.mx1 = __uint_as_float(ra.x);
  m.mz1 = __uint_as_float(ra.y);
  m.D = D;
  return m;
}

// a mover (main record of an op of this pass) from its slot's state: end = current position,
// start = the start-of-pass state k_apply recorded (mover_of of its grid record, without the gather)
__device__ __forceinline__ Mover slot_mover(const SweepArgs& a, uint32_t s, float D) {
  Mover m;
  m.slot = s;
  m.q = a.opq[s];
  m.q0 = a.old_seq[s];
  m.rank = m.q - a.base;
  m.valid0 = m.q0 != 0;
  m.valid1 = true;
  m.mx0 = a.old_x[s];
  m.mz0 = a.old_z[s];
  m.mx1 = a.pos_x[s];
  m.mz1 = a.pos_z[s];
  m.D = D;
  return m;
}

// a Leave op's mover, from the slot's start-of-pass state recorded by k_apply
__device__ __forceinline__ Mover leaver(const SweepArgs& a, uint32_t i, float D) {
  Mover m;
  m.slot = a.op_slot[i];
  m.q = a.base + i;
  m.q0 = a.old_seq[m.slot];
  m.rank = i;
  m.valid0 = m.q0 != 0;
  m.valid1 = false;
  m.mx0 = a.old_x[m.slot];
  m.mz0 = a.old_z[m.slot];
  m.mx1 = m.mx0;
  m.mz1 = m.mz0;
  m.D = D;
  return m;
}

// XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs (block b runs on XCD
// b % 8), each with its own L2. Give XCD x a contiguous run of tiles, visited in order, so the halo a
// tile shares with its predecessor is still in that XCD's L2. A bijection on [0, n).
constexpr uint32_t kXcds = 8;

__device__ __forceinline__ bool is_mover(const uint4 ra, uint32_t base, uint32_t n_ops) {
  return !(ra.z & REC_GHOST) && (ra.w - base) < n_ops;
}

// a mover whose events are reported (not an OP_SILENT halo copy)
__device__ __forceinline__ bool is_walker(const SweepArgs& a, const uint4 ra) {
  return is_mover(ra, a.base, a.n_ops) && !(a.op_kind && (a.op_kind[ra.w - a.base] & OP_SILENT));
}

// a mover from its staged LDS record (lds_record's form; movers are main records of this pass's ops)
template <class S>
__device__ __forceinline__ Mover lds_mover(const S& sm, uint32_t i, uint32_t base, float D) {
  const uint4 p = sm.rp[i];
  const uint2 q = sm.rm[i];
  Mover m;
  m.slot = sm.rslot[i];
  m.rank = q.x & ~kTopBit;
  m.q = base + m.rank;
  m.q0 = q.y & ~kTopBit;
  m.valid0 = m.q0 != 0;
  m.valid1 = true;
  m.mx0 = __uint_as_float(p.x);
  m.mz0 = __uint_as_float(p.y);
  m.mx1 = __uint_as_float(p.z);
  m.mz1 = __uint_as_float(p.w);
  m.D = D;
  return m;
}

// One work item of k_sweep: a tile. Stage its region (which lists the tile's movers); walk them, one
// thread per mover, consecutive rounds of the block in alternating direction (a tile holds ~520
// movers for 512 threads). The block's LDS event queue is flushed with one global atomic at the end.
template <class C>
__device__ __forceinline__ void sweep_item(const SweepArgs& a, SweepSmemT<C>& sm, const uint32_t item) {
  constexpr int kSweepBlock = C::kBlk, kCap = C::kCap;
  uint32_t nent = 0;  // enter events of this thread's movers
  const uint32_t t = item;
  auto no_events = [&]() {
    if (a.ev_fix && threadIdx.x == 0) a.tile_ev[t] = 0u, a.tile_ent[t] = 0u;
  };
  // block-uniform: a scalar index, so the Space's geometry comes in with scalar loads
  const uint32_t sp = __builtin_amdgcn_readfirstlane(a.g.tile_space[t]);
  const Geom g = uniform_geom(&a.g.geom[sp]);
  // a Space takes the small sweep (reach), the big one (pad) or neither; a tile of the other kernel's
  // Space is left alone entirely (that kernel stores its events and counts)
  const bool mid = (g.pad & kPadMid) != 0;
  if (C::kBig ? !(g.reach == 0 && g.pad > 0 && mid == C::kMid) : (g.reach == 0 && g.pad > 0 && a.use_lds)) return;
  if (a.tile_walk) {
    if (!a.tile_walk[t]) return no_events();  // block-uniform: no reported mover in the tile (k_bin_tsort)
  } else {
    const uint32_t e0 = a.g.cs[t << kTileCellShift], e1 = a.g.cs[(t + 1) << kTileCellShift];
    bool mine = false;
    for (uint32_t j = e0 + threadIdx.x; j < e1 && !mine; j += kSweepBlock) mine = is_walker(a, a.g.rec[j].a);
    if (!__syncthreads_or(mine)) return no_events();  // nothing queued: the caller's barrier follows
  }
  const int reach = C::kBig ? (int)(g.pad & ~kPadMid) : g.reach;
  bool lds = a.use_lds && reach > 0;
  Region R;
  int tcx = 0, tcz = 0;
  if (lds) {
    const uint32_t tl = t - g.tile_base;
    // the division runs on the VALU: pin the (block-uniform) tile coordinates, and with them the region
    // bounds, to scalar registers (in VGPRs they were spilled once per mover)
    const int tz = __builtin_amdgcn_readfirstlane((int)(tl / (uint32_t)g.ntx));
    const int tx = __builtin_amdgcn_readfirstlane((int)(tl - (uint32_t)tz * (uint32_t)g.ntx));
    R.zr0 = max(0, tz * kTile - reach);
    R.zr1 = min(g.ncz - 1, tz * kTile + kTile - 1 + reach);
    R.xr0 = max(0, tx * kTile - reach);
    R.xr1 = min(g.ncx - 1, tx * kTile + kTile - 1 + reach);
    R.ncols = R.xr1 - R.xr0 + 1;
    R.nrows = R.zr1 - R.zr0 + 1;
    R.ncells = R.nrows * R.ncols;
    tcx = tx * kTile - R.xr0;
    tcz = tz * kTile - R.zr0;
    lds = R.ncells <= C::kCells && R.nrows <= C::kRows && R.ncols <= C::kRows;
  }
  if (lds) {
    GW_STAMP(1, __builtin_amdgcn_s_memrealtime());
    const uint32_t nst = stage<C>(a, g, R, tcx, tcz, sm);
    lds = nst <= (uint32_t)kCap;  // block-uniform
    if (a.size_tiles && lds && threadIdx.x == 0) atomicAdd(&a.size_tiles[C::kMid ? 1 : C::kBig ? 2 : 0], 1u);
    __syncthreads();
    GW_STAMP(2, __builtin_amdgcn_s_memrealtime());
    GW_STAMP(5, nst);
    GW_STAMP(6, (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                    ((unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32));
  }
  if (!lds) {
    // region over the LDS budget (or the LDS path off, use_lds 0): every mover of the tile to k_sweep_dense (the tile's entries reserved by ONE atomic per block: an append per wave on
    // the one counter serialised at the memory side, ~48k of them per skew50 launch)
    const uint32_t e0 = a.g.cs[t << kTileCellShift], e1 = a.g.cs[(t + 1) << kTileCellShift];
    uint32_t mine = 0;
    for (uint32_t j = e0 + threadIdx.x; j < e1; j += kSweepBlock) mine += is_walker(a, a.g.rec[j].a) ? 1u : 0u;
    uint32_t tot;
    const uint32_t pre = block_excl_scan_big<kSweepBlock>(mine, sm.ws, &tot);
    if (threadIdx.x == 0) sm.base = tot ? atomicAdd(&a.ctr[CTR_DENSE], tot) : 0u;
    __syncthreads();
    uint32_t di = sm.base + pre;
    for (uint32_t j = e0 + threadIdx.x; j < e1; j += kSweepBlock) {
      const uint4 ra = a.g.rec[j].a;
      if (!is_walker(a, ra)) continue;
      if (di < a.dense_cap) {
        a.dense[di++] = ra.z & REC_SLOT;
        continue;
      }
      ++di;
      const Mover m = mover_of(ra, a.g.rec[j].b, a.base, g.D);
      const uint32_t cnt = sweep_global(a, sm, m, g, nent);
      if (cnt > 1u) flag_op(a, m.rank), sm.unsorted = 1u;  // numbered in walk order
      put_count(a.rank_cnt, m.rank, cnt);
    }
  } else {
    const uint32_t nm = sm.nmv;
    if (a.use_lds != 2) {  // 2: ablation (timing only), staging and ordering without the walk
      // (one wave per mover for a tile's few movers beyond a full round: measured 110 -> 123 us; the
      // planner sizes tiles below one round instead, compute_geometry)
      for (uint32_t r = 0; r * kSweepBlock < nm; ++r) {
        const uint32_t p = r * kSweepBlock + ((r & 1u) ? (uint32_t)(kSweepBlock - 1) - threadIdx.x : threadIdx.x);
        if (p >= nm) continue;
        const Mover m = lds_mover(sm, sm.mv[p], a.base, g.D);
        const CellBox A0 = qbox(g, m.mx0, m.mz0), A1 = qbox(g, m.mx1, m.mz1);
        // movers whose boxes leave the staged region (teleports) go to k_sweep_dense: one wave per
        // mover, candidates 64 at a time
        const bool in_lds = R.holds(A1) && (!m.valid0 || R.holds(A0));
        const uint32_t di = wave_append(&a.ctr[CTR_DENSE], !in_lds);
        if (!in_lds) {
          if (di < a.dense_cap) a.dense[di] = m.slot;
          continue;
        }
        const uint32_t cnt = sweep_lds(a, sm, m, make_walk(m, g, A0, A1), R, g, nent);
        put_count(a.rank_cnt, m.rank, cnt);  // zeroed by k_apply
      }
    }
  }
  // flush the block's events with one global atomic
  if (nent) atomicAdd(&sm.enter, nent);
  GW_STAMP(7, __builtin_amdgcn_s_memrealtime());  // thread 0's walk done
  __syncthreads();
  GW_STAMP(3, __builtin_amdgcn_s_memrealtime());
  if (threadIdx.x == 0 && sm.unsorted) a.ctr[CTR_UNS_SOME] = 1u;
  const uint32_t nq = min(sm.n, (uint32_t)kEvLds);
  if (a.ev_fix) {  // the tile's own region: counts stored, no atomics (two per block cost 10 us at config 2)
    if (threadIdx.x == 0) a.tile_ev[t] = nq, a.tile_ent[t] = sm.enter;
    uint4* dst = a.ev_fix + (size_t)t * kEvLds;
    for (uint32_t i = threadIdx.x; i < nq; i += kSweepBlock) dst[i] = sm.ev[i];
  } else {
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
  GW_STAMP(4, __builtin_amdgcn_s_memrealtime());
}

// 3 blocks x 8 waves per CU (49 KB of LDS each) = 6 waves per SIMD: at most 80 VGPRs. (A VGPR count
// that allows fewer waves per SIMD than the blocks need loses a whole block per CU, whatever the
// occupancy API reports.)
template <class C>
__global__ void __launch_bounds__(C::kBlk) __attribute__((amdgpu_waves_per_eu(C::kWpe)))
k_sweep(SweepArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  SweepSmemT<C>& sm = *reinterpret_cast<SweepSmemT<C>*>(smem_raw);
  // one block per tile of [t0, t0 + n) (all tiles; the big sweep: the range of its Spaces' tiles), tiles
  // mapped XCD-aware by block index
  const uint32_t t0 = C::kMid ? a.mid_t0 : C::kBig ? a.big_t0 : 0u, nt = C::kMid ? a.mid_n : C::kBig ? a.big_n : a.ntiles;
  if (threadIdx.x == 0) {
    const uint32_t xcd = blockIdx.x % kXcds;
    const uint32_t per = nt / kXcds, rem = nt % kXcds;
    const uint32_t b = blockIdx.x;
    sm.item = t0 + xcd * per + min(xcd, rem) + b / kXcds;
    sm.n = 0;
    sm.enter = 0;
    sm.unsorted = 0;
  }
  __syncthreads();
  GW_STAMP(0, __builtin_amdgcn_s_memrealtime());
  sweep_item<C>(a, sm, __builtin_amdgcn_readfirstlane(sm.item));
}

int read_stamps(void* host, size_t bytes) {
#if GW_STAMPS
  if (bytes > sizeof(gw_stamps)) bytes = sizeof(gw_stamps);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(gw_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
#else
  (void)host;
  (void)bytes;
  return -1;
#endif
}

int sweep_occupancy(int* blocks) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, reinterpret_cast<const void*>(&k_sweep<SwSmall>),
                                                      kSweepBlock, sizeof(SweepSmem)) == hipSuccess ? 0 : -3;
}

void sweep_init() {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sweep<SwSmall>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(SweepSmem));
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sweep<SwBig>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(SweepSmemT<SwBig>));
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sweep<SwMid>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(SweepSmemT<SwMid>));
}

// The event queue of the one-thread-per-op global walks (k_sweep_leaves): only the queue in LDS.
struct FlatQ {
  uint32_t n, enter, base, flags;
  uint4 ev[kEvLds];
};

// Leaves of a mixed device batch (or host-staged Leaves): each leaver's old neighbours through the
// global-memory walk, one thread per leaver.
__global__ void __launch_bounds__(kBlock) k_sweep_leaves(SweepArgs a) {
  __shared__ FlatQ q;
  uint32_t nent = 0;
  if (threadIdx.x == 0) {
    q.n = 0;
    q.enter = 0;
    q.flags = 0;
  }
  __syncthreads();
  const uint32_t nl = a.n_leaves_dev ? *a.n_leaves_dev : a.n_leaves;
  for (uint32_t t = blockIdx.x * kBlock + threadIdx.x; t < nl; t += gridDim.x * kBlock) {
    const uint32_t i = a.leave_ops[t];
    if (a.op_kind && (a.op_kind[i] & OP_SILENT)) continue;
    const Geom g = a.g.geom[a.space_of[a.op_slot[i]]];
    const Mover m = leaver(a, i, g.D);
    const uint32_t cnt = sweep_global(a, q, m, g, nent);
    if (cnt > 1u) flag_op(a, i), q.flags = 1u;  // numbered in walk order: k_slice_sort sorts
    put_count(a.rank_cnt, i, cnt);
  }
  if (nent) atomicAdd(&q.enter, nent);
  __syncthreads();
  const uint32_t nq = min(q.n, (uint32_t)kEvLds);
  if (threadIdx.x == 0) {
    q.base = nq ? atomicAdd(&a.ctr[CTR_EVENTS], nq) : 0u;
    if (q.enter) atomicAdd(&a.ctr[CTR_ENTER], q.enter);
    if (q.flags) a.ctr[CTR_UNS_SOME] = 1u;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nq; i += kBlock) {
    const uint32_t gi = q.base + i;
    if (gi < a.ev_cap) a.ev_tmp[gi] = q.ev[i];
  }
}

// ---- Band keys (k_sweep_dense's band walk) -------------------------------------------
// A candidate can only change state for a mover m if its judge position p lies in the symmetric difference
// of m's old and new boxes: p.x within the band between the two left (or the two right) box edges, or p.z
// between the two bottom (top) edges. In a crowd those bands are ~1 unit wide while a cell is 12.5-25, so
// the records of a ring cell are sorted by search key (x, and separately z) and the walk binary-searches
// the window of keys that can hold p in the band, instead of reading the whole cell.
//
// Search key of a record: its binned position, except for a main record without a ghost whose entity
// acted in this pass and was present at the start: judge() then meets it at its start OR its end position
// (which one depends on the mover's rank), both in the binned cell, and the key is their midpoint; hd
// (per Space and axis) bounds |p - key| over all records.
#ifndef GW_BAND_SEARCH_MIN  // cells of fewer records are read whole instead of searched
#define GW_BAND_SEARCH_MIN 4u
#endif
constexpr uint32_t kBandSearchMin = GW_BAND_SEARCH_MIN;
#ifndef GW_BAND_TABLE  // 1: key tables (one lookup per searched cell); 0: the fanout-4 key search (A/B)
#define GW_BAND_TABLE 1
#endif
constexpr uint32_t kBandLdsGeoms = 16;  // Spaces whose geometry the band walk keeps in LDS
// The bucket of key k inside cell c (column for x keys, row for z keys) of a Space with origin o and 1 / side
// inv: 64 equal parts of the cell, clamped (keys of a clamped border cell lie outside it). Monotone in k (every
// step is), which is all the key tables need: the builder (k_band_sort) and the walk use this one function.
__device__ __forceinline__ int band_bucket(float k, float o, float inv, int c) {
  const float f = ((k - o) * inv - (float)c) * (float)kBandBuckets;
  return f >= (float)(kBandBuckets - 1) ? kBandBuckets - 1 : (f > 0.0f ? (int)f : 0);
}
__device__ __forceinline__ void band_key(const uint4 ra, const uint4 rb, float& kx, float& kz, float& hx, float& hz) {
  const float bx = __uint_as_float(ra.x), bz = __uint_as_float(ra.y);
  kx = bx, kz = bz, hx = 0.0f, hz = 0.0f;
  if ((ra.z & (REC_GHOST | REC_HASG)) || rb.z == 0u || (rb.x == ra.x && rb.y == ra.y)) return;
  const float sx = __uint_as_float(rb.x), sz = __uint_as_float(rb.y);
  const float mx = 0.5f * sx + 0.5f * bx, mz = 0.5f * sz + 0.5f * bz;  // (no overflow for finite coordinates)
  kx = mx, kz = mz;
  hx = fmaxf(fabsf(sx - mx), fabsf(bx - mx));
  hz = fmaxf(fabsf(sz - mz), fabsf(bz - mz));
}

// Search keys, the per-Space key spread and each record's rank by x key and by z key inside its cell (ties by
// record index), in ONE kernel: a block takes kBandSortRecs consecutive records, computes the keys of every
// record of the cells they lie in (from the start of its first record's cell to the end of its last one's)
// into LDS, and ranks its own records from there (a hotspot cell's ~50 records read ~50 keys each: from LDS,
// not L1/L2); each record writes itself into the x-sorted records and keys and the z-sorted keys and indices.
// Cells over kBandCellMax records are copied in place, unsorted (the walk reads them whole). The spread is
// reduced per block in LDS and raised in global memory once per block, Space and axis, only when it exceeds
// the current value (one atomic per wave on the same words serialised at the memory side: 1.49 ms per skew50
// pass, r05_b2). A range over the LDS stage (a cell over kBandCellMax records at an edge) ranks from the
// records themselves. (Two kernels before, keys then ranks through a key array: 197 vs 137 us at skew50,
// r05_c28.)
constexpr uint32_t kBandSortRecs = 4 * kBlock, kBandSortStage = 1536;
__device__ __forceinline__ float2 rec_key(const Rec* rec, uint32_t i) {
  const Rec r = rec[i];
  float kx, kz, hx, hz;
  band_key(r.a, r.b, kx, kz, hx, hz);
  return make_float2(kx, kz);
}
__global__ void __launch_bounds__(kBlock) k_band_sort(BandArgs a) {
  // (the staged keys as two float arrays instead of float2 pairs: 174.8 us either way at skew50, r06_a15)
  __shared__ float2 kk[kBandSortStage];
  __shared__ Geom gs[kLdsGeoms];
  __shared__ uint32_t bh[2 * kLdsGeoms];
  __shared__ uint32_t rng[2];
  const bool lgeo = a.nspaces <= kLdsGeoms;
  if (lgeo)
    for (uint32_t i = threadIdx.x; i < a.nspaces; i += kBlock) gs[i] = a.g.geom[i], bh[2 * i] = 0u, bh[2 * i + 1] = 0u;
  __syncthreads();
  const uint32_t n = min(*a.nrec, a.rec_bound);
  const uint32_t j0 = blockIdx.x * kBandSortRecs;
  if (j0 >= n) return;  // block-uniform
  const uint32_t jl = min(j0 + kBandSortRecs, n) - 1u;
  auto cell_of = [&](const uint4 ra, uint32_t& s, uint32_t& e) {
    const uint32_t sp = a.space_of[ra.z & REC_SLOT];
    const float bx = __uint_as_float(ra.x), bz = __uint_as_float(ra.y);
    const uint32_t key = lgeo ? cell_key_of(gs[sp], bx, bz) : cell_key_of(a.g.geom[sp], bx, bz);
    s = a.g.cs[key], e = a.g.cs[key + 1];
    return sp;
  };
  if (threadIdx.x < 2) {
    uint32_t s, e;
    cell_of(a.g.rec[threadIdx.x == 0 ? j0 : jl].a, s, e);
    rng[threadIdx.x] = threadIdx.x == 0 ? s : e;
  }
  __syncthreads();
  const uint32_t lo = rng[0], hi = rng[1];
  const bool staged = hi - lo <= kBandSortStage;  // block-uniform
  if (staged)
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kBlock) kk[i - lo] = rec_key(a.g.rec, i);
  __syncthreads();
#pragma unroll 1
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t j = j0 + k * kBlock + threadIdx.x;
    if (j >= n || j > jl) continue;
    const Rec r = a.g.rec[j];
    uint32_t s, e;
    const uint32_t sp = cell_of(r.a, s, e);
    float kx, kz, hx, hz;
    band_key(r.a, r.b, kx, kz, hx, hz);
    if (hx > 0.0f || hz > 0.0f) {
      uint32_t* w = lgeo ? &bh[2 * sp] : &a.hd[2 * sp];
      if (hx > 0.0f) atomicMax(&w[0], __float_as_uint(hx));
      if (hz > 0.0f) atomicMax(&w[1], __float_as_uint(hz));
    }
    if (e - s > kBandCellMax) {  // copied in place, unsorted (the walk reads the cell whole)
      a.rec_out[j] = r;
      continue;
    }
    uint32_t rx = 0, rz = 0;
    float px = -__builtin_inff(), pz = -__builtin_inff();  // the largest keys ranked below this one
    for (uint32_t i = s; i < e; ++i) {
      const float2 ki = staged ? kk[i - lo] : rec_key(a.g.rec, i);
      const bool bx = ki.x < kx || (ki.x == kx && i < j), bz = ki.y < kz || (ki.y == kz && i < j);
      rx += bx ? 1u : 0u;
      rz += bz ? 1u : 0u;
      px = bx ? fmaxf(px, ki.x) : px;
      pz = bz ? fmaxf(pz, ki.y) : pz;
    }
    a.rec_out[s + rx] = r;
    a.xk[s + rx] = kx;
    a.zk[s + rz] = kz;
    a.zi[s + rz] = s + rx;
    const uint32_t nc = e - s;
    if (a.tab && nc >= kBandSearchMin) {
      // this key's share of its cell's tables: byte b = rank for the buckets b after the predecessor's bucket up
      // to its own (every byte 1..63 of a table is written by exactly one key of the cell; the largest key
      // also writes the buckets above its own with the cell's count)
      const Geom gg = lgeo ? gs[sp] : a.g.geom[sp];
      const int cx = cellc(__uint_as_float(r.a.x), gg.x0, gg.inv_c, gg.ncx);
      const int cz = cellc(__uint_as_float(r.a.y), gg.z0, gg.inv_c, gg.ncz);
      uint8_t* tb = a.tab + (size_t)(s >> 2) * kBandBuckets;
      auto fill = [&](uint8_t* t, uint32_t rk, float k, float pk, float o, int c) {
        const int ib = band_bucket(k, o, gg.inv_c, c), pb = rk ? band_bucket(pk, o, gg.inv_c, c) : 0;
        for (int b = pb + 1; b <= ib; ++b) t[b] = (uint8_t)rk;
        if (rk == nc - 1)
          for (int b = ib + 1; b < kBandBuckets; ++b) t[b] = (uint8_t)nc;
      };
      fill(tb, rx, kx, px, gg.x0, cx);
      fill(tb + a.tab_half, rz, kz, pz, gg.z0, cz);
    }
  }
  if (!lgeo) return;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 2 * a.nspaces; i += kBlock) {
    const uint32_t v = bh[i];
    if (v && v > __hip_atomic_load(&a.hd[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&a.hd[i], v);
  }
}

void launch_band_keys(const BandArgs& b, hipStream_t st) {
  if (!b.rec_bound) return;
  hipLaunchKernelGGL(k_band_sort, dim3((b.rec_bound + kBandSortRecs - 1) / kBandSortRecs), dim3(kBlock), 0, st, b);
}

// The band walk's plan for one mover (wave-uniform): the union box's cells, the cell columns that can
// hold p.x in the left / right band and the rows that can hold p.z in the bottom / top band, and per band
// the window of keys that can belong to such a p. False: no band walk (an Enter, or bands so wide that the
// left and right (bottom and top) columns meet: the ring walk instead).
struct BandPlan {
  int x0, x1, z0, z1;      // union box (cells)
  int cl0, cl1, cr0, cr1;  // x-strip columns: left band, right band
  int rb0, rb1, rt0, rt1;  // z-strip rows: bottom band, top band
  float wl0, wl1, wr0, wr1, wb0, wb1, wt0, wt1;  // key windows
  int zrun;                // z-strips in runs (a sparse edge): see band_item
};

__device__ __forceinline__ bool band_plan(const Mover& m, const Geom& g, const Judge& J, float hdx, float hdz,
                                          BandPlan& P) {
  if (!(m.valid0 && m.valid1)) return false;
  const CellBox A0 = qbox(g, m.mx0, m.mz0), A1 = qbox(g, m.mx1, m.mz1);
  P.x0 = min(A0.x0, A1.x0), P.x1 = max(A0.x1, A1.x1);
  P.z0 = min(A0.z0, A1.z0), P.z1 = max(A0.z1, A1.z1);
  const float D = m.D;
  // the core bands: p outside them on both axes is on the same side of every box edge before and after
  // (by more than judge()'s near margin eps, so the symmetric test decides and no event is possible)
  const float mg = 4.0f * J.eps;
  const float xa = fminf(m.mx0, m.mx1), xb = fmaxf(m.mx0, m.mx1);
  const float za = fminf(m.mz0, m.mz1), zb = fmaxf(m.mz0, m.mz1);
  const float l0 = (xa - D) - mg, l1 = (xb - D) + mg, r0 = (xa + D) - mg, r1 = (xb + D) + mg;
  const float b0 = (za - D) - mg, b1 = (zb - D) + mg, t0 = (za + D) - mg, t1 = (zb + D) + mg;
  // key windows: |p - key| <= hd (widened for the rounding of hd and of the window bounds)
  const float wx = hdx * 1.001f + mg, wz = hdz * 1.001f + mg;
  P.wl0 = l0 - wx, P.wl1 = l1 + wx, P.wr0 = r0 - wx, P.wr1 = r1 + wx;
  P.wb0 = b0 - wz, P.wb1 = b1 + wz, P.wt0 = t0 - wz, P.wt1 = t1 + wz;
  P.cl0 = max(P.x0, cellc(l0, g.x0, g.inv_c, g.ncx)), P.cl1 = min(P.x1, cellc_hi(l1, g.x0, g.inv_c, g.ncx));
  P.cr0 = max(P.x0, cellc(r0, g.x0, g.inv_c, g.ncx)), P.cr1 = min(P.x1, cellc_hi(r1, g.x0, g.inv_c, g.ncx));
  P.rb0 = max(P.z0, cellc(b0, g.z0, g.inv_c, g.ncz)), P.rb1 = min(P.z1, cellc_hi(b1, g.z0, g.inv_c, g.ncz));
  P.rt0 = max(P.z0, cellc(t0, g.z0, g.inv_c, g.ncz)), P.rt1 = min(P.z1, cellc_hi(t1, g.z0, g.inv_c, g.ncz));
  P.zrun = 0;
  return P.cl1 < P.cr0 && P.rb1 < P.rt0;
}

// A plan as the band walk keeps it in LDS (60 B instead of 80: five blocks per CU): the cell bounds as
// 16-bit offsets from the union box's corner (band_plan sends boxes too wide for them to the ring walk).
struct BandPlanL {
  int x0, z0;
  short o[10];  // x1, cl0, cl1, cr0, cr1 (from x0); z1, rb0, rb1, rt0, rt1 (from z0)
  float w[8];   // wl0, wl1, wr0, wr1, wb0, wb1, wt0, wt1
  int zrun;
};
__device__ __forceinline__ void plan_store(BandPlanL& L, const BandPlan& P) {
  L.x0 = P.x0, L.z0 = P.z0;
  L.o[0] = (short)(P.x1 - P.x0), L.o[1] = (short)(P.cl0 - P.x0), L.o[2] = (short)(P.cl1 - P.x0);
  L.o[3] = (short)(P.cr0 - P.x0), L.o[4] = (short)(P.cr1 - P.x0);
  L.o[5] = (short)(P.z1 - P.z0), L.o[6] = (short)(P.rb0 - P.z0), L.o[7] = (short)(P.rb1 - P.z0);
  L.o[8] = (short)(P.rt0 - P.z0), L.o[9] = (short)(P.rt1 - P.z0);
  L.w[0] = P.wl0, L.w[1] = P.wl1, L.w[2] = P.wr0, L.w[3] = P.wr1;
  L.w[4] = P.wb0, L.w[5] = P.wb1, L.w[6] = P.wt0, L.w[7] = P.wt1;
  L.zrun = P.zrun;
}
__device__ __forceinline__ BandPlan plan_load(const BandPlanL& L) {
  BandPlan P;
  P.x0 = L.x0, P.z0 = L.z0;
  P.x1 = P.x0 + L.o[0], P.cl0 = P.x0 + L.o[1], P.cl1 = P.x0 + L.o[2], P.cr0 = P.x0 + L.o[3], P.cr1 = P.x0 + L.o[4];
  P.z1 = P.z0 + L.o[5], P.rb0 = P.z0 + L.o[6], P.rb1 = P.z0 + L.o[7], P.rt0 = P.z0 + L.o[8], P.rt1 = P.z0 + L.o[9];
  P.wl0 = L.w[0], P.wl1 = L.w[1], P.wr0 = L.w[2], P.wr1 = L.w[3];
  P.wb0 = L.w[4], P.wb1 = L.w[5], P.wt0 = L.w[6], P.wt1 = L.w[7];
  P.zrun = L.zrun;
  return P;
}
// every cell bound of the plan within a 16-bit offset of the union box's corner
__device__ __forceinline__ bool plan_fits(const BandPlan& P) {
  auto ok = [](int v) { return v >= -32000 && v <= 32000; };
  return ok(P.x1 - P.x0) && ok(P.cl0 - P.x0) && ok(P.cl1 - P.x0) && ok(P.cr0 - P.x0) && ok(P.cr1 - P.x0) &&
         ok(P.z1 - P.z0) && ok(P.rb0 - P.z0) && ok(P.rb1 - P.z0) && ok(P.rt0 - P.z0) && ok(P.rt1 - P.z0);
}

// a wave-uniform plan pinned to scalar registers
__device__ __forceinline__ void band_pin(BandPlan& P) {
  auto u = [](int& v) { v = __builtin_amdgcn_readfirstlane(v); };
  auto uf = [](float& v) { v = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
  u(P.x0), u(P.x1), u(P.z0), u(P.z1), u(P.cl0), u(P.cl1), u(P.cr0), u(P.cr1), u(P.rb0), u(P.rb1), u(P.rt0), u(P.rt1);
  uf(P.wl0), uf(P.wl1), uf(P.wr0), uf(P.wr1), uf(P.wb0), uf(P.wb1), uf(P.wt0), uf(P.wt1);
}

// Dense movers: one WAVE per mover (k_sweep lists them: boxes beyond the tile's LDS region, tiles whose
// region does not fit, Spaces whose region cannot). The walk is the same row walk as sweep_global, but
// lane-parallel: each lane takes one part (a row segment inside one tile: ONE contiguous record range),
// the parts' ranges come in with one round trip for up to 64 parts, and the concatenated candidate
// stream is judged 128 at a time (each lane finds its range by a binary search over the lanes'
// inclusive prefix), so every 128 candidates cost one coalesced memory round trip whatever the number
// of cells they come from. A mover's events are numbered by a ballot prefix on top of the
// wave-uniform running count and written into event slots the wave reserves kEvChunk at a time.
// (Measured against this, on skew50 / skew: the candidates listed in LDS by the wave instead of the
// binary search, 6.53 -> 6.95 / 3.06 -> 3.30 ms; four candidates per lane per round at 5 waves/SIMD,
// slower again. The walk is bound by its candidate records, not by locating them.)
constexpr int kDenseBlock = 256;
#ifndef GW_DENSE_WPE
#define GW_DENSE_WPE 6
#endif
#ifndef GW_EV_CHUNK
#define GW_EV_CHUNK 128
#endif
constexpr uint32_t kEvChunk = GW_EV_CHUNK;  // event slots a wave reserves at a time (one returning atomic
                                      // on the shared counter each: ~11 ns apiece when serialised)

// Diagnostic build only (GW_STAMPS=1): per-wave cycle accounting of the dense walk's phases, summed over
// the waves into the last 16 words of gw_stamps (bench.py --stamps): [0] batch loads, [1] mover setup,
// [2] part enumeration, [3] range loads, [4] candidate rounds, [8] movers, [9] flushes, [10] rounds.
#if GW_STAMPS
#define GW_DPH(k)                                           \
  do {                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    dph[k] += t_ - dt0;                                     \
    dt0 = t_;                                               \
  } while (0)
#define GW_DCNT(k) (++dph[k])
#else
#define GW_DPH(k) \
  do {            \
  } while (0)
#define GW_DCNT(k) \
  do {             \
  } while (0)
#endif

// kRing: the list of the movers k_sweep_band handed over (dense2), else k_sweep's dense list
template <bool kRing>
__global__ void __launch_bounds__(kDenseBlock) __attribute__((amdgpu_waves_per_eu(GW_DENSE_WPE)))
k_sweep_dense(SweepArgs a) {
  const int lane = threadIdx.x & 63;
  // XCD-aware wave numbering (block b runs on XCD b % 8; the grid is a multiple of 8 blocks): the waves
  // of one XCD take consecutive list entries, so the movers walked together on an XCD are neighbours
  // and share that XCD's L2 (skew50: dense walk 6.84 -> 6.57 ms with the batch below)
  const uint32_t wv = threadIdx.x >> 6, nwaves = gridDim.x * (kDenseBlock / 64);
  const uint32_t wave = ((blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u) * (kDenseBlock / 64) + wv;
  // (kRing: dense2 runs parallel to the dense list, the band walk's movers marked kNoKey, so the ring walk
  // visits the rest in the same grid order: handed over compacted, its waves lost their L2 locality)
  const uint32_t* list = kRing ? a.dense2 : a.dense;
  // (kRing: nothing handed over, the usual case now that every mover with a band plan takes it: the list
  // is not scanned)
  const uint32_t nd = kRing && a.ctr[CTR_RING_MV] == 0u ? 0u : min(a.ctr[CTR_DENSE], a.dense_cap);
  const unsigned long long below = (1ull << lane) - 1ull;
  uint32_t nent = 0;
  uint32_t cur = 0, left = 0;  // the wave's current chunk of event slots (wave-uniform)
  __shared__ uint4 mb[kDenseBlock / 64][64][2];  // the wave's batch of movers: {slot, Space, opq, seq0}, {x0, z0, x1, z1}
  __shared__ uint32_t orow[kDenseBlock / 64][128];  // stream_owners' marks
#if GW_STAMPS
  unsigned long long dph[16] = {}, dt0 = __builtin_amdgcn_s_memtime();
#endif
  // The wave walks list entries wave, wave + nwaves, wave + 2 nwaves, ...: at any time the waves of the
  // grid walk one window of nwaves consecutive entries (a few neighbouring tiles' movers: their ring
  // cells stay in L2). The slot state of the wave's next 64 entries is loaded in one go (lane i: entry
  // wave + (b0 + i) nwaves), so a batch costs one dependent chain of loads instead of one per mover.
  for (uint32_t b0 = 0; wave + b0 * nwaves < nd; b0 += 64u) {
    const uint32_t di = wave + (b0 + (uint32_t)lane) * nwaves;
    const uint32_t ls = di < nd ? list[di] : kNoKey;
    if (ls != kNoKey) {
      mb[wv][lane][0] = make_uint4(ls, a.space_of[ls], a.opq[ls], a.old_seq[ls]);
      mb[wv][lane][1] = make_uint4(__float_as_uint(a.old_x[ls]), __float_as_uint(a.old_z[ls]),
                                   __float_as_uint(a.pos_x[ls]), __float_as_uint(a.pos_z[ls]));
    }
    unsigned long long todo = __ballot(ls != kNoKey);  // the batch's movers
    __builtin_amdgcn_wave_barrier();  // the wave's LDS ops stay in program order
    GW_DPH(0);
    uint32_t gsp = ~0u;
    Geom g;
    while (todo) {
      const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane(__ffsll((long long)todo) - 1);
      todo &= todo - 1ull;
      // the mover's state from the wave's batch (uniform LDS address: one broadcast read per half)
      const uint4 u0 = mb[wv][k][0], u1 = mb[wv][k][1];
      const uint32_t sp = (uint32_t)__builtin_amdgcn_readfirstlane((int)u0.y);
      if (sp != gsp) {  // wave-uniform: neighbouring list entries are mostly one Space
        g = uniform_geom(&a.g.geom[sp]);
        gsp = sp;
      }
      Mover m;
      m.slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)u0.x);
      m.q = (uint32_t)__builtin_amdgcn_readfirstlane((int)u0.z);
      m.q0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)u0.w);
      m.rank = m.q - a.base;
      m.valid0 = m.q0 != 0;
      m.valid1 = true;
      m.mx0 = __int_as_float(__builtin_amdgcn_readfirstlane((int)u1.x));
      m.mz0 = __int_as_float(__builtin_amdgcn_readfirstlane((int)u1.y));
      m.mx1 = __int_as_float(__builtin_amdgcn_readfirstlane((int)u1.z));
      m.mz1 = __int_as_float(__builtin_amdgcn_readfirstlane((int)u1.w));
      m.D = g.D;
      const Judge J = make_judge(m, a.base);
      uint32_t local = 0;  // wave-uniform
      GW_DCNT(8);
      GW_DPH(1);
      // one sub-round's events: numbered by a ballot prefix on top of the wave-uniform running count,
      // slots from the wave's current chunk of ev_tmp (a fresh one reserved when it fills up)
      auto emit_round = [&](int ev, uint32_t other) {
        const unsigned long long em = __ballot(ev != 0);
        if (!em) return;
        const uint32_t cnt = (uint32_t)__popcll(em);
        const uint32_t pre = (uint32_t)__popcll(em & below);
        uint32_t gi = cur + pre;
        if (cnt > left) {  // this chunk fills up: the rest goes to a fresh one
          uint32_t nbk = 0;
          if (lane == 0) nbk = atomicAdd(&a.ctr[CTR_EVENTS], kEvChunk);
          nbk = __shfl(nbk, 0, 64);
          if (pre >= left) gi = nbk + (pre - left);
          cur = nbk + (cnt - left);
          left = kEvChunk - (cnt - left);
        } else {
          cur += cnt;
          left -= cnt;
        }
        if (ev) {
          if (gi < a.ev_cap) a.ev_tmp[gi] = make_uint4(m.rank, local + pre, m.slot, other | (ev == 2 ? 0x80000000u : 0u));
          nent += ev == 2 ? 1u : 0u;
        }
        local += cnt;
      };
      const Walk w = make_walk(m, g);
      // the parts of up to 64 lanes: ranges in one round trip, then the candidates 128 at a time (two
      // loads in flight per lane); candidate k belongs to the first part whose inclusive prefix exceeds
      // k (a binary search over the lanes' prefixes)
      auto flush = [&](uint32_t pk, uint32_t pe, int np) {
        uint32_t rs = 0, rl = 0;
        if (lane < np) {
          rs = a.g.cs[pk];
          rl = a.g.cs[pe] - rs;
        }
        const uint32_t incl = wave_incl_scan(rl);
        const uint32_t excl = incl - rl;
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        GW_DCNT(9);
        GW_DPH(3);
        auto locate = [&](uint32_t k, int lo) -> uint32_t {  // record index of candidate k (owner lane lo)
          return __shfl(rs, lo, 64) + (k - __shfl(excl, lo, 64));
        };
        for (uint32_t b = 0; b < total; b += 128) {
          const uint32_t kA = b + lane, kB = b + 64 + lane;
          int oA, oB;
          stream_owners(orow[wv], excl, rl, b, oA, oB);
          const uint32_t jA = locate(kA, oA);
          const bool hasB = b + 64 < total;  // wave-uniform
          const uint32_t jB = hasB ? locate(kB, oB) : 0u;
          uint4 aA = make_uint4(0, 0, 0, 0), bA = aA, aB = aA, bB = aA;
          if (kA < total) aA = a.g.rec[jA].a, bA = a.g.rec[jA].b;
          if (hasB && kB < total) aB = a.g.rec[jB].a, bB = a.g.rec[jB].b;
          emit_round(kA < total ? judge(J, aA, bA) : 0, aA.z & REC_SLOT);
          if (hasB) emit_round(kB < total ? judge(J, aB, bB) : 0, aB.z & REC_SLOT);
          GW_DCNT(10);
        }
        GW_DPH(4);
      };
      // the walk, lane-parallel: lane = (row, segment) of 32 rows at a time; each segment splits into
      // one part per tile it touches; part p is taken by lane p % 64 (binary search over the prefix)
      const int h = w.z1 - w.z0 + 1;
      for (int rb = 0; rb < h; rb += 32) {
        const int r = w.z0 + rb + (lane >> 1);
        int a0, a1, b0r, b1r;
        walk_row(w, rb + (lane >> 1) < h ? r : w.z1 + 1, a0, a1, b0r, b1r);
        const int c0 = (lane & 1) ? b0r : a0, c1 = (lane & 1) ? b1r : a1;
        const uint32_t nparts = c0 <= c1 ? (uint32_t)((c1 >> kTileShift) - (c0 >> kTileShift) + 1) : 0u;
        const uint32_t pincl = wave_incl_scan(nparts);
        const uint32_t T = __builtin_amdgcn_readlane(pincl, 63);
        for (uint32_t pb = 0; pb < T; pb += 64) {
          const uint32_t p = pb + lane;
          int lo = 0, hi = 63;
#pragma unroll
          for (int st = 0; st < 6; ++st) {
            const int mid = (lo + hi) >> 1;
            if (__shfl(pincl, mid, 64) > p) hi = mid;
            else lo = mid + 1;
          }
          const int q = (int)(p - (__shfl(pincl, lo, 64) - __shfl(nparts, lo, 64)));
          const int sc0 = __shfl(c0, lo, 64), sc1 = __shfl(c1, lo, 64), sr = __shfl(r, lo, 64);
          const int tx = (sc0 >> kTileShift) + q;
          const int plo = max(sc0, tx << kTileShift), phi = min(sc1, (tx << kTileShift) + kTile - 1);
          const uint32_t pk = g.base + ((uint32_t)((sr >> kTileShift) * g.ntx) << kTileCellShift) +
                              (uint32_t)((sr & (kTile - 1)) << kTileShift) + ((uint32_t)tx << kTileCellShift) +
                              (uint32_t)(plo & (kTile - 1));
          GW_DPH(2);
          flush(pk, pk + (uint32_t)(phi - plo) + 1, (int)min(64u, T - pb));
        }
      }
      if (lane == 0) put_count(a.rank_cnt, m.rank, local);
    }
    __builtin_amdgcn_wave_barrier();  // every read of the batch before the next batch is written
  }
  for (uint32_t i = lane; i < left; i += 64)
    if (cur + i < a.ev_cap) a.ev_tmp[cur + i] = make_uint4(kEvHole, 0u, 0u, 0u);
  if (lane == 0 && left) atomicAdd(&a.ctr[CTR_HOLES], left);
  const uint32_t went = __shfl(wave_incl_scan(nent), 63, 64);  // one add per wave, not per lane
  if (lane == 0 && went) atomicAdd(&a.ctr[CTR_ENTER], went);
  // (a dense mover's events are numbered in walk order: the slices are sorted whenever the list is not
  // empty. Flagging only the movers with two or more events, a per-mover flag in the walk loop, made
  // this kernel 66% slower on strips_skew: 484 -> 803 us, r04_c9)
  if (blockIdx.x == 0 && threadIdx.x == 0 && nd) a.ctr[CTR_UNSORTED] = 1u;
#if GW_STAMPS
  if (lane == 0)
    for (int k = 0; k < 16; ++k) atomicAdd(&gw_stamps[kStampWords * 16383 + k], dph[k]);
#endif
}

// ---- The band walk --------------------------------------------------------------------
// k_sweep_dense's list walked by the band walk. For an ordinary move only the cells that can hold a judge
// position in the symmetric difference of the two boxes are read (the x-strip columns of the left / right
// band over the union's rows, the z-strip rows of the bottom / top band over its columns), and in each
// such cell only the window of search keys that can (a fanout-4 search per cell: k_band_sort
// sorted the cells' records). A hotspot cell of ~50 records yields ~3 candidates instead of 50.
//
// Every global round trip costs ~3.5k cycles under this load (GW_STAMPS phases, r05_b6), so the walk is
// flat over the wave's batch of 64 movers: the batch's cells form ONE item stream (2 per lane per round:
// cell starts, then two search levels, all lanes' loads in flight together), whose candidates form one
// candidate stream (2 per lane per round), whatever mover they belong to. A mover's plan is recomputed
// from the batch's LDS copy wherever it is needed (VALU is idle here); its judge data, dedupe windows
// and event count live in LDS. (One mover per wave at a time, as k_sweep_dense: ~6 trips per mover,
// no faster than the ring walk, r05_b5.) The movers without a band plan (Enters, moves whose bands meet)
// or for which the cost model prefers the ring walk are left to k_sweep_dense<true> (dense2).
#ifndef GW_BAND_WPE  // 4 waves per SIMD: 118 VGPRs (two cells and two candidates per lane in flight)
#define GW_BAND_WPE 5
#endif
#ifndef GW_BAND_FAN
#define GW_BAND_FAN 4
#endif
[[maybe_unused]] constexpr uint32_t kBandFan = GW_BAND_FAN;  // probes per search level (cells of up to kBandFan keys: one level)
#ifndef GW_BAND_RUN
#define GW_BAND_RUN 4.0f
#endif
constexpr float kBandRun = GW_BAND_RUN;  // z-strips in runs when the bottom / top edge cells hold fewer records

// z-strip runs (BandPlan.zrun, a mover whose bottom / top edges lie in a sparse part of the world): a z-strip
// row is one item per cell of the x-strip columns (searched, or read whole, with the corner-cell dedupe as
// usual) plus one item per tile-row piece of the columns outside them, read whole: a piece's cells are
// consecutive cell keys, so its records are ONE range (two cell-start loads for up to 32 cells, where the
// per-cell items cost a decode, two loads and a search each, for a handful of records)
__device__ __forceinline__ int seg_pieces(int a, int b) { return a <= b ? (b >> kTileShift) - (a >> kTileShift) + 1 : 0; }
__device__ __forceinline__ void run_cols(const BandPlan& P, int& xl0, int& xl1, int& xr0, int& xr1) {
  // the x-strip column sets, an empty one moved to the end of the row it lies at
  const bool el = P.cl1 < P.cl0, er = P.cr1 < P.cr0;
  xl0 = el ? P.x0 : P.cl0, xl1 = el ? P.x0 - 1 : P.cl1;
  xr0 = er ? P.x1 + 1 : P.cr0, xr1 = er ? P.x1 : P.cr1;
}
__device__ __forceinline__ int run_row_items(const BandPlan& P) {
  int xl0, xl1, xr0, xr1;
  run_cols(P, xl0, xl1, xr0, xr1);
  return (xl1 - xl0 + 1) + (xr1 - xr0 + 1) + seg_pieces(P.x0, xl0 - 1) + seg_pieces(xl1 + 1, xr0 - 1) +
         seg_pieces(xr1 + 1, P.x1);
}
// the cell of item li of a band plan: x-strip cells (columns of the left / right band over the union's rows,
// keys by x), then z-strip cells (rows of the bottom / top band over the union's columns, keys by z; dd marks
// a column that is also in an x-strip, whose records with their x key in that strip's window were judged
// there); in run mode a z-strip piece [c, c + span] of one tile row is kind 4 (read whole)
__device__ __forceinline__ void band_item(const BandPlan& P, uint32_t li, int& c, int& r, float& w0, float& w1,
                                          int& kind, int& dd, int& span) {
  const int H = P.z1 - P.z0 + 1, W = P.x1 - P.x0 + 1;
  const int nxl = max(0, P.cl1 - P.cl0 + 1), nzb = max(0, P.rb1 - P.rb0 + 1);
  const uint32_t NX = (uint32_t)((nxl + max(0, P.cr1 - P.cr0 + 1)) * H);
  span = 0;
  if (li < NX) {
    const int ci = small_div((int)li, H);
    r = P.z0 + (int)li - ci * H;
    const bool left = ci < nxl;
    c = left ? P.cl0 + ci : P.cr0 + ci - nxl;
    w0 = left ? P.wl0 : P.wr0;
    w1 = left ? P.wl1 : P.wr1;
    kind = 0;
    dd = 0;
    return;
  }
  const int i2 = (int)(li - NX);
  const int Wz = P.zrun ? run_row_items(P) : W;
  const int ri = small_div(i2, Wz), k = i2 - ri * Wz;
  const bool bot = ri < nzb;
  r = bot ? P.rb0 + ri : P.rt0 + ri - nzb;
  w0 = bot ? P.wb0 : P.wt0;
  w1 = bot ? P.wb1 : P.wt1;
  kind = 1;
  if (!P.zrun) {
    c = P.x0 + k;
  } else {
    int xl0, xl1, xr0, xr1;
    run_cols(P, xl0, xl1, xr0, xr1);
    const int kl = xl1 - xl0 + 1, kc = kl + (xr1 - xr0 + 1);
    if (k < kc) {
      c = k < kl ? xl0 + k : xr0 + (k - kl);
    } else {  // a piece of the segments left of, between and right of the x-strip columns
      int j = k - kc, a = P.x0, b = xl0 - 1;
      const int p1 = seg_pieces(a, b);
      if (j >= p1) {
        j -= p1, a = xl1 + 1, b = xr0 - 1;
        const int p2 = seg_pieces(a, b);
        if (j >= p2) j -= p2, a = xr1 + 1, b = P.x1;
      }
      c = j == 0 ? a : ((a >> kTileShift) + j) << kTileShift;
      span = min(b, (((a >> kTileShift) + j + 1) << kTileShift) - 1) - c;
      kind = 4;
      dd = 0;
      return;
    }
  }
  dd = (c >= P.cl0 && c <= P.cl1 ? 1 : 0) | (c >= P.cr0 && c <= P.cr1 ? 2 : 0);
}
__device__ __forceinline__ uint32_t band_items(const BandPlan& P) {
  const int H = P.z1 - P.z0 + 1, W = P.x1 - P.x0 + 1;
  return (uint32_t)((max(0, P.cl1 - P.cl0 + 1) + max(0, P.cr1 - P.cr0 + 1)) * H +
                    (max(0, P.rb1 - P.rb0 + 1) + max(0, P.rt1 - P.rt0 + 1)) * (P.zrun ? run_row_items(P) : W));
}

// the lane whose inclusive prefix `incl` is the first above k (every lane of the wave takes part)
__device__ __forceinline__ int wave_owner(uint32_t incl, uint32_t k) {
  int lo = 0, hi = 63;
#pragma unroll
  for (int st = 0; st < 6; ++st) {
    const int mid = (lo + hi) >> 1;
    if ((uint32_t)__shfl((int)incl, mid, 64) > k) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// kBuf: the hot loads (cell starts, search keys, z order, candidate records) through buffer descriptors
// (32-bit offsets: the walk is VALU-issue bound, and a flat load's 64-bit address costs two or three VALU
// instructions); the launcher picks it when every array is below 2 GiB
template <bool kBuf>
__global__ void __launch_bounds__(kDenseBlock) __attribute__((amdgpu_waves_per_eu(GW_BAND_WPE)))
k_sweep_band(SweepArgs a) {
  // x keys and z keys are one allocation (zk = xk + zoff)
  const uint32_t zoff = (uint32_t)(a.band_zk - a.band_xk);
  const auto r_cs = __builtin_amdgcn_make_buffer_rsrc((void*)a.g.cs, 0, (int)((a.ncells + 1u) * 4u), 0x00020000);
  const auto r_key = __builtin_amdgcn_make_buffer_rsrc((void*)a.band_xk, 0, (int)(2u * zoff * 4u), 0x00020000);
  const auto r_zi = __builtin_amdgcn_make_buffer_rsrc((void*)a.band_zi, 0, (int)(zoff * 4u), 0x00020000);
  const auto r_rec = __builtin_amdgcn_make_buffer_rsrc((void*)a.g.rec, 0, (int)(a.n_rec * 32u), 0x00020000);
  auto ld_cs = [&](uint32_t k) -> uint32_t {
    if constexpr (kBuf) return __builtin_amdgcn_raw_buffer_load_b32(r_cs, k << 2, 0, 0);
    else return a.g.cs[k];
  };
  auto ld_key = [&](int kind, uint32_t i) -> float {  // kind 1: z key
    if constexpr (kBuf) return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r_key, ((kind == 1 ? zoff : 0u) + i) << 2, 0, 0));
    else return (kind == 1 ? a.band_zk : a.band_xk)[i];
  };
  (void)ld_key;  // (the search path, GW_BAND_TABLE=0)
  auto ld_zi = [&](uint32_t i) -> uint32_t {
    if constexpr (kBuf) return __builtin_amdgcn_raw_buffer_load_b32(r_zi, i << 2, 0, 0);
    else return a.band_zi[i];
  };
  const auto r_tab = __builtin_amdgcn_make_buffer_rsrc((void*)a.band_tab, 0, (int)(2u * a.band_tab_half), 0x00020000);
  auto ld_tab = [&](uint32_t i) -> uint32_t {
    if constexpr (kBuf) return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r_tab, i, 0, 0);
    else return a.band_tab[i];
  };
  auto ld_rec = [&](uint32_t j, uint4& ra, uint4& rb) {
    if constexpr (kBuf) {
      const auto qa = __builtin_amdgcn_raw_buffer_load_b128(r_rec, j << 5, 0, 0);
      const auto qb = __builtin_amdgcn_raw_buffer_load_b128(r_rec, (j << 5) + 16u, 0, 0);
      ra = make_uint4(qa[0], qa[1], qa[2], qa[3]);
      rb = make_uint4(qb[0], qb[1], qb[2], qb[3]);
    } else {
      ra = a.g.rec[j].a, rb = a.g.rec[j].b;
    }
  };
  const int lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6, nwaves = gridDim.x * (kDenseBlock / 64);
  const uint32_t wave = ((blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u) * (kDenseBlock / 64) + wv;
  const uint32_t nd = min(a.ctr[CTR_DENSE], a.dense_cap);
  const unsigned long long below = (1ull << lane) - 1ull;
  uint32_t nent = 0, nband = 0, nring = 0;  // the wave's movers that took the band walk / were handed over
  uint32_t cur = 0, left = 0;    // the wave's current chunk of event slots (wave-uniform)
  __shared__ uint4 mb[kDenseBlock / 64][64][2];  // the batch: {slot, Space, opq, seq0}, {x0, z0, x1, z1}
  __shared__ BandPlanL pl[kDenseBlock / 64][64];  // per batch mover: its band plan
  __shared__ uint2 pg[kDenseBlock / 64][64];     // per batch mover: its Space's {base, ntx} (cell keys)
  __shared__ float2 je[kDenseBlock / 64][64];    // per batch mover: {D, eps} of its judge
  __shared__ uint32_t lc[kDenseBlock / 64][64];  // per batch mover: its events so far
  __shared__ uint32_t orow[kDenseBlock / 64][128];  // stream_owners' marks
#if GW_BAND_TABLE
  // the Spaces' {x0, z0, 1 / cell side, D} for the key tables' buckets, in LDS (a global load per item round
  // was one more dependent round trip before the tables could be read); more Spaces: read from the grid
  __shared__ float4 sgq[kBandLdsGeoms];
  const bool lgq = a.nspaces <= kBandLdsGeoms;
  if (lgq)
    for (uint32_t k = threadIdx.x; k < a.nspaces; k += kDenseBlock)
      sgq[k] = *reinterpret_cast<const float4*>(&a.g.geom[k]);
  __syncthreads();
#endif
#if GW_STAMPS
  unsigned long long dph[16] = {}, dt0 = __builtin_amdgcn_s_memtime();
#endif
  for (uint32_t b0 = 0; wave + b0 * nwaves < nd; b0 += 64u) {
    // ---- this lane's mover: state into the batch, a band plan, the cost model, its item count ----
    const uint32_t di = wave + (b0 + (uint32_t)lane) * nwaves;
    bool elig = false;
    uint32_t ls = 0, nit = 0;
    if (di < nd) {
      ls = a.dense[di];
      const uint32_t sp = a.space_of[ls];
      const uint4 u0 = make_uint4(ls, sp, a.opq[ls], a.old_seq[ls]);
      const uint4 u1 = make_uint4(__float_as_uint(a.old_x[ls]), __float_as_uint(a.old_z[ls]),
                                  __float_as_uint(a.pos_x[ls]), __float_as_uint(a.pos_z[ls]));
      mb[wv][lane][0] = u0;
      mb[wv][lane][1] = u1;
      Mover m;
      m.slot = ls, m.q = u0.z, m.q0 = u0.w, m.rank = m.q - a.base;
      m.valid0 = m.q0 != 0, m.valid1 = true;
      m.mx0 = __uint_as_float(u1.x), m.mz0 = __uint_as_float(u1.y);
      m.mx1 = __uint_as_float(u1.z), m.mz1 = __uint_as_float(u1.w);
      const Geom gl = a.g.geom[sp];
      m.D = gl.D;
      const Judge J = make_judge(m, a.base);
      BandPlan P;
      elig = band_plan(m, gl, J, __uint_as_float(a.band_hd[2 * sp]), __uint_as_float(a.band_hd[2 * sp + 1]), P) &&
             plan_fits(P);
      if (elig) {
        // the records of the cells at the bottom / top edge midpoints: a hotspot mover's edges are crowded,
        // a large-D mover's in the sparse world around it; sparse bottom and top edges: z-strips in runs
        const int cx = (P.x0 + P.x1) >> 1;
        auto cnt = [&](int c, int r) {
          const uint32_t k = cell_key(gl, c, r);
          return (float)(a.g.cs[k + 1] - a.g.cs[k]);
        };
        const float nb = cnt(cx, P.rb0), nt = cnt(cx, P.rt1);
        P.zrun = kBandRun > 0.0f && nb + nt < 2.0f * kBandRun ? 1 : 0;
        nit = band_items(P);
        // (every mover with a band plan takes the band walk: a per-mover cost model choosing the ring walk
        // for the movers it rated cheaper there lost on skew50, skew and strips_skew alike, r05_c17 / c18)
      }
      if (elig) {
        plan_store(pl[wv][lane], P);
        pg[wv][lane] = make_uint2(gl.base, (uint32_t)gl.ntx);
        je[wv][lane] = make_float2(J.D, J.eps);
      }
      lc[wv][lane] = 0u;
    }
    if (di < nd) a.dense2[di] = elig ? kNoKey : ls;  // the ring walk's list, in the same order
    if (!elig) nit = 0;
    nband += (uint32_t)__popcll(__ballot(elig));
    nring += (uint32_t)__popcll(__ballot(di < nd && !elig));
    const uint32_t iincl = wave_incl_scan(nit), iexcl = iincl - nit;
    const uint32_t N = __builtin_amdgcn_readlane(iincl, 63);  // the batch's band cells
    __builtin_amdgcn_wave_barrier();  // the wave's LDS ops stay in program order
#if GW_STAMPS
    dph[11] += N;
    dph[15] += (uint32_t)__popcll(__ballot(elig));
#endif
    GW_DPH(0);
    // ---- item rounds: 2 cells per lane ----
    for (uint32_t ib = 0; ib < N; ib += 128u) {
      uint32_t p0[2], p1[2], mk[2];
      float w0[2], w1[2];
      int kind[2], dd[2], iow[2], span[2];
#if GW_BAND_TABLE
      int cl[2];     // the cell's column (x-strip item) or row (z-strip item): its key table's buckets
      float4 gq[2];  // the mover's Space: {x0, z0, 1 / cell side, D}
#endif
      stream_owners(orow[wv], iexcl, nit, ib, iow[0], iow[1]);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t it = ib + (uint32_t)(u * 64 + lane);
        // (every lane takes part in the lane moves: a source lane outside a divergent branch is inactive)
        const int k = iow[u];
        const uint32_t kex = (uint32_t)__shfl((int)iexcl, k, 64);
        mk[u] = (uint32_t)k;
        p0[u] = p1[u] = 0u;
        kind[u] = 3, dd[u] = 0, span[u] = 0, w0[u] = w1[u] = 0.0f;
#if GW_BAND_TABLE
        cl[u] = 0;
        gq[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#endif
        if (it < N) {
          const BandPlan P = plan_load(pl[wv][k]);
          const uint2 sg = pg[wv][k];
          int c, r;
          band_item(P, it - kex, c, r, w0[u], w1[u], kind[u], dd[u], span[u]);
#if GW_BAND_TABLE
          // an x-strip cell in a z-strip row (a corner cell): its candidates are judged only when their x key lies
          // in the window (the key table's range is the window's buckets, a superset), so that the z-strip item
          // of the same cell judges exactly the rest (dd 1 / 2: the left / right window)
          if (kind[u] == 0 && ((r >= P.rb0 && r <= P.rb1) || (r >= P.rt0 && r <= P.rt1)))
            dd[u] = c >= P.cl0 && c <= P.cl1 ? 1 : 2;
          cl[u] = kind[u] == 1 ? r : c;
          const uint32_t sp = mb[wv][k][0].y;
          gq[u] = lgq ? sgq[sp] : *reinterpret_cast<const float4*>(&a.g.geom[sp]);  // (x0, z0, inv_c, D lead Geom)
#endif
          // (cell_key on the Space's base and tile columns)
          p0[u] = sg.x + ((uint32_t)((r >> kTileShift) * (int)sg.y + (c >> kTileShift)) << kTileCellShift) +
                  (uint32_t)(((r & (kTile - 1)) << kTileShift) | (c & (kTile - 1)));  // (the key until its starts load)
        }
      }
      GW_DPH(1);
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // cell starts of both cells, loads in flight together
        if (kind[u] != 3) {
          const uint32_t ck = p0[u];
          p0[u] = ld_cs(ck);
          p1[u] = ld_cs(ck + 1 + (uint32_t)span[u]);  // (a run: its last cell's end)
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // a cell that is unsorted (over kBandCellMax records) or small (a search costs more round trips than
        // reading its few records) is read whole, once: by its x-strip item when it has one (dd: the z-strip
        // item of a corner cell then reads nothing; the rule depends only on the cell's size, so both
        // items of a corner cell apply it alike)
        const uint32_t nc = p1[u] - p0[u];
        if (kind[u] == 4) {
          kind[u] = 2;  // a run: read whole (no x-strip column in it: no dedupe)
        } else if (kind[u] != 3 && (nc > kBandCellMax || nc < kBandSearchMin || (GW_BAND_TABLE && !a.band_tab))) {
          if (dd[u] && kind[u] == 1) p1[u] = p0[u];
          if (kind[u] == 0) dd[u] = 0;  // (an x-strip cell read whole: no window test)
          kind[u] = 2;
        }
      }
#if GW_STAMPS
      for (int u = 0; u < 2; ++u) {
        dph[12] += (uint32_t)__popcll(__ballot(kind[u] < 2));
        dph[13] += (uint32_t)__popcll(__ballot(kind[u] == 2));
      }
#endif
      GW_DPH(2);
#if GW_BAND_TABLE
      // key windows of the sorted cells from their key tables: the window's first and last bucket, two bytes
      // (one round trip for both cells); the range is a superset of the window by under a bucket each side
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (kind[u] < 2) {
          const float o = kind[u] == 1 ? gq[u].y : gq[u].x;
          const int i0 = band_bucket(w0[u], o, gq[u].z, cl[u]), i1 = band_bucket(w1[u], o, gq[u].z, cl[u]);
          const uint32_t tb = (kind[u] == 1 ? a.band_tab_half : 0u) + (p0[u] >> 2) * (uint32_t)kBandBuckets;
          const uint32_t lo = i0 ? ld_tab(tb + (uint32_t)i0) : 0u;
          const uint32_t hi = i1 < kBandBuckets - 1 ? ld_tab(tb + (uint32_t)i1 + 1u) : p1[u] - p0[u];
          p1[u] = p0[u] + max(hi, lo);
          p0[u] += lo;
        }
      }
#else
      {  // key windows of the sorted cells: fanout kBandFan, both bounds of both cells per round trip; while
         // both bounds are still in the same key range (a narrow window: mostly), one set of probes serves both
        uint32_t ll[2], lh[2], ul[2], uh[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          ll[u] = ul[u] = p0[u];
          lh[u] = uh[u] = kind[u] < 2 ? p1[u] : p0[u];
        }
        while (__any(lh[0] > ll[0] || uh[0] > ul[0] || lh[1] > ll[1] || uh[1] > ul[1])) {
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const uint32_t sl = (lh[u] - ll[u] + kBandFan - 1) / kBandFan, su = (uh[u] - ul[u] + kBandFan - 1) / kBandFan;
            const bool same = ll[u] == ul[u] && lh[u] == uh[u];
            uint32_t cl = 0, cu = 0, cs = 0;  // probes below the bound (a prefix: the keys are sorted)
#pragma unroll
            for (uint32_t q = 0; q < kBandFan; ++q) {
              const uint32_t ql = ll[u] + (q + 1) * sl - 1, qu = ul[u] + (q + 1) * su - 1;
              const float kl = (sl && ql < lh[u]) ? ld_key(kind[u], ql) : __builtin_inff();
              const float ku = (!same && su && qu < uh[u]) ? ld_key(kind[u], qu) : __builtin_inff();
              cl += kl < w0[u] ? 1u : 0u;
              cs += kl <= w1[u] ? 1u : 0u;
              cu += ku <= w1[u] ? 1u : 0u;
            }
            if (same) cu = cs;
            if (sl) {
              const uint32_t nll = ll[u] + cl * sl, qc = ll[u] + (cl + 1) * sl - 1;
              lh[u] = min(lh[u], qc), ll[u] = min(nll, lh[u]);
            }
            if (su) {
              const uint32_t nul = ul[u] + cu * su, qc = ul[u] + (cu + 1) * su - 1;
              uh[u] = min(uh[u], qc), ul[u] = min(nul, uh[u]);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (kind[u] < 2) p0[u] = ll[u], p1[u] = max(ul[u], ll[u]);
      }
#endif
      GW_DPH(3);
      // ---- the round's candidates: one stream over both cells of every lane, 2 per lane per round ----
      const uint32_t c0 = p1[0] - p0[0], cnt = c0 + (p1[1] - p0[1]);
      const uint32_t cincl = wave_incl_scan(cnt), cexcl = cincl - cnt;
      const uint32_t total = __builtin_amdgcn_readlane(cincl, 63);
#if GW_STAMPS
      dph[14] += total;
#endif
      // what a candidate's lane needs of its owner: stream position -> record position of each cell
      // (cb0 / cb1), the first position of the second cell, and kind | dd | mover of both cells, packed
      const uint32_t cb0 = p0[0] - cexcl, cb1 = p0[1] - (cexcl + c0), csplit = cexcl + c0;
      const uint32_t cpk = (uint32_t)kind[0] | ((uint32_t)dd[0] << 2) | (mk[0] << 4) | ((uint32_t)kind[1] << 10) |
                           ((uint32_t)dd[1] << 12) | (mk[1] << 14);
      for (uint32_t b = 0; b < total; b += 128u) {
        uint32_t mo[2], oth[2];
        int ev[2], cow[2];
        stream_owners(orow[wv], cexcl, cnt, b, cow[0], cow[1]);
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const uint32_t kc = b + (uint32_t)(v * 64 + lane);
          const int L = cow[v];
          // (five lane moves: the owner's cell bases relative to the stream, its split and packed fields)
          const bool second = kc >= (uint32_t)__shfl((int)csplit, L, 64);
          const uint32_t ob0 = (uint32_t)__shfl((int)cb0, L, 64), ob1 = (uint32_t)__shfl((int)cb1, L, 64);
          const uint32_t pos = kc + (second ? ob1 : ob0);
          const uint32_t sel = (uint32_t)__shfl((int)cpk, L, 64) >> (second ? 10 : 0);
          const int kd = (int)(sel & 3u), dl = (int)((sel >> 2) & 3u);
          mo[v] = (sel >> 4) & 63u;
          ev[v] = 0;
          oth[v] = 0;
          if (kc < total) {
            const uint32_t j = kd == 1 ? ld_zi(pos) : pos;
            uint4 ra, rb;
            ld_rec(j, ra, rb);
            bool dup = false;
            if (dl) {
              // a corner cell: its z-strip item (kd 1) skips the records whose x key lies in the x-strip's window,
              // its searched x-strip item (kd 0, key tables) judges only those (the same float test on the same key)
              const float wl0 = pl[wv][mo[v]].w[0], wl1 = pl[wv][mo[v]].w[1];
              const float wr0 = pl[wv][mo[v]].w[2], wr1 = pl[wv][mo[v]].w[3];
              float kx, kz, hx, hz;
              band_key(ra, rb, kx, kz, hx, hz);
              dup = (((dl & 1) && kx >= wl0 && kx <= wl1) || ((dl & 2) && kx >= wr0 && kx <= wr1)) == (kd == 1);
            }
            if (!dup) {
              const uint4 u0 = mb[wv][mo[v]][0], u1 = mb[wv][mo[v]][1];
              const float2 e = je[wv][mo[v]];
              Judge J;
              J.mx0 = __uint_as_float(u1.x), J.mz0 = __uint_as_float(u1.y);
              J.mx1 = __uint_as_float(u1.z), J.mz1 = __uint_as_float(u1.w);
              J.D = e.x, J.eps = e.y;
              J.lx1 = J.mx1 - J.D, J.hx1 = J.mx1 + J.D, J.lz1 = J.mz1 - J.D, J.hz1 = J.mz1 + J.D;
              J.v0 = u0.w != 0u, J.v1 = true;
              J.base = a.base, J.q = u0.z, J.q0 = u0.w, J.rank = u0.z - a.base;
              ev[v] = judge(J, ra, rb);
            }
            oth[v] = ra.z & REC_SLOT;
          }
        }
        GW_DCNT(10);
        // the round's events: slots from the wave's current chunk of ev_tmp (a ballot prefix), each event
        // numbered inside its mover by the mover's LDS counter
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const unsigned long long em = __ballot(ev[v] != 0);
          if (!em) continue;
          const uint32_t ecnt = (uint32_t)__popcll(em);
          const uint32_t pre = (uint32_t)__popcll(em & below);
          uint32_t gi = cur + pre;
          if (ecnt > left) {  // this chunk fills up: the rest goes to a fresh one
            uint32_t nbk = 0;
            if (lane == 0) nbk = atomicAdd(&a.ctr[CTR_EVENTS], kEvChunk);
            nbk = __shfl(nbk, 0, 64);
            if (pre >= left) gi = nbk + (pre - left);
            cur = nbk + (ecnt - left);
            left = kEvChunk - (ecnt - left);
          } else {
            cur += ecnt;
            left -= ecnt;
          }
          if (ev[v]) {
            const uint32_t local = atomicAdd(&lc[wv][mo[v]], 1u);
            const uint4 u0 = mb[wv][mo[v]][0];
            if (gi < a.ev_cap)
              a.ev_tmp[gi] = make_uint4(u0.z - a.base, local, u0.x, oth[v] | (ev[v] == 2 ? 0x80000000u : 0u));
            nent += ev[v] == 2 ? 1u : 0u;
          }
        }
      }
      GW_DPH(4);
    }
    __builtin_amdgcn_wave_barrier();  // the counters' atomics before their reads
    if (elig) put_count(a.rank_cnt, mb[wv][lane][0].z - a.base, lc[wv][lane]);
    __builtin_amdgcn_wave_barrier();  // every read of the batch before the next batch is written
  }
  for (uint32_t i = lane; i < left; i += 64)
    if (cur + i < a.ev_cap) a.ev_tmp[cur + i] = make_uint4(kEvHole, 0u, 0u, 0u);
  if (lane == 0 && left) atomicAdd(&a.ctr[CTR_HOLES], left);
  const uint32_t went = __shfl(wave_incl_scan(nent), 63, 64);
  if (lane == 0 && went) atomicAdd(&a.ctr[CTR_ENTER], went);
  if (lane == 0 && nband) atomicAdd(&a.ctr[CTR_BAND_MV], nband);
  if (lane == 0 && nring) atomicAdd(&a.ctr[CTR_RING_MV], nring);
  // (events numbered in walk order: the slices are sorted whenever the list is not empty)
  if (blockIdx.x == 0 && threadIdx.x == 0 && nd) a.ctr[CTR_UNSORTED] = 1u;
#if GW_STAMPS
  if (lane == 0)
    for (int k = 0; k < 16; ++k) atomicAdd(&gw_stamps[kStampWords * 16381 + k], dph[k]);
#endif
}

// ---- Small pass (k_sweep_small) ---------------------------------------------------------------------
// A pass with few ops does not rebuild the grid: each op's mover (one wave) walks its boxes' cells in the
// grid of the last full build, then scans the overlay, and judges as the full sweep does:
//   - a grid record stands for its slot's CURRENT state when the slot has had no op since that build
//     (ov_tag != gen): its end position and seq (a slot without an op in a pass has start = end); ghosts
//     of that build are stale and skipped, as is every record of a slot in the overlay;
//   - an overlay record (one per slot with an op since the build, written by k_apply) is the record the
//     grid build would have written for the slot's last op; if that op was not in this pass, it is
//     likewise read as the slot's current state (a ghost: the slot is absent).
// Events are numbered in walk order (k_slice_sort sorts) and written into event slots the wave reserves
// kEvChunk at a time.
__device__ __forceinline__ int judge_small(const Judge& J, uint32_t base, uint32_t n_ops, uint4 ra, uint4 rb) {
  if (ra.w - base >= n_ops) {  // no op in this pass: the record's end state is the slot's state now
    if (ra.z & REC_GHOST) return 0;
    ra.z &= REC_SLOT;
    rb = make_uint4(ra.x, ra.y, rb.w, rb.w);
  }
  return judge(J, ra, rb);
}

// kW waves per op: a block of max(kBlock, 64 kW) threads takes kBlock / 64 ops (kW = 1) or one op (kW > 1);
// with kW > 1 the op's grid rows and overlay entries are dealt round-robin over its waves, and the
// mover's event numbering is an LDS counter the waves share (a pass of a single Enter: 16 waves walk its
// box and a 16k-entry overlay together, instead of one wave's 256 dependent loads).
// kOne (a pass of one host op, SmallArgs.one_op): thread 0 first applies the op (k_apply's work: no
// separate launch), the mover's state goes through LDS, the events are also kept in LDS, and after the
// walk the block orders the slice (rank by key) into ev_out and publishes the counters: one launch for
// the whole pass.
constexpr uint32_t kOneEv = 4096;  // kOne: events of the op kept in LDS
struct OneSmem {
  uint2 lev[kOneEv];
  uint32_t st[8];  // slot, raw kind, seq before, space, x0, z0, x1, z1 (float bits)
};
template <int kW, bool kOne>
__global__ void __launch_bounds__(kW == 1 ? kBlock : 64 * kW) k_sweep_small(SmallArgs a) {
  constexpr int kThreads = kW == 1 ? kBlock : 64 * kW;
  static_assert(!kOne || kW > 1, "one op per block");
  __shared__ uint32_t sloc;  // kW > 1: the op's events numbered so far
  __shared__ __attribute__((aligned(16))) uint32_t one_raw[kOne ? sizeof(OneSmem) / 4 : 1];
  OneSmem* one = reinterpret_cast<OneSmem*>(one_raw);  // (kOne only)
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const uint32_t i = kW == 1 ? blockIdx.x * (kThreads / 64) + wv : blockIdx.x;  // the wave's op
  const int sub = kW == 1 ? 0 : wv;  // the wave's share of the op's work
  const uint32_t n = a.n_dev ? min(*a.n_dev, a.n_ops) : a.n_ops;
  if (kW > 1 && threadIdx.x == 0) sloc = 0;
  if (kOne && threadIdx.x == 0) {  // k_apply for the op (host-staged: validated on the host)
    const ApplyArgs& p = a.ap;
    // the op from the kernel's arguments; then the slot's state, all loads in flight
    const uint32_t s = a.one_slot;
    const uint8_t raw = (uint8_t)a.one_kind, kind = raw & OP_KIND;
    const float ox = a.one_x, oz = a.one_z;
    const uint32_t osp = a.one_space;
    const uint32_t q = p.base, q0 = p.seq[s], sp0 = p.space_of[s], tag = p.ov_tag[s], oidx = p.ov_idx[s];
    const float x0 = p.pos_x[s], z0 = p.pos_z[s];
    p.cp_slot[0] = s;  // (a re-run of the sweep reads the op from the device copies)
    p.cp_kind[0] = raw;
    p.ctr[CTR_NOPS] = 1u;
    p.rank_cnt[0] = 0u;
    p.rank_cnt[1] = 0u;
    p.old_x[s] = x0;
    p.old_z[s] = z0;
    p.old_seq[s] = q0;
    p.opq[s] = q;
    const bool leave = kind == OP_LEAVE;
    const float x1 = leave ? x0 : ox, z1 = leave ? z0 : oz;
    const uint32_t sp = kind == OP_ENTER ? osp : sp0;
    p.seq[s] = leave ? 0u : q;
    if (!leave) {
      p.pos_x[s] = x1;
      p.pos_z[s] = z1;
    }
    if (kind == OP_ENTER) p.space_of[s] = sp;
    // overlay_put with the slot's tag already loaded
    uint32_t e = oidx;
    if (tag != p.gen) {
      e = atomicAdd(p.ov_count, 1u);
      p.ov_tag[s] = p.gen;
      p.ov_idx[s] = e;
    }
    if (e < p.ov_cap) {
      const uint4 ra = make_uint4(__float_as_uint(leave ? x0 : x1), __float_as_uint(leave ? z0 : z1),
                                  s | (leave ? REC_GHOST : 0u), q);
      const uint4 rb = make_uint4(__float_as_uint(q0 ? x0 : x1), __float_as_uint(q0 ? z0 : z1), q0, leave ? 0u : q);
      p.ov_rec[e] = Rec{ra, rb};
    }
    one[0].st[0] = s, one[0].st[1] = raw, one[0].st[2] = q0, one[0].st[3] = sp;
    one[0].st[4] = __float_as_uint(x0), one[0].st[5] = __float_as_uint(z0);
    one[0].st[6] = __float_as_uint(x1), one[0].st[7] = __float_as_uint(z1);
  }
  if (kW > 1) __syncthreads();
  bool run = i < n;  // wave-uniform (kW > 1: block-uniform)
  uint8_t kind = 0;
  uint32_t s = 0;
  if (kOne) {
    kind = (uint8_t)one[0].st[1];
    s = one[0].st[0];
  } else if (run) {
    kind = a.op_kind ? a.op_kind[i] : (uint8_t)OP_MOVE;
    s = a.op_slot[i];
    run = a.opq[s] == a.base + i;  // (a failed op: the batch is refused anyway)
  }
  run = run && !(kind & OP_SILENT);
  if (!kOne && !run) return;
  uint32_t local = 0, nent = 0, cur = 0, left = 0;  // (wave-uniform but nent)
  if (run) {
    const uint32_t sp = __builtin_amdgcn_readfirstlane(kOne ? one[0].st[3] : a.space_of[s]);
    const Geom g = uniform_geom(&a.g.geom[sp]);
    Mover m;
    m.slot = s;
    m.q = a.base + i;
    m.q0 = kOne ? one[0].st[2] : a.old_seq[s];
    m.rank = i;
    m.valid0 = m.q0 != 0;
    m.valid1 = (kind & OP_KIND) != OP_LEAVE;
    m.mx0 = kOne ? __uint_as_float(one[0].st[4]) : a.old_x[s];
    m.mz0 = kOne ? __uint_as_float(one[0].st[5]) : a.old_z[s];
    m.mx1 = !m.valid1 ? m.mx0 : kOne ? __uint_as_float(one[0].st[6]) : a.pos_x[s];
    m.mz1 = !m.valid1 ? m.mz0 : kOne ? __uint_as_float(one[0].st[7]) : a.pos_z[s];
    m.D = g.D;
    const Judge J = make_judge(m, a.base);
    const Walk w = make_walk(m, g);
    const unsigned long long below = (1ull << lane) - 1ull;
    auto emit_round = [&](int ev, uint32_t other) {
      const unsigned long long em = __ballot(ev != 0);
      if (!em) return;
      const uint32_t cnt = (uint32_t)__popcll(em), pre = (uint32_t)__popcll(em & below);
      uint32_t lb = local;  // this round's first local index
      if (kW > 1) {
        if (lane == 0) lb = atomicAdd(&sloc, cnt);  // LDS atomic
        lb = __shfl(lb, 0, 64);
      }
      uint32_t gi = cur + pre;
      if (cnt > left) {  // this reservation fills up: the rest goes to a fresh one
        // (kW > 1: small reservations — a small pass's events are few and spread over many waves, and
        // every reserved slot is read by the order stage, holes included)
        const uint32_t res = max(kW > 1 ? 16u : kEvChunk, cnt);
        uint32_t nb = 0;
        if (lane == 0) nb = atomicAdd(&a.ctr[CTR_EVENTS], res);
        nb = __shfl(nb, 0, 64);
        if (pre >= left) gi = nb + (pre - left);
        cur = nb + (cnt - left);
        left = res - (cnt - left);
      } else {
        cur += cnt;
        left -= cnt;
      }
      if (ev) {
        const uint32_t ow = other | (ev == 2 ? 0x80000000u : 0u);
        if (gi < a.ev_cap) a.ev_tmp[gi] = make_uint4(m.rank, lb + pre, m.slot, ow);
        if (kOne && lb + pre < kOneEv) one[0].lev[lb + pre] = make_uint2(m.slot, ow);
        nent += ev == 2 ? 1u : 0u;
      }
      local += cnt;
    };
    // (o == the mover: never an event; in kOne its overlay tag and entry were written by this block)
    auto cand = [&](uint32_t j, bool on) {  // grid record j (on: a candidate of this lane)
      int ev = 0;
      uint32_t o = 0;
      if (on) {
        const uint4 ra = a.g.rec[j].a;
        o = ra.z & REC_SLOT;
        if (o != s && a.ov_tag[o] != a.gen) ev = judge_small(J, a.base, a.n_ops, ra, a.g.rec[j].b);
      }
      emit_round(ev, o);
    };
    // the grid: the walk's rows (this wave's share), each row segment's records 64 at a time across the lanes
    for (int r = w.z0 + sub; r <= w.z1; r += kW) {
      int a0, a1, b0, b1;
      walk_row(w, r, a0, a1, b0, b1);
      auto seg = [&](int c0, int c1) {
        row_entries_ranges(g, a.g.cs, r, c0, c1, [&](uint32_t jb, uint32_t je) {
          for (uint32_t j = jb; j < je; j += 64) cand(j + lane, j + lane < je);
        });
      };
      seg(a0, a1);
      seg(b0, b1);
    }
    // the overlay (this wave's share), four entries per lane in flight
    const uint32_t nov = __hip_atomic_load(a.ov_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    constexpr uint32_t kStride = 64u * kW;
    for (uint32_t e0 = 64u * sub; e0 < nov; e0 += 4u * kStride) {
      Rec r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t e = e0 + k * kStride + lane;
        if (e < nov) r[k] = a.ov_rec[e];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t e = e0 + k * kStride + lane;
        int ev = 0;
        uint32_t o = 0;
        if (e < nov) {
          o = r[k].a.z & REC_SLOT;
          if (o != s) ev = judge_small(J, a.base, a.n_ops, r[k].a, r[k].b);
        }
        emit_round(ev, o);
      }
    }
    for (uint32_t k = lane; k < left; k += 64)
      if (cur + k < a.ev_cap) a.ev_tmp[cur + k] = make_uint4(kEvHole, 0u, 0u, 0u);
    if (lane == 0 && left) atomicAdd(&a.ctr[CTR_HOLES], left);
    const uint32_t went = __shfl(wave_incl_scan(nent), 63, 64);
    if (lane == 0 && went) atomicAdd(&a.ctr[CTR_ENTER], went);
  }
  if (kW == 1) {
    if (lane == 0) {
      put_count(a.rank_cnt, i, local);
      if (local > 1u) a.ctr[CTR_UNSORTED] = 1u;
    }
    return;
  }
  __syncthreads();  // every wave's events numbered
  const uint32_t nev = sloc;
  if (!kOne) {
    if (threadIdx.x == 0) {
      put_count(a.rank_cnt, i, nev);
      if (nev > 1u) a.ctr[CTR_UNSORTED] = 1u;
    }
    return;
  }
  // kOne: the order stage of the pass (k_order_small's work for one op, the slice in LDS)
  const OrderArgs& o = a.od;
  uint32_t* ctr = a.ctr;
  const uint32_t slots = __hip_atomic_load(&ctr[CTR_EVENTS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool fits = slots <= o.g.tmp_cap && o.g.keep + nev <= o.g.out_cap;
  if (threadIdx.x == 0) {
    ctr[CTR_NEV] = nev;  // (also on overflow: the host sizes ev_out by it)
    a.rank_cnt[1] = nev;  // the scanned form: [0, nev)
    if (nev > 1u) ctr[CTR_UNSORTED] = 1u;
  }
  if (fits) {
    if (threadIdx.x < CTR_N) o.ctr_next[threadIdx.x] = 0u;
    if (threadIdx.x == 0) ctr[CTR_RECORDS] = *o.grid_total;
    if (nev > kOneEv) {
      if (threadIdx.x == 0) ctr[CTR_SMALL_OVF] = 1u;  // the host orders from ev_tmp
    } else {
      for (uint32_t e = threadIdx.x; e < nev; e += kThreads) {
        const uint2 v = one[0].lev[e];
        uint32_t pos = 0;
        for (uint32_t k = 0; k < nev; ++k) {
          const uint32_t kk = one[0].lev[k].y;
          pos += (kk < v.y || (kk == v.y && k < e)) ? 1u : 0u;
        }
        o.ev_out[pos] = v;
        if (o.host_out) o.host_out[pos] = v;  // (mapped host memory: visible at the publication below)
      }
    }
  }
  if (!o.pub) return;
  __threadfence();
  __syncthreads();
  if (threadIdx.x < (uint32_t)kPubWords) {
    __hip_atomic_store(&o.pub[threadIdx.x], atomicAdd(&ctr[threadIdx.x], 0u), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
  }
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&o.pub[kPubWords], o.pub_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr uint32_t kSmallWideOps = 64;  // passes of at most this many ops: 16 waves per op
void launch_sweep_small(const SmallArgs& a, hipStream_t st) {
  if (!a.n_ops) return;
  if (a.one_op)
    hipLaunchKernelGGL((k_sweep_small<16, true>), dim3(1), dim3(1024), 0, st, a);
  else if (a.n_ops <= kSmallWideOps)
    hipLaunchKernelGGL((k_sweep_small<16, false>), dim3(a.n_ops), dim3(1024), 0, st, a);
  else if (a.n_ops <= kOrderSmallOps)
    hipLaunchKernelGGL((k_sweep_small<4, false>), dim3(a.n_ops), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((k_sweep_small<1, false>), dim3((a.n_ops + kBlock / 64 - 1) / (kBlock / 64)), dim3(kBlock), 0,
                       st, a);
}

uint32_t sweep_ev_lds() { return kEvLds; }

// The global walks' grids: GW_*_WPE waves per SIMD on every CU of the device, the CU count rounded up to a
// multiple of the 8 XCDs (their wave numbering is XCD-aware and needs it). 256 CUs on MI355X; read from the
// device once per process and device (a fixed 256 assumed the part).
uint32_t cu_grid(int wpe) {
  static int cus[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  int& c = cus[dev & 63];
  if (!c) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    c = (v + 7) / 8 * 8;
  }
  return (uint32_t)c * (uint32_t)wpe;
}

void launch_sweep(const SweepArgs& a, hipStream_t st) {
  if (a.ntiles) hipLaunchKernelGGL(k_sweep<SwSmall>, dim3(a.ntiles), dim3(kSweepBlock), sizeof(SweepSmem), st, a);
  if (a.mid_n && a.use_lds)
    hipLaunchKernelGGL(k_sweep<SwMid>, dim3(a.mid_n), dim3(SwMid::kBlk), sizeof(SweepSmemT<SwMid>), st, a);
  if (a.big_n && a.use_lds)
    hipLaunchKernelGGL(k_sweep<SwBig>, dim3(a.big_n), dim3(SwBig::kBlk), sizeof(SweepSmemT<SwBig>), st, a);
  if (a.leave_blocks)
    hipLaunchKernelGGL(k_sweep_leaves, dim3(a.leave_blocks * ((kSweepBlock + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       st, a);
  // the dense list's length is on the device: a fixed grid that exits at once when it is empty. Not
  // launched at all when the previous pass had no dense mover (an empty launch cost 4.8 us per config-2
  // tick): if this pass lists some after all, the host re-runs the sweep with it (run_pass)
  if (a.dense && a.dense_hint) {
    if (a.band_xk && a.dense2) {  // the band walk, then the ring walk of the movers it hands over
      // (buffer loads when every array the band walk reads is below 2 GiB; the keys as one allocation)
      const bool buf = (uint64_t)a.n_rec * 32u < (1ull << 31) && ((uint64_t)a.ncells + 1u) * 4u < (1ull << 31) &&
                       (uint64_t)(a.band_zk - a.band_xk) * 8u < (1ull << 31) && a.band_zk > a.band_xk;
      if (buf)
        hipLaunchKernelGGL(k_sweep_band<true>, dim3(cu_grid(GW_BAND_WPE)), dim3(kDenseBlock), 0, st, a);
      else
        hipLaunchKernelGGL(k_sweep_band<false>, dim3(cu_grid(GW_BAND_WPE)), dim3(kDenseBlock), 0, st, a);
      hipLaunchKernelGGL(k_sweep_dense<true>, dim3(cu_grid(GW_DENSE_WPE)), dim3(kDenseBlock), 0, st, a);
    } else {
      hipLaunchKernelGGL(k_sweep_dense<false>, dim3(cu_grid(GW_DENSE_WPE)), dim3(kDenseBlock), 0, st, a);
    }
  }
}

// Canonical order: events bucketed by the mover's op rank (scan of per-rank counts), then each
// rank's slice sorted by other|kind (LEAVE = bit31 clear sorts first). Every step checks on the
// device that the sweep's events fit the buffers (else it writes nothing; the host grows them and
// re-runs), so the host synchronises once per pass. Two side jobs ride along: k_place zeroes the
// cell counts of the grid the NEXT pass builds and the next pass's counter block; k_slice_sort
// validates device-staged batches (every op's slot must carry that op's seq).
// slots of the shared region, and the pass's events (the scan total of the per-op counts)
__device__ __forceinline__ bool ev_fits(const OrderArgs& o, uint32_t* slots, uint32_t* n) {
  *slots = o.g.ctr[CTR_EVENTS];
  *n = o.rank_off[o.n_ops];
  return *slots <= o.g.tmp_cap && o.g.keep + *n <= o.g.out_cap;
}

#ifndef GW_PLACE_UNROLL
#define GW_PLACE_UNROLL 8
#endif
constexpr int kPlaceU = GW_PLACE_UNROLL;
__global__ void __launch_bounds__(kBlock) k_place(OrderArgs o) {
  const uint32_t tid = blockIdx.x * kBlock + threadIdx.x, nth = gridDim.x * kBlock;
  uint32_t slots, n;
  const bool fits = ev_fits(o, &slots, &n);
  if (tid == 0) const_cast<uint32_t*>(o.g.ctr)[CTR_NEV] = n;  // (also on overflow: the host sizes ev_out by it)
  // An overflowing pass is re-run from the sweep, which still reads the old grid: side jobs only
  // once the pass is final.
  if (!fits) return;
  for (uint32_t i = tid; i < o.zero_n; i += nth) o.zero_cs[i] = 0u;
  if (tid < CTR_N) o.ctr_next[tid] = 0u;
  if (tid == 0) const_cast<uint32_t*>(o.g.ctr)[CTR_RECORDS] = *o.grid_total;
  if (o.ev_fix) {
    // the tiles' regions: entry r of tile t holds an event when r < tile_ev[t]. Four entries per thread
    // and round, every entry and count loaded before any test (one memory round trip, then the gathers)
    const uint32_t nf = o.ntiles_fix * (uint32_t)kEvLds;
    constexpr int kU = 4;
    for (uint32_t i0 = tid; i0 < nf; i0 += kU * nth) {
      uint4 e[kU];
      uint32_t c[kU];
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const uint32_t i = i0 + k * nth;
        c[k] = i < nf ? o.tile_ev[i / (uint32_t)kEvLds] : 0u;
        e[k] = i < nf ? o.ev_fix[i] : make_uint4(0u, 0u, 0u, 0u);
      }
      uint32_t pos[kU];
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const uint32_t i = i0 + k * nth;
        const bool on = i < nf && i % (uint32_t)kEvLds < c[k];
        c[k] = on;
        pos[k] = on ? o.rank_off[e[k].x] + e[k].y : 0u;
      }
#pragma unroll
      for (int k = 0; k < kU; ++k)
        if (c[k]) o.ev_out[pos[k]] = make_uint2(e[k].z, e[k].w);
    }
    if (blockIdx.x == 0) {  // the tiles' enter events into the pass counter (one atomic)
      uint32_t ne = 0;
      for (uint32_t t = threadIdx.x; t < o.ntiles_fix; t += kBlock) ne += o.tile_ent[t];
      uint32_t tot;
      block_excl_scan(ne, &tot);
      if (threadIdx.x == 0 && tot) atomicAdd(const_cast<uint32_t*>(&o.g.ctr[CTR_ENTER]), tot);
    }
  }
  if (o.ntiles_acted && blockIdx.x == 1 % gridDim.x) {  // device batch: every op on a slot of its own
    uint32_t na = 0;
    for (uint32_t t = threadIdx.x; t < o.ntiles_acted; t += kBlock) na += o.tile_acted[t];
    uint32_t tot;
    block_excl_scan(na, &tot);
    // (an overflowed one-pass build published an empty grid: the pass re-runs, nothing to check)
    if (threadIdx.x == 0 && tot != o.g.ctr[CTR_NOPS] && !o.g.ctr[CTR_BOVF])
      atomicOr(const_cast<uint32_t*>(&o.g.ctr[CTR_ERR]), ERR_DUP_SLOT);
  }
  // kPlaceU slots per thread and round, every load of a round issued before the first use: one event at a
  // time, each thread's chain (the slot, then its op's offset, then the store) waited out two memory round
  // trips per event (skew50's 21M events: 180 us)
  for (uint32_t i0 = tid; i0 < slots; i0 += kPlaceU * nth) {
    uint4 e[kPlaceU];
#pragma unroll
    for (int k = 0; k < kPlaceU; ++k) {
      const uint32_t i = i0 + (uint32_t)k * nth;
      e[k] = i < slots ? o.ev_tmp[i] : make_uint4(kEvHole, 0u, 0u, 0u);
    }
    uint32_t ro[kPlaceU];
#pragma unroll
    for (int k = 0; k < kPlaceU; ++k) ro[k] = e[k].x != kEvHole ? o.rank_off[e[k].x] : 0u;
#pragma unroll
    for (int k = 0; k < kPlaceU; ++k)
      if (e[k].x != kEvHole) o.ev_out[ro[k] + e[k].y] = make_uint2(e[k].z, e[k].w);
  }
}

// Per-op slices are sorted by .y (other | ENTER bit: LEAVE first, then other ascending), inside one
// kernel without global atomics (a shared work-list counter bumped by every wave serialises at ~88
// returning atomics per us): slices of up to kSmallSlice events (config 2: ~0.3 per op) are sorted in
// registers by their op's thread (an odd-even transposition network, static indices only); up to
// GW_MED_MAX by the op's wave (each lane holds events and counts the events ordered before them); longer ones
// (crowds: hundreds per mover) by the whole block: chunks of kBigChunk events are bitonic-sorted in
// LDS, and a slice of several chunks is merged by rank: an element's final index is its index in its
// sorted chunk plus, for every other chunk, the count of elements ordered before it there (binary
// search; ties go to the earlier chunk, so the merge is stable). The chunks are parked in ev_tmp,
// free once k_place has run (its uint2 view has 2 x slots >= n entries).
// Ascending sort of N registers by Batcher's odd-even merge network for any N (comparators past N
// dropped): 191 / 305 / 384 / 543 compare-exchanges for N = 32 / 40 / 48 / 64 (bitonic 64: 672).
template <int N>
__device__ __forceinline__ void net_sort(uint32_t (&r)[N]) {
#pragma unroll
  for (int p = 1; p < N; p <<= 1) {
#pragma unroll
    for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
      for (int j = k % p; j + k < N; j += 2 * k) {
#pragma unroll
        for (int i = 0; i < k && i + j + k < N; ++i) {
          if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            const uint32_t x = r[i + j], y = r[i + j + k];
            r[i + j] = min(x, y);
            r[i + j + k] = max(x, y);
          }
        }
      }
    }
  }
}

constexpr uint32_t kSmallSlice = 8;
constexpr uint32_t kBigChunk = 2048;
// diagnosis only (A/B of where k_slice_sort's time goes; the result is then NOT sorted): 1 skips the wave
// windows, 2 the block sorts, 3 the register sorts, 4 every sort; 5 the windows' ranking and stores (loads
// only), 6 the windows' stores
#ifndef GW_DIAG_SORT
#define GW_DIAG_SORT 0
#endif
// longest slice ranked by one wave in its LDS window (below: the block's bitonic sort). Round 6: 64 -> 256
#ifndef GW_MED_MAX
#define GW_MED_MAX 256u
#endif
__device__ __forceinline__ uint32_t seg_key(const uint2 v) { return v.y; }
__device__ __forceinline__ uint32_t seg_key(const uint32_t v) { return v; }
template <class T> __device__ __forceinline__ T seg_pad();
template <> __device__ __forceinline__ uint2 seg_pad<uint2>() { return make_uint2(0xffffffffu, 0xffffffffu); }
template <> __device__ __forceinline__ uint32_t seg_pad<uint32_t>() { return 0xffffffffu; }
__device__ __forceinline__ uint32_t ld_cg(const uint32_t* p) {  // bypass the CU cache: written by this block
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint2 ld_cg(const uint2* p) {
  return make_uint2(ld_cg(&p->x), ld_cg(&p->y));
}

// one long segment d[0, len), the whole block (kBlock threads); tmp[0, len) is scratch
template <class T>
__device__ void seg_sort_long(T* __restrict__ d, T* __restrict__ tmp, uint32_t len, T* sk) {
  const uint32_t nch = (len + kBigChunk - 1) / kBigChunk;
  for (uint32_t c = 0; c < nch; ++c) {
    const uint32_t c0 = c * kBigChunk, cl = min(kBigChunk, len - c0);
    uint32_t P = 64;
    while (P < cl) P <<= 1;
    for (uint32_t i = threadIdx.x; i < P; i += kBlock) sk[i] = i < cl ? d[c0 + i] : seg_pad<T>();
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t i = threadIdx.x; i < P; i += kBlock) {
          const uint32_t l = i ^ j;
          if (l > i) {
            const T u = sk[i], v = sk[l];
            if ((seg_key(u) > seg_key(v)) == ((i & k) == 0)) {
              sk[i] = v;
              sk[l] = u;
            }
          }
        }
        __syncthreads();
      }
    }
    T* dst = nch == 1 ? d : tmp + c0;
    for (uint32_t i = threadIdx.x; i < cl; i += kBlock) dst[i] = sk[i];
    __syncthreads();
  }
  if (nch > 1) {
    __threadfence();
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < len; i += kBlock) {
      const T v = ld_cg(tmp + i);
      const uint32_t kv = seg_key(v);
      const uint32_t c = i / kBigChunk;
      uint32_t pos = i - c * kBigChunk;
      for (uint32_t c2 = 0; c2 < nch; ++c2) {
        if (c2 == c) continue;
        const T* ch = tmp + c2 * kBigChunk;
        uint32_t lo = 0, hi = min(kBigChunk, len - c2 * kBigChunk);
        while (lo < hi) {  // earlier chunks: count keys <= v (ties before); later: keys < v
          const uint32_t mid = (lo + hi) >> 1;
          const uint32_t ky = seg_key(ld_cg(ch + mid));
          if (c2 < c ? ky <= kv : ky < kv) lo = mid + 1;
          else hi = mid;
        }
        pos += lo;
      }
      d[pos] = v;
    }
    __syncthreads();
  }
}

// Segmented sort, one segment per thread of the block: segment [b, b + len) of d (len = 0: none).
// Every thread of the block must call it. Short segments by their thread, medium by their wave,
// long ones by the block; tmp mirrors d (scratch for segments longer than one LDS chunk).
template <class T>
__device__ void seg_sort(T* __restrict__ d, T* __restrict__ tmp, uint32_t b, uint32_t len, T* sk, uint2* bigq,
                         uint32_t* nbig) {
  if (threadIdx.x == 0) *nbig = 0;
  if (GW_DIAG_SORT != 3 && GW_DIAG_SORT != 4 && len >= 2u && len <= kSmallSlice &&
      std::is_same<T, uint2>::value) {
    // an event slice: .x is its mover for every element, so only the keys move (Batcher's network, 19
    // min / max pairs for 8; equal keys are equal events)
    uint32_t y[kSmallSlice];
    uint32_t x0 = 0;
#pragma unroll
    for (uint32_t i = 0; i < kSmallSlice; ++i) {
      const T e = i < len ? d[b + i] : seg_pad<T>();
      y[i] = seg_key(e);
      if (i == 0) x0 = reinterpret_cast<const uint2&>(e).x;
    }
    net_sort<kSmallSlice>(y);
#pragma unroll
    for (uint32_t i = 0; i < kSmallSlice; ++i)
      if (i < len) reinterpret_cast<uint2*>(d)[b + i] = make_uint2(x0, y[i]);
  } else if (GW_DIAG_SORT != 3 && GW_DIAG_SORT != 4 && len >= 2u && len <= kSmallSlice) {
    T v[kSmallSlice];
#pragma unroll
    for (uint32_t i = 0; i < kSmallSlice; ++i) v[i] = i < len ? d[b + i] : seg_pad<T>();
#pragma unroll
    for (uint32_t p = 0; p < kSmallSlice; ++p) {
#pragma unroll
      for (uint32_t i = p & 1u; i + 1 < kSmallSlice; i += 2) {
        const T x = v[i], y = v[i + 1];
        const bool sw = seg_key(x) > seg_key(y);  // strict: equal keys keep their order (stable)
        v[i] = sw ? y : x;
        v[i + 1] = sw ? x : y;
      }
    }
#pragma unroll
    for (uint32_t i = 0; i < kSmallSlice; ++i)
      if (i < len) d[b + i] = v[i];
  }
  // medium segments (kSmallSlice < len <= GW_MED_MAX): the wave's together, in windows of up to kMedWin elements
  // (whole segments, in lane order) staged in the wave's share of sk with all loads in flight at once; an
  // element's final index is the count of its segment's elements ordered before it (key, then position:
  // stable), read from the window (the lanes of one segment read the same element at a time: broadcast).
  // (One segment at a time, the wave paid a dependent global round trip per segment: skew50's ~1M medium
  // slices made k_slice_sort 338 us. Slices of 65..256 went to the block's bitonic sort, one slice at a time
  // with a barrier per stage; in a wave window each costs ~len / 64 rounds of len LDS reads.)
  constexpr uint32_t kMedWin = kBigChunk / (kBlock / 64);
  constexpr uint32_t kMedRounds = kMedWin / 64u;
  const uint32_t lane = threadIdx.x & 63u;
  T* win = sk + (threadIdx.x >> 6) * kMedWin;
  static_assert(GW_MED_MAX <= kMedWin, "a medium slice fits one wave window");
  const uint32_t lm = (len > kSmallSlice && len <= (uint32_t)GW_MED_MAX) ? len : 0u;
  const uint32_t incl = wave_incl_scan(lm), excl = incl - lm;
  const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  for (uint32_t w0 = 0; w0 < ((GW_DIAG_SORT == 1 || GW_DIAG_SORT == 4) ? 0u : tot);) {  // wave-uniform; each window holds the next segment at least
    const unsigned long long fit = __ballot(incl <= w0 + kMedWin);  // a prefix of the lanes
    const int last = __builtin_amdgcn_readfirstlane(63 - __clzll((long long)fit));
    const uint32_t wend = (uint32_t)__builtin_amdgcn_readlane((int)incl, last);
    const uint32_t n = wend - w0;
    T v[kMedRounds];
    int own[kMedRounds];  // the lane owning the round's element, found once per window
#pragma unroll
    for (uint32_t k = 0; k < kMedRounds; ++k) {
      const uint32_t i = k * 64u + lane;
      v[k] = seg_pad<T>();
      own[k] = 0;
      if (k * 64u < n) {  // wave-uniform: every lane takes part in the lane moves
        const uint32_t g = w0 + min(i, n - 1u);
        const int L = wave_owner(incl, g);
        own[k] = L;
        const uint32_t sb = (uint32_t)__shfl((int)b, L, 64), se = (uint32_t)__shfl((int)excl, L, 64);
        if (i < n) v[k] = d[sb + (g - se)];
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < kMedRounds; ++k)
      if (k * 64u + lane < n) win[k * 64u + lane] = v[k];
    __builtin_amdgcn_wave_barrier();  // the window's writes before its reads
    if (GW_DIAG_SORT == 5) {
      __builtin_amdgcn_wave_barrier();
      w0 = wend;
      continue;
    }
    // (The owner lanes found once per window (own[]) and the key-only network for short event slices: 198 ->
    // 180 us at skew50, r06_a15. Not kept: the window read 4, 8 or 16 keys per step, r06_a9; the ranking split
    // into two loops around the element without the tie test (lanes of one slice then read different words:
    // bank conflicts 3% -> 15%), r06_a12; a range sort, one block per 2,048 consecutive events with every slice
    // of up to 256 ranked in LDS, 243 us, r06_a11. The diagnosis builds put ~100 us of 198 in this ranking, ~32
    // in the window loads, ~15 in the stores, r06_a10.)
#pragma unroll
    for (uint32_t k = 0; k < kMedRounds; ++k) {
      const uint32_t i = k * 64u + lane;
      if (k * 64u < n) {
        const uint32_t g = w0 + min(i, n - 1u);
        const int L = own[k];
        const uint32_t sb = (uint32_t)__shfl((int)b, L, 64), se = (uint32_t)__shfl((int)excl, L, 64);
        const uint32_t sl = (uint32_t)__shfl((int)lm, L, 64);
        if (i < n) {
          const uint32_t kv = seg_key(v[k]), o = g - se, s0 = se - w0;
          uint32_t pos = 0;
          for (uint32_t j = 0; j < sl; ++j) {
            const uint32_t kj = seg_key(win[s0 + j]);
            pos += (kj < kv || (kj == kv && j < o)) ? 1u : 0u;
          }
          if (GW_DIAG_SORT != 6) d[sb + pos] = v[k];
          else if (pos == 0xFFFFFFFFu) d[0] = v[k];  // (keeps the ranking)
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the window's reads before the next window's writes
    w0 = wend;
  }
  // long segments: the whole block
  __syncthreads();
  if (len > (uint32_t)GW_MED_MAX) bigq[atomicAdd(nbig, 1u)] = make_uint2(b, len);  // LDS atomic
  __syncthreads();
  const uint32_t nb = *nbig;
  for (uint32_t q = 0; q < ((GW_DIAG_SORT == 2 || GW_DIAG_SORT == 4) ? 0u : nb); ++q) {
    const uint2 sg = bigq[q];
    seg_sort_long(d + sg.x, tmp + sg.x, sg.y, sk);
  }
}

struct SegSmem {
  uint2 bigq[kBlock];
  uint32_t nbig;
};

// Grid-stride over the ops (kBlock per block and round). Nothing to sort when every op's events were
// numbered in canonical order by the sweep (CTR_UNSORTED and CTR_UNS_SOME clear) and no batch check is
// asked; with CTR_UNS_SOME only, only the ops flagged in o.uns (the walks that number a mover's events in
// walk order flag that mover's op), whose flag words are cleared here for the next pass. When the
// previous pass needed no sort either (o.sorted_hint), the kernel runs as kSortFewBlocks blocks and the
// last one to finish (a ticket) publishes the pass's counters to mapped host memory (o.pub): no separate
// one-thread kernel (3.8 us per pass at config 2). (A ticket per block of the one-thread-per-op grid,
// 3,907 blocks at config 2, serialises on the one counter: 9 -> 15 us measured with 1,024 blocks.)
// Otherwise one thread per op, and k_publish after it.
constexpr uint32_t kSortFewBlocks = 32;
#ifndef GW_SORT_BLOCKS
#define GW_SORT_BLOCKS 0  // a sorting pass's grid at most (0: one block per kBlock ops)
#endif
__global__ void __launch_bounds__(kBlock) k_slice_sort(OrderArgs o) {
  __shared__ uint2 sk[kBigChunk];
  __shared__ SegSmem ss;
  __shared__ uint32_t last;
  uint32_t slots, n;
  const bool fits = ev_fits(o, &slots, &n);
  const bool sort_all = fits && o.g.ctr[CTR_UNSORTED] != 0u;  // grid-uniform
  const bool flagged = fits && o.g.ctr[CTR_UNS_SOME] != 0u;
  const bool sort = sort_all || flagged;
  if (sort || o.check_ops) {
    const uint32_t nr = o.n_dev ? min(*o.n_dev, o.n_ops) : o.n_ops;
    for (uint32_t r0 = blockIdx.x * kBlock; r0 < o.n_ops; r0 += gridDim.x * kBlock) {  // block-uniform
      const uint32_t r = r0 + threadIdx.x;
      const bool op = r < nr;
      if (op && o.check_ops) {
        const uint32_t s = o.op_slot[r];
        if (s < o.cap && o.opq[s] != o.base + r) atomicOr(const_cast<uint32_t*>(&o.g.ctr[CTR_ERR]), ERR_DUP_SLOT);
      }
      if (!sort) continue;
      uint32_t fw = 0;  // the op's flag word (read before the clear below)
      if (flagged && r < o.n_ops) fw = o.uns[r >> 5];
      const bool mine = op && (sort_all || ((fw >> (r & 31u)) & 1u));
      const uint32_t b = mine ? o.rank_off[r] : 0u, len = mine ? o.rank_off[r + 1] - b : 0u;
      // ev_tmp is free once k_place has run; its uint2 view has 2 x (tile regions + slots) >= n entries
      seg_sort(o.ev_out, o.scratch, b, len, sk, ss.bigq, &ss.nbig);
      if (flagged && r < o.n_ops && (r & 31u) == 0u && fw) o.uns[r >> 5] = 0u;
    }
  }
  if (!o.pub || !o.sorted_hint) return;
  // publication: the last block's ticket. Every earlier block's device-scope atomics (CTR_ERR) were
  // performed before its ticket; the counters are read with atomics too, where those meet.
  __syncthreads();
  if (threadIdx.x == 0) last = (atomicAdd(const_cast<uint32_t*>(&o.g.ctr[CTR_SDONE]), 1u) + 1u) % gridDim.x == 0u;
  __syncthreads();
  if (!last) return;
  uint32_t* ctr = const_cast<uint32_t*>(o.g.ctr);
  if (threadIdx.x < (uint32_t)kPubWords) {  // one counter per lane
    __hip_atomic_store(&o.pub[threadIdx.x], atomicAdd(&ctr[threadIdx.x], 0u), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();  // complete before the flag below
  }
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&o.pub[kPubWords], o.pub_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Deliver the ordered events to mapped pinned host memory (GPU-initiated PCIe writes), so the host
// needs no second round trip to learn the count before a copy.
__global__ void __launch_bounds__(kBlock) k_copy_out(OrderArgs o) {
  uint32_t slots, n;
  if (!ev_fits(o, &slots, &n)) return;
  // a small pass whose events overflowed k_order_small's LDS placed nothing: the host zeroes the flag and
  // runs the general order stage, whose own copy delivers them
  if (o.g.ctr[CTR_SMALL_OVF]) return;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) o.host_out[i] = o.ev_out[i];
}

void launch_order(const OrderArgs& o, hipStream_t st) {
  hipLaunchKernelGGL(k_place, dim3(o.place_blocks ? o.place_blocks : 1024u), dim3(kBlock), 0, st, o);
  const uint32_t per_op = std::max(1u, (o.n_ops + kBlock - 1) / kBlock);
  const uint32_t full = GW_SORT_BLOCKS ? std::min(per_op, (uint32_t)GW_SORT_BLOCKS) : per_op;  // (grid-stride)
  hipLaunchKernelGGL(k_slice_sort, dim3(o.sorted_hint ? std::min(per_op, kSortFewBlocks) : full), dim3(kBlock), 0,
                     st, o);
  if (o.host_out) hipLaunchKernelGGL(k_copy_out, dim3(512), dim3(kBlock), 0, st, o);
  if (o.pub && !o.sorted_hint) launch_publish(o.g.ctr, o.pub, o.pub_seq, st);
}

// The order stage of a small pass (at most kOrderSmallOps ops) as one block: the per-op counts scanned
// in LDS (and written back, as launch_scan leaves them), the events placed into LDS by op rank, each
// op's slice ordered by rank (an event's position = the events of its slice ordered before it: key,
// then index), written out once, the counters published. Replaces scan + k_place + k_slice_sort (+
// k_publish): four dependent launches of a pass whose work is a few hundred events. The side jobs of
// k_place ride along (next pass's counter block, CTR_NEV, CTR_RECORDS); the batch check of k_slice_sort
// too. A pass with more events than the LDS holds sets CTR_SMALL_OVF and places nothing.
constexpr int kOrdThreads = 1024;
constexpr uint32_t kOrdSmallEv = 4096;
static_assert(kOrderSmallOps <= (uint32_t)kOrdThreads, "one op per thread in the scan");
__global__ void __launch_bounds__(kOrdThreads) k_order_small(OrderArgs o) {
  __shared__ uint2 lev[kOrdSmallEv];            // placed events
  __shared__ uint32_t off[kOrderSmallOps + 1];  // scanned counts
  __shared__ uint32_t ws[kOrdThreads / 64];
  const uint32_t t = threadIdx.x;
  uint32_t* ctr = const_cast<uint32_t*>(o.g.ctr);
  uint32_t* rank = const_cast<uint32_t*>(o.rank_off);  // counts on entry, offsets on exit
  const uint32_t nops = o.n_ops;
  // scan (one op per thread)
  const uint32_t c = t < nops ? rank[t] : 0u;
  const uint32_t inc = wave_incl_scan(c);
  if ((t & 63) == 63) ws[t >> 6] = inc;
  __syncthreads();
  uint32_t pre = inc - c, n = 0;
#pragma unroll
  for (int k = 0; k < kOrdThreads / 64; ++k) {
    pre += k < (int)(t >> 6) ? ws[k] : 0u;
    n += ws[k];
  }
  if (t < nops) off[t] = pre, rank[t] = pre;
  if (t == 0) off[nops] = n, rank[nops] = n;
  const uint32_t slots = ctr[CTR_EVENTS];
  const bool fits = slots <= o.g.tmp_cap && o.g.keep + n <= o.g.out_cap;
  __syncthreads();
  if (t == 0) ctr[CTR_NEV] = n;  // (also on overflow: the host sizes ev_out by it)
  if (fits) {
    if (t < CTR_N) o.ctr_next[t] = 0u;
    if (t == 0) ctr[CTR_RECORDS] = *o.grid_total;
    if (o.check_ops) {
      const uint32_t nr = o.n_dev ? min(*o.n_dev, nops) : nops;
      if (t < nr) {
        const uint32_t s = o.op_slot[t];
        if (s < o.cap && o.opq[s] != o.base + t) atomicOr(&ctr[CTR_ERR], ERR_DUP_SLOT);
      }
    }
    if (n > kOrdSmallEv) {
      if (t == 0) ctr[CTR_SMALL_OVF] = 1u;
    } else {
      for (uint32_t i = t; i < slots; i += kOrdThreads) {
        const uint4 e = o.ev_tmp[i];
        if (e.x != kEvHole) lev[off[e.x] + e.y] = make_uint2(e.z, e.w);
      }
      __syncthreads();
      const bool sort = ctr[CTR_UNSORTED] != 0u;  // (written by the sweep kernel before this one)
      for (uint32_t i = t; i < n; i += kOrdThreads) {
        const uint2 v = lev[i];
        uint32_t pos = i;
        if (sort) {
          uint32_t lo = 0, hi = nops;  // the op whose slice holds event i: off[r] <= i < off[r + 1]
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (off[mid] <= i) lo = mid;
            else hi = mid;
          }
          const uint32_t b = off[lo], e = off[lo + 1];
          pos = b;
          for (uint32_t j = b; j < e; ++j) {
            const uint32_t kj = lev[j].y;
            pos += (kj < v.y || (kj == v.y && j < i)) ? 1u : 0u;
          }
        }
        o.ev_out[pos] = v;
      }
    }
  }
  if (!o.pub) return;
  __threadfence();  // this kernel's counter stores (CTR_NEV, CTR_RECORDS, ...) reach L2 before they are read
  __syncthreads();
  if (t < (uint32_t)kPubWords) {  // one counter per lane (atomics: where the sweep's atomics meet)
    __hip_atomic_store(&o.pub[t], atomicAdd(&ctr[t], 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
  }
  __syncthreads();
  if (t == 0) __hip_atomic_store(&o.pub[kPubWords], o.pub_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_copy_out(const OrderArgs& o, hipStream_t st) {
  if (o.host_out) hipLaunchKernelGGL(k_copy_out, dim3(512), dim3(kBlock), 0, st, o);
}

void launch_order_small(const OrderArgs& o, hipStream_t st) {
  hipLaunchKernelGGL(k_order_small, dim3(1), dim3(kOrdThreads), 0, st, o);
  if (o.host_out) hipLaunchKernelGGL(k_copy_out, dim3(512), dim3(kBlock), 0, st, o);
}

// End-of-pass publication (when k_slice_sort does not publish): the counters the host reads, then a
// sequence word, written by one thread into mapped (coherent) host memory with system-scope stores;
// the host spins on the sequence word instead of a DMA copy plus a stream synchronisation.
__global__ void k_publish(const uint32_t* __restrict__ ctr, uint32_t* pub, uint32_t seq) {
  const int i = threadIdx.x;
  if (i < kPubWords) {  // one counter per lane
    __hip_atomic_store(&pub[i], ctr[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();  // complete before the flag below
  }
  __syncthreads();
  if (i == 0) __hip_atomic_store(&pub[kPubWords], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_publish(const uint32_t* ctr, uint32_t* pub, uint32_t seq, hipStream_t st) {
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, st, ctr, pub, seq);
}

// A few device words the host must read between launches (the relation's sizes), published the same
// way: words a[0, na) then b[0, nb), then the sequence word.
__global__ void k_publish_words(const uint32_t* __restrict__ a, uint32_t na, const uint32_t* __restrict__ b,
                                uint32_t nb, uint32_t* pub, uint32_t seq) {
  const uint32_t i = threadIdx.x;
  if (i < na + nb) {
    __hip_atomic_store(&pub[i], i < na ? a[i] : b[i - na], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
  }
  __syncthreads();
  if (i == 0) __hip_atomic_store(&pub[kPubWords], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_publish_words(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb, uint32_t* pub,
                          uint32_t seq, hipStream_t st) {
  hipLaunchKernelGGL(k_publish_words, dim3(1), dim3(64), 0, st, a, na, b, nb, pub, seq);
}

// ---------------------------------------------------------------------------------------------
// Relation export: row s = {o : N(s,o)} = {o : in(L, F)}, L = later actor, over the END-of-pass
// state (main records only). Count pass (row_ptr null) then fill pass; rows sorted afterwards.
// One block per grid tile: the records of the tile plus a halo of `reach` cells are staged in LDS in
// row-major cell order (stage_region), so a box row is one contiguous LDS range; the block's threads
// take the tile's main records (binned = current position, b.w = current seq) in grid order. A box
// that leaves the region, or a region over the LDS budget (crowds), walks the global grid. The pair
// test is the reference's from the perspective of whichever member acted last (N(a,b) = in(L, F)).
constexpr int kRelLdsRecs = 1536;  // 24 KB (a config-2 region holds ~850 records)
__global__ void __launch_bounds__(kBlock) k_relation(RelArgs a) {
  __shared__ uint16_t cst[kSweepRegCells + 1];
  __shared__ uint4 rl[kRelLdsRecs];  // {x, z, seq_end, slot | flags}
  __shared__ uint32_t red[kBlock / 64];
  __shared__ uint32_t tot_sh;
  const uint32_t t = blockIdx.x;
  const Geom g = a.g.geom[a.g.tile_space[t]];
  const int lt = (int)(t - g.tile_base);
  const int tx = lt % g.ntx, tz = lt / g.ntx;
  const uint32_t k0 = g.base + ((uint32_t)lt << kTileCellShift);
  const uint32_t j0 = a.g.cs[k0], j1 = a.g.cs[k0 + kTileCells];
  if (j0 == j1) {
    if (!a.row_ptr && threadIdx.x == 0) a.tstat[t] = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  const int R = g.reach;
  const int cx0 = max(tx * kTile - R, 0), cx1 = min(tx * kTile + kTile - 1 + R, g.ncx - 1);
  const int cz0 = max(tz * kTile - R, 0), cz1 = min(tz * kTile + kTile - 1 + R, g.ncz - 1);
  const int W = cx1 - cx0 + 1, ncell = W * (cz1 - cz0 + 1);
  const bool lds = R > 0 && ncell <= kSweepRegCells &&
                   stage_region<kBlock, kSweepRegCells, kRelLdsRecs>(g, a.g.cs, cx0, cz0, W, ncell, cst, rl, red,
                                                                     &tot_sh, [&](uint32_t q) {
                                                          const Rec r = a.g.rec[q];
                                                          return make_uint4(r.a.x, r.a.y, r.b.w, r.a.z);
                                                        });
  const float D = g.D;
  unsigned long long rsum = 0;  // count pass: this thread's row lengths
  uint32_t rmax = 0;            // count pass: this thread's longest row
  for (uint32_t j = j0 + threadIdx.x; j < j1; j += kBlock) {
    const uint4 ma = a.g.rec[j].a;
    if (ma.z & REC_GHOST) continue;
    const uint32_t s = ma.z & REC_SLOT;
    const uint32_t qs = a.g.rec[j].b.w;
    const float sx = __uint_as_float(ma.x), sz = __uint_as_float(ma.y);
    const CellBox B = qbox(g, sx, sz);
    uint32_t n = 0;
    uint32_t w = a.row_ptr ? a.row_ptr[s] : 0u;
    // slab output, interleaved by record: entry k of grid record j at
    // slab[(j / 64) * slab_s * 64 + k * 64 + j % 64], so the lanes of a wave (consecutive j) that find
    // their k-th neighbour together store into one 256-B run
    uint32_t* const srow = a.slab && j < a.slab_recs ? a.slab + (size_t)(j >> 6) * a.slab_s * 64 + (j & 63u) : nullptr;
    auto judge = [&](uint32_t rz, uint32_t qo, float ox, float oz) {
      const uint32_t o = rz & REC_SLOT;
      if ((rz & REC_GHOST) || o == s) return;
      const bool in = (qo > qs) ? inbox(ox, oz, D, sx, sz) : inbox(sx, sz, D, ox, oz);
      if (in) {
        if (a.row_ptr) a.cols[w++] = o;
#ifndef GW_ABL_NOSLAB  // ablation (timing only): the walk without the slab stores
        if (srow && n < a.slab_s) srow[(size_t)n * 64] = o;
#endif
        ++n;
      }
    };
    if (lds && B.x0 >= cx0 && B.x1 <= cx1 && B.z0 >= cz0 && B.z1 <= cz1) {
      for (int r = B.z0; r <= B.z1; ++r) {
        const int rb = (r - cz0) * W - cx0;
        const uint32_t e = cst[rb + B.x1 + 1];
        uint32_t p = cst[rb + B.x0];
        for (; p < e; ++p) {  // (four reads per step, issued together: 167 -> 188 us, r06_a10)
          const uint4 c = rl[p];
          judge(c.w, c.z, __uint_as_float(c.x), __uint_as_float(c.y));
        }
      }
    } else {
      for (int r = B.z0; r <= B.z1; ++r) {
        row_entries_global(g, a.g.cs, r, B.x0, B.x1, [&](uint32_t k) {
          const uint4 ra = a.g.rec[k].a;
          judge(ra.z, a.g.rec[k].b.w, __uint_as_float(ra.x), __uint_as_float(ra.y));
        });
      }
    }
    if (!a.row_ptr) a.row_cnt[s] = n, rsum += n, rmax = max(rmax, (a.slab && !srow) ? a.slab_s + 1u : n);
  }
  if (!a.row_ptr) {  // the tile's totals, stored (k_rel_total sums them; the host checks the total
                     // before it sizes cols). One atomic per wave on one word instead: serialised.
    __shared__ unsigned long long rs[kBlock / 64];
    __shared__ uint32_t rm[kBlock / 64];
    for (int o = 32; o > 0; o >>= 1) rsum += __shfl_xor(rsum, o, 64);
    for (int o = 32; o > 0; o >>= 1) rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, o, 64));
    if ((threadIdx.x & 63) == 0) rs[threadIdx.x >> 6] = rsum, rm[threadIdx.x >> 6] = rmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long ts = 0;
      uint32_t tm = 0;
      for (int k = 0; k < kBlock / 64; ++k) ts += rs[k], tm = max(tm, rm[k]);
      a.tstat[t] = make_uint4((uint32_t)ts, (uint32_t)(ts >> 32), tm, 0u);
    }
  }
}

// the count pass's totals over the tiles: sum of the row lengths (64 bits) and the longest row
__global__ void __launch_bounds__(1024) k_rel_total(const uint4* __restrict__ tstat, uint32_t ntiles,
                                                    unsigned long long* total64, uint32_t* maxlen) {
  __shared__ unsigned long long ss[1024 / 64];
  __shared__ uint32_t sm_[1024 / 64];
  unsigned long long p = 0;
  uint32_t mx = 0;
  for (uint32_t i = threadIdx.x; i < ntiles; i += 1024) {
    const uint4 v = tstat[i];
    p += (unsigned long long)v.x | ((unsigned long long)v.y << 32);
    mx = max(mx, v.z);
  }
  for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o, 64), mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
  if ((threadIdx.x & 63) == 0) ss[threadIdx.x >> 6] = p, sm_[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 1024 / 64; ++k) p += ss[k], mx = max(mx, sm_[k]);
    *total64 = p;
    *maxlen = mx;
  }
}

void launch_relation(const RelArgs& a, hipStream_t st) {
  if (!a.ntiles) return;
  hipLaunchKernelGGL(k_relation, dim3(a.ntiles), dim3(kBlock), 0, st, a);
  if (!a.row_ptr)
    hipLaunchKernelGGL(k_rel_total, dim3(1), dim3(1024), 0, st, (const uint4*)a.tstat, a.ntiles, a.total64, a.maxlen);
}

// Neighbours of each row in ascending slot order. A wave takes 64 consecutive rows (a contiguous
// range of cols): each row is loaded with one coalesced load (lanes over its entries) into a per-wave
// LDS tile that holds entry k of row r at k * 65 + r (the padding makes both the row-wise writes and
// the lane-per-row reads conflict-free); each lane then sorts its row in registers with a fixed
// bitonic network (32 or 64 wide, by the wave's longest row; padded with ~0), and the rows go back
// out the way they came in. A row is a SET of slots (each entity has one main record, ghosts are
// skipped), so keys are distinct. A block holding a row longer than 64 takes the segmented sort of
// k_slice_sort (registers / wave / LDS bitonic chunks merged by rank).
// (Measured before, config 2: ranking each entry by a scan of its row in LDS, 0.43 ms; insertion
// sort in LDS, 0.88 ms; the network over unpadded LDS rows, 0.18 ms, bank conflicts.)
constexpr uint32_t kRowNetMax = 64;  // longest row sorted by the register network
constexpr int kRowPitch = 65;

template <int N>
__device__ __forceinline__ void sort_row_net(uint32_t* ww, int lane, uint32_t len) {
  uint32_t r[N];
#pragma unroll
  for (int k = 0; k < N; ++k) r[k] = (uint32_t)k < len ? ww[k * kRowPitch + lane] : 0xffffffffu;
  net_sort<N>(r);
#pragma unroll
  for (int k = 0; k < N; ++k)
    if ((uint32_t)k < len) ww[k * kRowPitch + lane] = r[k];
}

__global__ void __launch_bounds__(kBlock) k_row_sort(const uint32_t* __restrict__ row_ptr, uint32_t cap,
                                                     uint32_t* __restrict__ cols, uint32_t* __restrict__ tmp) {
  __shared__ uint32_t w[kBlock / 64][64 * kRowPitch];  // also the fallback's bitonic chunk
  __shared__ SegSmem ss;
  static_assert((kBlock / 64) * 64 * kRowPitch >= (int)kBigChunk, "fallback chunk aliases w");
  const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t b = s < cap ? row_ptr[s] : 0u, len = s < cap ? row_ptr[s + 1] - b : 0u;
  const bool long_row = __syncthreads_or(len > kRowNetMax) != 0;
  if (long_row) {  // block-uniform
    seg_sort(cols, tmp, b, len, &w[0][0], ss.bigq, &ss.nbig);
    return;
  }
  const int lane = threadIdx.x & 63;
  uint32_t* ww = w[threadIdx.x >> 6];
  for (int r = 0; r < 64; ++r) {  // row r of the wave: lanes over its entries
    const uint32_t lr = (uint32_t)__builtin_amdgcn_readlane((int)len, r);
    const uint32_t br = (uint32_t)__builtin_amdgcn_readlane((int)b, r);
    if ((uint32_t)lane < lr) ww[lane * kRowPitch + r] = cols[br + lane];
  }
  __syncthreads();
  uint32_t wmax = len;
  for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o, 64));
  if (wmax <= 32u) {  // wave-uniform
    sort_row_net<32>(ww, lane, len);
  } else if (wmax <= 48u) {
    sort_row_net<48>(ww, lane, len);
  } else {
    sort_row_net<64>(ww, lane, len);
  }
  __syncthreads();
  for (int r = 0; r < 64; ++r) {
    const uint32_t lr = (uint32_t)__builtin_amdgcn_readlane((int)len, r);
    const uint32_t br = (uint32_t)__builtin_amdgcn_readlane((int)b, r);
    if ((uint32_t)lane < lr) cols[br + lane] = ww[lane * kRowPitch + r];
  }
}

// The slab path: rows straight from the count pass's interleaved slab, in grid-record order (a wave =
// 64 consecutive records = one 64-wide column group of the slab, so entry k of all 64 rows is one
// coalesced load into lane = row registers), sorted by the register network, then out through the
// padded LDS tile one row at a time to cols[row_ptr[slot] ...]. Rows longer than 64 (every row is at
// most slab_s) are listed in fix[] and finished by k_row_fix.
template <int N>
__device__ __forceinline__ void slab_row_net(const uint32_t* __restrict__ col, uint32_t* ww, int lane, uint32_t len) {
  uint32_t r[N];
#pragma unroll
  for (int k = 0; k < N; ++k) r[k] = (uint32_t)k < len ? col[(size_t)k * 64] : 0xffffffffu;
  net_sort<N>(r);
#pragma unroll
  for (int k = 0; k < N; ++k)
    if ((uint32_t)k < len) ww[k * kRowPitch + lane] = r[k];
}

__global__ void __launch_bounds__(kBlock) k_row_sort_slab(const Rec* __restrict__ rec, const uint32_t* __restrict__ nrec_p,
                                                          const uint32_t* __restrict__ row_ptr,
                                                          const uint32_t* __restrict__ slab, uint32_t S,
                                                          uint32_t* __restrict__ cols, uint4* __restrict__ fix,
                                                          uint32_t* __restrict__ nfix) {
  __shared__ uint32_t w[kBlock / 64][64 * kRowPitch];
  const uint32_t nrec = *nrec_p;
  const uint32_t jw = blockIdx.x * kBlock + (threadIdx.x & ~63u);  // the wave's first record
  if (jw >= nrec) return;  // wave-uniform; no block barrier below
  const int lane = threadIdx.x & 63;
  const uint32_t j = jw + (uint32_t)lane;
  uint32_t b = 0, len = 0;
  if (j < nrec) {
    const uint32_t z = rec[j].a.z;
    if (!(z & REC_GHOST)) {
      const uint32_t s = z & REC_SLOT;
      b = row_ptr[s];
      len = row_ptr[s + 1] - b;
    }
  }
  if (len > kRowNetMax) {  // rare: k_row_fix
    fix[atomicAdd(nfix, 1u)] = make_uint4(b, len, j, 0u);
    len = 0;
  }
  uint32_t wmax = len;
  for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o, 64));
  uint32_t* ww = w[threadIdx.x >> 6];
  const uint32_t* col = slab + (size_t)(j >> 6) * S * 64 + (j & 63u);
  if (wmax <= 32u) {  // wave-uniform
    slab_row_net<32>(col, ww, lane, len);
  } else if (wmax <= 40u) {
    slab_row_net<40>(col, ww, lane, len);
  } else if (wmax <= 48u) {
    slab_row_net<48>(col, ww, lane, len);
  } else {
    slab_row_net<64>(col, ww, lane, len);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  for (int r = 0; r < 64; ++r) {
    const uint32_t lr = (uint32_t)__builtin_amdgcn_readlane((int)len, r);
    const uint32_t br = (uint32_t)__builtin_amdgcn_readlane((int)b, r);
    if ((uint32_t)lane < lr) cols[br + lane] = ww[lane * kRowPitch + r];
  }
}

void launch_row_sort(const uint32_t* row_ptr, uint32_t cap, uint32_t* cols, uint32_t* tmp, hipStream_t st) {
  hipLaunchKernelGGL(k_row_sort, dim3((cap + kBlock - 1) / kBlock), dim3(kBlock), 0, st, row_ptr, cap, cols, tmp);
}

// The rows k_row_sort_slab listed (longer than its network, at most slab_s <= 128): one wave per row,
// two entries per lane, each ranked by a pass over the row (keys are distinct), stored at its rank.
// A fixed grid walks the list (its length is read on the device).
__global__ void __launch_bounds__(kBlock) k_row_fix(const uint32_t* __restrict__ slab, uint32_t S,
                                                    const uint4* __restrict__ fix, const uint32_t* __restrict__ nfix,
                                                    uint32_t* __restrict__ cols) {
  const uint32_t nf = *nfix;
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (kBlock / 64);
  for (uint32_t q = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); q < nf; q += nw) {  // wave-uniform
    const uint4 f = fix[q];
    const uint32_t b = f.x, len = min(f.y, 128u);
    const uint32_t* col = slab + (size_t)(f.z >> 6) * S * 64 + (f.z & 63u);
    const uint32_t e0 = (uint32_t)lane < len ? col[(size_t)lane * 64] : 0xffffffffu;
    const uint32_t e1 = (uint32_t)lane + 64u < len ? col[(size_t)(lane + 64) * 64] : 0xffffffffu;
    uint32_t r0 = 0, r1 = 0;
    for (uint32_t t = 0; t < len; ++t) {
      const uint32_t v = t < 64u ? (uint32_t)__shfl((int)e0, (int)t, 64) : (uint32_t)__shfl((int)e1, (int)(t - 64u), 64);
      r0 += v < e0 ? 1u : 0u;
      r1 += v < e1 ? 1u : 0u;
    }
    if ((uint32_t)lane < len) cols[b + r0] = e0;
    if ((uint32_t)lane + 64u < len) cols[b + r1] = e1;
  }
}

void launch_row_sort_slab(const Rec* rec, const uint32_t* nrec, uint32_t rec_bound, const uint32_t* row_ptr,
                          const uint32_t* slab, uint32_t slab_s, uint32_t* cols, uint32_t* tmp, uint4* fix,
                          uint32_t* nfix, hipStream_t st) {
  hipLaunchKernelGGL(k_row_sort_slab, dim3((rec_bound + kBlock - 1) / kBlock), dim3(kBlock), 0, st, rec, nrec, row_ptr,
                     slab, slab_s, cols, fix, nfix);
  hipLaunchKernelGGL(k_row_fix, dim3(64), dim3(kBlock), 0, st, slab, slab_s, fix, nfix, cols);
}

// ---------------------------------------------------------------------------------------------
// Relation view, incremental: the view after a tick = the view before it + the tick's pair events
// (every pass of the tick, in ev_out). N is symmetric, so event (m, o, +-) changes rows m and o; the
// net change of (row, col) over the tick is the sum of its signs, in {-1, 0, +1} (the events are
// exactly the relation's changes, in sequence: transient enter/leave pairs cancel). Entries are
// placed by rank arithmetic: an old entry v at index i of row r goes to ns[r] + i + (sum of the signs
// of r's changes with col < v), and is dropped when the signs of col == v sum to -1; a col whose
// signs sum to +1 is written once at ns[r] + #(old entries < col) + (sum of the signs of the changes
// < col). A row with at most kRdShort changes is scanned linearly (unsorted); a longer one (a mover
// crossing a crowd) is sorted in LDS with the prefix of its signs, then searched.
constexpr uint32_t kRdShort = 32;
constexpr uint32_t kRdLongMax = 4096;  // longest change list sorted in LDS (longer: the view is rebuilt)

__global__ void __launch_bounds__(kBlock) k_rd_count(RelDeltaArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.nev) return;
  const uint2 e = a.ev[i];
  atomicAdd(&a.dn[e.x], 1u);
  atomicAdd(&a.dn[e.y & 0x7FFFFFFFu], 1u);
}

__global__ void __launch_bounds__(kBlock) k_rd_fill(RelDeltaArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.nev) return;
  const uint2 e = a.ev[i];
  const uint32_t sg = e.y & 0x80000000u, o = e.y & 0x7FFFFFFFu;
  const uint32_t p = a.dn[e.x] + atomicAdd(&a.dcur[e.x], 1u);
  a.dch[p] = o | sg;
  a.dchrow[p] = e.x;
  const uint32_t q = a.dn[o] + atomicAdd(&a.dcur[o], 1u);
  a.dch[q] = e.x | sg;
  a.dchrow[q] = o;
}

// new row lengths (rp_new, scanned by the caller; rp_new[cap] = 0); rows with many changes listed
__global__ void __launch_bounds__(kBlock) k_rd_len(RelDeltaArgs a) {
  const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
  if (r == 0) a.rp_new[a.cap] = 0u;
  if (r >= a.cap) return;
  const uint32_t cs = a.dn[r], ce = a.dn[r + 1];
  int s = 0;
  for (uint32_t k = cs; k < ce; ++k) s += (a.dch[k] >> 31) ? 1 : -1;
  if (ce - cs > kRdLongMax) {
    atomicOr(a.flag, 1u);
  } else if (ce - cs > kRdShort) {
    const uint32_t li = atomicAdd(a.nlong, 1u);  // every listed index < long_cap is written
    if (li < a.long_cap) a.longrows[li] = r;
    else atomicOr(a.flag, 1u);
  }
  a.rp_new[r] = (uint32_t)((int)(a.rp_old[r + 1] - a.rp_old[r]) + s);
}

// One block per listed row (grid-stride): its changes sorted by col in LDS (bitonic over key
// col * 2 + ENTER, padded to a power of two), written back in place, with the inclusive prefix of
// their signs in psum.
__global__ void __launch_bounds__(kBlock) k_rd_sort_long(RelDeltaArgs a) {
  __shared__ uint32_t key[kRdLongMax];
  if (*a.flag) return;  // set by k_rd_len (earlier in the stream): the update is abandoned
  const uint32_t nl = min(*a.nlong, a.long_cap);
  for (uint32_t li = blockIdx.x; li < nl; li += gridDim.x) {
    const uint32_t r = a.longrows[li];
    const uint32_t cs = a.dn[r], n = a.dn[r + 1] - cs;  // kRdShort < n <= kRdLongMax
    uint32_t np = 64;
    while (np < n) np <<= 1;
    for (uint32_t k = threadIdx.x; k < np; k += kBlock) {
      const uint32_t c = k < n ? a.dch[cs + k] : 0xFFFFFFFFu;
      key[k] = k < n ? ((c & 0x7FFFFFFFu) << 1) | (c >> 31) : 0xFFFFFFFFu;
    }
    __syncthreads();
    for (uint32_t size = 2; size <= np; size <<= 1) {
      for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
        for (uint32_t k = threadIdx.x; k < np; k += kBlock) {
          const uint32_t l = k ^ stride;
          if (l > k) {
            const uint32_t x = key[k], y = key[l];
            const bool up = (k & size) == 0;
            if ((x > y) == up) {
              key[k] = y;
              key[l] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    // inclusive prefix of the signs: kRdLongMax / kBlock consecutive entries per thread
    constexpr uint32_t kPer = kRdLongMax / kBlock;
    const uint32_t k0 = threadIdx.x * kPer;
    int loc = 0;
    for (uint32_t q = 0; q < kPer; ++q)
      if (k0 + q < n) loc += (key[k0 + q] & 1u) ? 1 : -1;
    uint32_t total;
    int run = (int)block_excl_scan((uint32_t)loc, &total);
    for (uint32_t q = 0; q < kPer; ++q) {
      const uint32_t k = k0 + q;
      if (k < n) {
        const uint32_t kk = key[k];
        run += (kk & 1u) ? 1 : -1;
        a.dch[cs + k] = (kk >> 1) | (kk << 31);
        a.psum[cs + k] = run;
      }
    }
    __syncthreads();  // key[] is reused by the next row
  }
}

// sorted change list [cs, ce) of a long row: (sum of signs of cols < v, sum of signs of cols == v)
__device__ __forceinline__ int2 rd_long_sums(const RelDeltaArgs& a, uint32_t cs, uint32_t ce, uint32_t v) {
  uint32_t lo = cs, hi = ce;
  while (lo < hi) {  // first col >= v
    const uint32_t mid = (lo + hi) >> 1;
    if ((a.dch[mid] & 0x7FFFFFFFu) < v) lo = mid + 1;
    else hi = mid;
  }
  uint32_t lo2 = lo, hi2 = ce;
  while (lo2 < hi2) {  // first col > v
    const uint32_t mid = (lo2 + hi2) >> 1;
    if ((a.dch[mid] & 0x7FFFFFFFu) <= v) lo2 = mid + 1;
    else hi2 = mid;
  }
  const int below = lo > cs ? a.psum[lo - 1] : 0;
  const int upto = lo2 > cs ? a.psum[lo2 - 1] : 0;
  return make_int2(below, upto - below);
}

// Old entries to their new places: a wave takes 64 consecutive rows (one contiguous range of the old
// cols, ~2,080 entries at config 2) and walks it 64 entries at a time; each lane finds its entry's row
// among the few rows the chunk touches (a wave-uniform loop over readlanes). The group's old entries
// are loaded into registers first (one chunk per register, every load in flight at once) and its
// change lists (one contiguous range of dch, ~42 changes, with the sign prefixes of long rows) into
// the wave's LDS: the walk then reads no global memory and its stores never wait (gfx9 counts stores
// and loads on one vmcnt, so a global load in the walk waits for every store before it: 121 us at
// config 2 that way; staging the entries in LDS instead cost occupancy, 145 us).
template <bool B>
struct BoolTag {
  static constexpr bool value = B;
};
constexpr uint32_t kRdWaveCh = 256;    // changes of a 64-row group staged in LDS (+ their sign prefixes)
// staged sorted list of a long row, indices relative to the group: (signs < v, signs == v)
__device__ __forceinline__ int2 rd_long_sums_lds(const uint32_t* ch, const int32_t* ps, uint32_t cs, uint32_t ce,
                                                 uint32_t v) {
  uint32_t lo = cs, hi = ce;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((ch[mid] & 0x7FFFFFFFu) < v) lo = mid + 1;
    else hi = mid;
  }
  uint32_t lo2 = lo, hi2 = ce;
  while (lo2 < hi2) {
    const uint32_t mid = (lo2 + hi2) >> 1;
    if ((ch[mid] & 0x7FFFFFFFu) <= v) lo2 = mid + 1;
    else hi2 = mid;
  }
  const int below = lo > cs ? ps[lo - 1] : 0;
  const int upto = lo2 > cs ? ps[lo2 - 1] : 0;
  return make_int2(below, upto - below);
}

constexpr int kRdRegChunks = 36;  // chunks of a group held in registers (config 2: 33 +- 1)
// staged groups: each entry's row (0..63) in a per-wave LDS map, written by the rows' lanes, instead of a walk
// over the rows each chunk touches (readlanes per row and chunk)
#ifndef GW_RD_ROWMAP
#define GW_RD_ROWMAP 1
#endif
// diagnosis only (A/B of where k_rd_merge's time goes; the view is then wrong): 1 skips the row search
#ifndef GW_DIAG_MERGE
#define GW_DIAG_MERGE 0
#endif
__global__ void __launch_bounds__(kBlock) k_rd_merge(RelDeltaArgs a) {
  __shared__ uint32_t chs_all[kBlock / 64][kRdWaveCh];
  __shared__ int32_t pss_all[kBlock / 64][kRdWaveCh];
  __shared__ uint8_t rid_all[kBlock / 64][GW_RD_ROWMAP ? kRdRegChunks * 64 : 1];
  const int lane = threadIdx.x & 63;
  uint32_t* chs = chs_all[threadIdx.x >> 6];
  int32_t* pss = pss_all[threadIdx.x >> 6];
  uint8_t* rid = rid_all[threadIdx.x >> 6];
  const uint32_t r0 = ((blockIdx.x * kBlock + threadIdx.x) >> 6) * 64u;
  if (r0 >= a.cap || *a.flag) return;  // wave-uniform
  const uint32_t nr = min(64u, a.cap - r0);
  uint32_t os = 0, ns = 0, cs = 0, ce = 0;
  if ((uint32_t)lane < nr) {
    const uint32_t r = r0 + lane;
    os = a.rp_old[r];
    ns = a.rp_new[r];
    cs = a.dn[r];
    ce = a.dn[r + 1];
  }
  const uint32_t G0 = __builtin_amdgcn_readfirstlane(os);
  const uint32_t G1 = __builtin_amdgcn_readfirstlane(a.rp_old[r0 + nr]);
  const uint32_t C0 = __builtin_amdgcn_readfirstlane(cs);
  const uint32_t C1 = __builtin_amdgcn_readfirstlane(a.dn[r0 + nr]);
  // registers: the group's old entries, all loads issued at once, one chunk per register
  const bool staged = C1 - C0 <= kRdWaveCh && G1 - G0 <= (uint32_t)kRdRegChunks * 64u;  // wave-uniform
  uint32_t L0 = 0;  // first row the chunk touches (wave-uniform)
  // one chunk: entries b + lane (value v); the row of each among the rows the chunk touches, its
  // offset from the row's changes, the store
  auto chunk = [&](uint32_t b, uint32_t v, auto tag) {
    constexpr bool kStaged = decltype(tag)::value;
    const uint32_t e = b + lane;
    const bool act = e < G1;
    const uint32_t cend = min(b + 64u, G1);
    uint32_t ri = L0, mos = 0, mns = 0, mcs = 0, mce = 0;
    if (kStaged && GW_RD_ROWMAP) {  // the entry's row from the wave's LDS map, its bounds from that row's lane
      ri = act ? (uint32_t)rid[e - G0] : 0u;
      mos = (uint32_t)__shfl((int)os, (int)ri, 64);
      mns = (uint32_t)__shfl((int)ns, (int)ri, 64);
      mcs = (uint32_t)__shfl((int)cs, (int)ri, 64);
      mce = (uint32_t)__shfl((int)ce, (int)ri, 64);
    }
    for (uint32_t L = L0; L < ((GW_DIAG_MERGE == 1 || (kStaged && GW_RD_ROWMAP)) ? 0u : nr); ++L) {
      const uint32_t osL = __builtin_amdgcn_readlane(os, L);
      if (osL >= cend) break;  // wave-uniform
      const uint32_t nsL = __builtin_amdgcn_readlane(ns, L), csL = __builtin_amdgcn_readlane(cs, L),
                     ceL = __builtin_amdgcn_readlane(ce, L);
      const bool in = e >= osL;  // the last such row holds e (an empty row shares its start with the next)
      ri = in ? L : ri;
      mos = in ? osL : mos;
      mns = in ? nsL : mns;
      mcs = in ? csL : mcs;
      mce = in ? ceL : mce;
    }
    if (act) {
      int sl = 0, se = 0;
      auto scan = [&](uint32_t c) {
        const uint32_t col = c & 0x7FFFFFFFu;
        const int sg = (c >> 31) ? 1 : -1;
        sl += col < v ? sg : 0;
        se += col == v ? sg : 0;
      };
      if (kStaged && mce - mcs <= kRdShort) {
        for (uint32_t k = mcs - C0; k < mce - C0; ++k) scan(chs[k]);
      } else if (kStaged) {  // a long (sorted) row of a staged group (<= kRdWaveCh changes)
        const int2 ss = rd_long_sums_lds(chs, pss, mcs - C0, mce - C0, v);
        sl = ss.x;
        se = ss.y;
      } else if (mce - mcs <= kRdShort) {
        for (uint32_t k = mcs; k < mce; ++k) scan(a.dch[k]);
      } else if (mce - mcs <= kRdLongMax) {  // a long (sorted) row: binary searches in global memory
        const int2 ss = rd_long_sums(a, mcs, mce, v);
        sl = ss.x;
        se = ss.y;
      }
      const uint32_t o = mns + (e - mos) + (uint32_t)sl;
      if (se >= 0 && o < a.cols_cap) a.cols_new[o] = v;  // (the bound holds for a consistent event stream)
    }
    L0 = __builtin_amdgcn_readlane(ri, 63);
  };
  if (staged) {
    uint32_t vv[kRdRegChunks];
#pragma unroll
    for (int i = 0; i < kRdRegChunks; ++i) {
      const uint32_t e = G0 + (uint32_t)i * 64u + lane;
      vv[i] = e < G1 ? a.cols_old[e] : 0u;
    }
    for (uint32_t k = lane; k < C1 - C0; k += 64) chs[k] = a.dch[C0 + k];
    for (uint32_t k = lane; k < C1 - C0; k += 64) pss[k] = a.psum[C0 + k];  // (meaningful for long rows)
    if (GW_RD_ROWMAP) {  // row L's entries [os, next row's os) -> L
      const uint32_t nxt = (uint32_t)__shfl_down((int)os, 1, 64);
      const uint32_t oe = (uint32_t)lane + 1u < nr ? nxt : G1;
      if ((uint32_t)lane < nr)
        for (uint32_t k = os - G0; k < oe - G0; ++k) rid[k] = (uint8_t)lane;
    }
    // every load complete before the first store: the walk's uses of vv then wait on nothing (a wait
    // for one of them after stores were issued would be vmcnt(0), i.e. for the stores too)
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < kRdRegChunks; ++i) {
      const uint32_t b = G0 + (uint32_t)i * 64u;
      if (b >= G1) break;  // wave-uniform
      chunk(b, vv[i], BoolTag<true>{});
    }
  } else {
    for (uint32_t b = G0; b < G1; b += 64) chunk(b, b + lane < G1 ? a.cols_old[b + lane] : 0u, BoolTag<false>{});
  }
}

// New entries: one thread per change. A short row's col is written by its first ENTER change, a long
// (sorted) row's by the first change of its run of equal cols, when its signs sum to +1.
__global__ void __launch_bounds__(kBlock) k_rd_adds(RelDeltaArgs a) {
  const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
  if (j >= 2u * a.nev || *a.flag) return;
  const uint32_t c = a.dch[j];
  const uint32_t r = a.dchrow[j], col = c & 0x7FFFFFFFu;
  const uint32_t cs = a.dn[r], ce = a.dn[r + 1];
  int sl = 0, se = 0;
  if (ce - cs <= kRdShort) {
    if (!(c >> 31)) return;
    bool first = true;
    for (uint32_t k = cs; k < ce; ++k) {
      const uint32_t c2 = a.dch[k], col2 = c2 & 0x7FFFFFFFu;
      const int sg = (c2 >> 31) ? 1 : -1;
      sl += col2 < col ? sg : 0;
      se += col2 == col ? sg : 0;
      first = first && !(col2 == col && (c2 >> 31) && k < j);
    }
    if (!first) return;
  } else {
    if (ce - cs > kRdLongMax) return;  // flagged by k_rd_len
    if (j > cs && (a.dch[j - 1] & 0x7FFFFFFFu) == col) return;
    const int2 ss = rd_long_sums(a, cs, ce, col);
    sl = ss.x;
    se = ss.y;
  }
  if (se <= 0) return;
  uint32_t lo = a.rp_old[r], hi = a.rp_old[r + 1];
  const uint32_t os = lo;
  while (lo < hi) {  // old entries < col
    const uint32_t mid = (lo + hi) >> 1;
    if (a.cols_old[mid] < col) lo = mid + 1;
    else hi = mid;
  }
  const uint32_t o = a.rp_new[r] + (lo - os) + (uint32_t)sl;
  if (o < a.cols_cap) a.cols_new[o] = col;
}

void launch_rel_delta_count(const RelDeltaArgs& a, hipStream_t st) {
  const uint32_t nb = (a.nev + kBlock - 1) / kBlock;
  if (nb) hipLaunchKernelGGL(k_rd_count, dim3(nb), dim3(kBlock), 0, st, a);
}

void launch_rel_delta_apply(const RelDeltaArgs& a, ScanCtx& sc, hipStream_t st) {
  // dn holds the scanned change offsets on entry
  const uint32_t nb = (a.nev + kBlock - 1) / kBlock;
  if (nb) hipLaunchKernelGGL(k_rd_fill, dim3(nb), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(k_rd_len, dim3((a.cap + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(k_rd_sort_long, dim3(512), dim3(kBlock), 0, st, a);
  launch_scan(sc, a.rp_new, a.cap + 1, st);
  const uint32_t waves = (a.cap + 63) / 64;
  hipLaunchKernelGGL(k_rd_merge, dim3((waves + kBlock / 64 - 1) / (kBlock / 64)), dim3(kBlock), 0, st, a);
  const uint32_t nb2 = (2 * a.nev + kBlock - 1) / kBlock;
  if (nb2) hipLaunchKernelGGL(k_rd_adds, dim3(nb2), dim3(kBlock), 0, st, a);
}

// ---------------------------------------------------------------------------------------------
// Relation delta export (gwaoi_export_relation_delta): the NET changes of the relation over the last
// tick, from its events alone, O(events) with no sort. A pair's events alternate ENTER / LEAVE in
// sequence, so the pair changed iff it has an odd number of events, and the kind of its LAST event is
// the change. Pairs are grouped through an open-addressing hash table keyed by the unordered pair
// (min, max); per slot: the event count and the largest event index. The event that is its pair's
// last one, with an odd count, emits the change in both directions, at its place in event order
// (flags -> scan -> emit), so the output is deterministic.
__device__ __forceinline__ uint32_t dx_hash(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (uint32_t)k;
}

__global__ void __launch_bounds__(kBlock) k_dx_insert(DeltaExportArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.nev) return;
  const uint2 e = a.ev[i];
  const uint32_t m = e.x, o = e.y & 0x7FFFFFFFu;
  const unsigned long long key = (unsigned long long)min(m, o) << 32 | max(m, o);
  uint32_t h = dx_hash(key) & a.mask;
  for (;;) {  // the table has at least 2 x nev slots: a free one is always found
    const unsigned long long prev = atomicCAS(&a.keys[h], ~0ull, key);
    if (prev == ~0ull || prev == key) break;
    h = (h + 1) & a.mask;
  }
  atomicAdd(&a.cnt[h], 1u);
  atomicMax(&a.last[h], i);
  a.slot_of[i] = h;
}

__global__ void __launch_bounds__(kBlock) k_dx_flag(DeltaExportArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i == 0) a.flags[a.nev] = 0u;  // the scan's total
  if (i >= a.nev) return;
  const uint32_t h = a.slot_of[i];
  a.flags[i] = ((a.cnt[h] & 1u) && a.last[h] == i) ? 1u : 0u;
}

__global__ void __launch_bounds__(kBlock) k_dx_emit(DeltaExportArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.nev) return;
  const uint32_t p = a.flags[i];
  if (a.flags[i + 1] == p) return;  // not kept (flags scanned: kept iff the offset steps)
  const uint2 e = a.ev[i];
  const uint32_t m = e.x, o = e.y & 0x7FFFFFFFu, sg = e.y & 0x80000000u;
  a.out[2 * p] = make_uint2(m, o | sg);
  a.out[2 * p + 1] = make_uint2(o, m | sg);
}

void launch_delta_export(const DeltaExportArgs& a, ScanCtx& sc, hipStream_t st) {
  const uint32_t nb = (a.nev + kBlock - 1) / kBlock;
  if (!nb) return;
  hipLaunchKernelGGL(k_dx_insert, dim3(nb), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(k_dx_flag, dim3(nb), dim3(kBlock), 0, st, a);
  launch_scan(sc, a.flags, a.nev + 1, st);
  hipLaunchKernelGGL(k_dx_emit, dim3(nb), dim3(kBlock), 0, st, a);
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

// several Spaces of n_per entities each (slot = space * n_per + i, seed of a Space = seed0 + space);
// nhot > 0: the skewed crowd placement of config 5
__global__ void __launch_bounds__(kBlock) k_wl_init_spaces(float* x, float* z, uint32_t n_per, uint32_t nspaces,
                                                           uint64_t seed0, float L, uint32_t nhot, float sigma,
                                                           uint32_t hot_every) {
  const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= (uint64_t)n_per * nspaces) return;
  const uint32_t sp = (uint32_t)(k / n_per), i = (uint32_t)(k - (uint64_t)sp * n_per);
  x[k] = gww_skew_init_coord(seed0 + sp, n_per, i, 0, L, nhot, sigma, hot_every);
  z[k] = gww_skew_init_coord(seed0 + sp, n_per, i, 1, L, nhot, sigma, hot_every);
}

__global__ void __launch_bounds__(kBlock) k_wl_step_spaces(const float* xp, const float* zp, float* xo, float* zo,
                                                           uint32_t n_per, uint32_t nspaces, uint64_t seed0,
                                                           uint64_t tick, float L, float s) {
  const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= (uint64_t)n_per * nspaces) return;
  const uint32_t sp = (uint32_t)(k / n_per), i = (uint32_t)(k - (uint64_t)sp * n_per);
  const float x = gww_step_coord(xp[k], seed0 + sp, tick, n_per, i, 0, L, s);
  const float z = gww_step_coord(zp[k], seed0 + sp, tick, n_per, i, 1, L, s);
  xo[k] = x;
  zo[k] = z;
}

void launch_wl_init_spaces(float* x, float* z, uint32_t n_per, uint32_t nspaces, uint64_t seed0, float L,
                           uint32_t nhot, float sigma, uint32_t hot_every, hipStream_t st) {
  const uint64_t n = (uint64_t)n_per * nspaces;
  if (n)
    hipLaunchKernelGGL(k_wl_init_spaces, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, x, z, n_per,
                       nspaces, seed0, L, nhot, sigma, hot_every);
}

void launch_wl_step_spaces(const float* xp, const float* zp, float* xo, float* zo, uint32_t n_per, uint32_t nspaces,
                           uint64_t seed0, uint64_t tick, float L, float s, hipStream_t st) {
  const uint64_t n = (uint64_t)n_per * nspaces;
  if (n)
    hipLaunchKernelGGL(k_wl_step_spaces, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, xp, zp, xo,
                       zo, n_per, nspaces, seed0, tick, L, s);
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

// ---------------------------------------------------------------------------------------------
// Pinned host staging (gwaoi_stage_moves_pinned): the cgo wrapper writes one tick's Moved calls into
// library-owned pinned arrays; after one DMA copy the GPU validates the batch (what gwaoi_stage_moves
// did on one host thread) and finds where a slot repeats (the sub-pass rule of host staging). Neither
// kernel changes the manager's state, so a refused batch leaves it untouched (all-or-nothing).
//   first[s] (64 bit, never reset): max over this call's ops naming s of (id << 32 | ~i), so the
//   first op naming s in call `id` is ~low32 when high32 == id.
__device__ __forceinline__ uint32_t ord_key(float f) {  // order-preserving float -> uint32
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__global__ void __launch_bounds__(kBlock) k_pin_check(PinCheckArgs a) {
  const uint32_t i = a.seg + blockIdx.x * kBlock + threadIdx.x;
  uint32_t err = 0, bad = 0xFFFFFFFFu;
  bool out_ext = false;
  if (i < a.n) {
    const uint32_t s = a.slot[i];
    const float x = a.x[i], z = a.z[i];
    if (s >= a.cap) {
      err |= ERR_BAD_SLOT;
    } else {
      if (a.validate && a.seq[s] == 0u) err |= ERR_ABSENT_SLOT;
      atomicMax(&a.first[s], (unsigned long long)a.id << 32 | (unsigned long long)(~i));
      if (a.ext) {  // auto-extent Spaces: coordinates beyond the current grid extent (rare) are reported
        const uint32_t sp = a.space_of[s];
        const float4 e = a.ext[sp];
        if (!(x >= e.x && x <= e.z && z >= e.y && z <= e.w) && finite_bits(__float_as_uint(x)) &&
            finite_bits(__float_as_uint(z))) {
          out_ext = true;
          atomicMin(&a.seen[4 * sp + 0], ord_key(x));
          atomicMin(&a.seen[4 * sp + 1], ord_key(z));
          atomicMax(&a.seen[4 * sp + 2], ord_key(x));
          atomicMax(&a.seen[4 * sp + 3], ord_key(z));
        }
      }
    }
    if (a.validate && !(finite_bits(__float_as_uint(x)) && finite_bits(__float_as_uint(z)))) err |= ERR_BAD_COORD;
    if (err) bad = i;
  }
  for (int o = 32; o > 0; o >>= 1) {
    err |= (uint32_t)__shfl_xor(err, o, 64);
    bad = min(bad, (uint32_t)__shfl_xor(bad, o, 64));
  }
  const bool anyx = __any(out_ext);
  if ((threadIdx.x & 63) == 0) {
    if (err) {
      atomicOr(&a.out[0], err);
      atomicMin(&a.out[2], bad);
    }
    if (anyx) atomicOr(&a.out[3], 1u);
  }
}

__global__ void __launch_bounds__(kBlock) k_pin_cut(PinCheckArgs a) {
  const uint32_t i = a.seg + blockIdx.x * kBlock + threadIdx.x;
  uint32_t c = 0xFFFFFFFFu;
  if (i < a.n) {
    const uint32_t s = a.slot[i];
    if (s < a.cap) {
      const unsigned long long v = a.first[s];
      if ((uint32_t)(v >> 32) == a.id && ~(uint32_t)v != i) c = i;
    }
  }
  for (int o = 32; o > 0; o >>= 1) c = min(c, (uint32_t)__shfl_xor(c, o, 64));
  if ((threadIdx.x & 63) == 0 && c != 0xFFFFFFFFu) atomicMin(&a.out[1], c);
}

__global__ void k_pin_init(uint32_t* out, uint32_t n, uint32_t* seen, uint32_t nseen) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) {
    out[0] = 0u;
    out[1] = n;
    out[2] = 0xFFFFFFFFu;
    out[3] = 0u;
  }
  if (seen && t < nseen) seen[t] = (t & 2u) ? 0u : 0xFFFFFFFFu;  // [min x, min z, max x, max z] per Space
}

void launch_pin_check(const PinCheckArgs& a, bool reset_seen, uint32_t nspaces, hipStream_t st) {
  const uint32_t nseen = reset_seen && a.seen ? 4u * nspaces : 0u;
  hipLaunchKernelGGL(k_pin_init, dim3((std::max(nseen, 1u) + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a.out, a.n,
                     nseen ? a.seen : (uint32_t*)nullptr, nseen);
  const uint32_t m = a.n - a.seg;
  if (!m) return;
  hipLaunchKernelGGL(k_pin_check, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(k_pin_cut, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, st, a);
}

// One thread, after k_pin_check / k_pin_cut: the sub-pass's op count for the device-counted batch (the
// apply kernels read it), and the check's words for the host, read after the pass's end-of-pass sync.
__global__ void k_pin_count(const uint32_t* out, uint32_t n, uint32_t seg, int validate, uint32_t* n_dev,
                            uint32_t* host_out) {
  if (threadIdx.x != 0) return;
  const uint32_t err = validate ? out[0] : 0u;
  const uint32_t cut = min(out[1], n);
  *n_dev = err ? 0u : cut - seg;
  host_out[0] = out[0];
  host_out[1] = out[1];
  host_out[2] = out[2];
  host_out[3] = out[3];
}

void launch_pin_count(const uint32_t* out, uint32_t n, uint32_t seg, int validate, uint32_t* n_dev,
                      uint32_t* host_out, hipStream_t st) {
  hipLaunchKernelGGL(k_pin_count, dim3(1), dim3(64), 0, st, out, n, seg, validate, n_dev, host_out);
}

float ord_float(uint32_t k) {  // inverse of ord_key (host)
  const uint32_t b = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  float f;
  std::memcpy(&f, &b, 4);
  return f;
}

}  // namespace gw
