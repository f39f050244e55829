// gwaoi_strips.hip — per-GPU kernels of the X-strip partition (include/gwaoi_strips.h; host side in
// goworld_amd/strips.py). State is indexed by global entity id; every pass is a flat, coalesced sweep
// over the n ids or over a received record list. The id-ordered op list is a stream compaction
// (block counts -> scan -> block-local scan and write), so the manager sees the global op order.
#include <hip/hip_runtime.h>

#include "gwaoi.h"
#include "gwaoi_internal.h"
#include "gwaoi_strips.h"
#include "gwaoi_workload.h"

namespace gw {
namespace {

constexpr int kSBlock = 256;
constexpr int kSItems = 16;  // ids per thread in the compaction (one uint4 of flags)
constexpr uint32_t kSChunk = kSBlock * kSItems;

__device__ __forceinline__ bool in_range(float x, float lo, float hi) { return x >= lo && x < hi; }

// one atomic per wave for the lanes with `pred`; returns this lane's slot
__device__ __forceinline__ uint32_t wave_append_s(uint32_t* ctr, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (!m) return 0u;
  const int leader = __ffsll((long long)m) - 1;
  const int lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

__device__ __forceinline__ uint32_t block_scan_s(uint32_t v, uint32_t* total) {
  __shared__ uint32_t ws[kSBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kSBlock / 64; ++k) {
    pre += k < w ? ws[k] : 0u;
    tot += ws[k];
  }
  __syncthreads();
  *total = tot;
  return pre + inc - v;
}

__global__ void __launch_bounds__(kSBlock) k_strip_init_walk(gwaoi_strip_geom g, uint8_t* flags, float* ex, float* ez,
                                                             uint64_t seed, float L) {
  const uint32_t i = blockIdx.x * kSBlock + threadIdx.x;
  if (i >= g.n) return;
  const float x = gww_init_coord(seed, g.n, i, 0, L), z = gww_init_coord(seed, g.n, i, 1, L);
  uint8_t f = 0;
  if (in_range(x, g.ra, g.rb)) {
    f |= GWAOI_STRIP_END;
    ex[i] = x;
    ez[i] = z;
  }
  if (in_range(x, g.xa, g.xb)) f |= GWAOI_STRIP_OWNED;
  flags[i] = f;
}

__global__ void __launch_bounds__(kSBlock) k_strip_init_skew(gwaoi_strip_geom g, uint8_t* flags, float* ex, float* ez,
                                                             uint64_t seed, float L, uint32_t nhot, float sigma,
                                                             uint32_t hot_every) {
  const uint32_t i = blockIdx.x * kSBlock + threadIdx.x;
  if (i >= g.n) return;
  const float x = gww_skew_init_coord(seed, g.n, i, 0, L, nhot, sigma, hot_every);
  const float z = gww_skew_init_coord(seed, g.n, i, 1, L, nhot, sigma, hot_every);
  uint8_t f = 0;
  if (in_range(x, g.ra, g.rb)) {
    f |= GWAOI_STRIP_END;
    ex[i] = x;
    ez[i] = z;
  }
  if (in_range(x, g.xa, g.xb)) f |= GWAOI_STRIP_OWNED;
  flags[i] = f;
}

// n state entries; l2g (region state, ABI 2.1): entry k is local slot k, its global id l2g[k] (else: id k)
__global__ void __launch_bounds__(kSBlock) k_strip_walk(gwaoi_strip_geom g, uint8_t* flags, const float* sx,
                                                        const float* sz, float* ex, float* ez, uint64_t seed,
                                                        uint64_t tick, float L, float step, uint32_t* err, uint32_t n,
                                                        const uint32_t* l2g) {
  const uint32_t k = blockIdx.x * kSBlock + threadIdx.x;
  if (k >= n) return;
  const uint8_t f = flags[k];
  if (!(f & GWAOI_STRIP_OWNED)) return;
  const uint32_t i = l2g ? l2g[k] : k;
  const float x0 = sx[k];
  const float x = gww_step_coord(x0, seed, tick, g.n, i, 0, L, step);
  const float z = gww_step_coord(sz[k], seed, tick, g.n, i, 1, L, step);
  if (!(fabsf(x - x0) <= g.max_step)) atomicOr(err, GWAOI_STRIP_ERR_STEP);
  ex[k] = x;
  ez[k] = z;
  flags[k] = f | GWAOI_STRIP_END;
}

// g2l (region state): the state is indexed by local slot g2l[id]
__global__ void __launch_bounds__(kSBlock) k_strip_ingest(gwaoi_strip_geom g, uint8_t* flags, const float* sx,
                                                          float* ex, float* ez, const uint32_t* ids,
                                                          const float* xs, const float* zs, uint32_t n,
                                                          uint32_t* err, const uint32_t* g2l) {
  const uint32_t k = blockIdx.x * kSBlock + threadIdx.x;
  if (k >= n) return;
  const uint32_t id = ids[k];
  const uint32_t i = id < g.n ? (g2l ? g2l[id] : id) : GWAOI_STRIP_NO_SLOT;
  if (i == GWAOI_STRIP_NO_SLOT || !(flags[i] & GWAOI_STRIP_OWNED)) {
    atomicOr(err, GWAOI_STRIP_ERR_NOT_OWNED);
    return;
  }
  const float x = xs[k];
  if (!(fabsf(x - sx[i]) <= g.max_step)) atomicOr(err, GWAOI_STRIP_ERR_STEP);
  ex[i] = x;
  ez[i] = zs[k];
  flags[i] |= GWAOI_STRIP_END;
}

// One block per kSelChunk ids, kSelItems rounds of one id per thread (coalesced flag reads); a
// thread remembers its selected rounds in two bit masks, the block scans the per-thread counts and
// reserves its range of each list with ONE atomic per list, then writes. (One wave-aggregated atomic
// per wave with a selection serialised on the two counters when the world's ids are spread over many
// strips: 270 us for a 16M-id world at 8 strips.)
// Rounds per block (items): enough blocks to fill the device (~1k: 2M ids -> 8 rounds; a 16M-id world at
// most 64), so a small world is not walked by two blocks per CU (64 rounds at 2M ids: 122 blocks, 40 us).
constexpr int kSelItems = 64;  // at most (one bit per round in two 64-bit masks)
inline uint32_t sel_items(uint32_t n) {
  const uint32_t want = (n + 1024u * kSBlock - 1) / (1024u * kSBlock);
  return want < 4 ? 4u : want > (uint32_t)kSelItems ? (uint32_t)kSelItems : want;
}
// n state entries; l2g (region state, ABI 2.1): entry k is local slot k, the record carries its id l2g[k]
__global__ void __launch_bounds__(kSBlock) k_strip_select(gwaoi_strip_geom g, const uint8_t* flags, const float* sx,
                                                          const float* ex, const float* ez, uint4* left,
                                                          uint4* right, uint32_t cap, uint32_t* counts,
                                                          uint32_t* err, uint32_t items, uint32_t n,
                                                          const uint32_t* l2g) {
  __shared__ uint32_t base_sh[2];
  const uint32_t c0 = blockIdx.x * kSBlock * items + threadIdx.x;
  unsigned long long ml = 0, mr = 0;
#pragma unroll 4
  for (int r = 0; r < (int)items; ++r) {
    const uint32_t i = c0 + (uint32_t)r * kSBlock;
    if (i >= n) break;
    const uint8_t f = flags[i];
    if ((f & GWAOI_STRIP_OWNED) && (f & GWAOI_STRIP_END)) {
      const float x0 = sx[i], x1 = ex[i];
      if (g.has_left && (x0 < g.left_hi || x1 < g.left_hi)) ml |= 1ull << r;
      if (g.has_right && (x0 >= g.right_lo || x1 >= g.right_lo)) mr |= 1ull << r;
    }
  }
  uint32_t totl, totr;
  uint32_t pl = block_scan_s((uint32_t)__popcll(ml), &totl);
  uint32_t pr = block_scan_s((uint32_t)__popcll(mr), &totr);
  if (threadIdx.x == 0) {
    base_sh[0] = totl ? atomicAdd(&counts[0], totl) : 0u;
    base_sh[1] = totr ? atomicAdd(&counts[1], totr) : 0u;
  }
  __syncthreads();
  pl += base_sh[0];
  pr += base_sh[1];
  unsigned long long m = ml | mr;
  while (m) {
    const int r = __ffsll((long long)m) - 1;
    m &= m - 1ull;
    const uint32_t i = c0 + (uint32_t)r * kSBlock;
    const uint4 rec = make_uint4(l2g ? l2g[i] : i, __float_as_uint(ex[i]), __float_as_uint(ez[i]), 0u);
    if ((ml >> r) & 1ull) {
      if (pl < cap) left[pl] = rec;
      else atomicOr(err, GWAOI_STRIP_ERR_OVERFLOW);
      ++pl;
    }
    if ((mr >> r) & 1ull) {
      if (pr < cap) right[pr] = rec;
      else atomicOr(err, GWAOI_STRIP_ERR_OVERFLOW);
      ++pr;
    }
  }
}

__global__ void __launch_bounds__(kSBlock) k_strip_absorb(uint8_t* flags, float* ex, float* ez, const uint4* recs,
                                                          uint32_t n, const uint32_t* d_n, uint32_t* err) {
  const uint32_t k = blockIdx.x * kSBlock + threadIdx.x;
  if (d_n) {  // received count (device): the launch covers the message's capacity
    const uint32_t got = *d_n;
    // a sender past its capacity kept counting: the list was cut, so this rank's AOI would miss halo
    // entities. The sender flags its own overflow; the receiver fails its protocol check as well.
    if (got > n && k == 0 && err) atomicOr(err, GWAOI_STRIP_ERR_OVERFLOW);
    n = min(n, got);
  }
  if (k >= n) return;
  const uint4 r = recs[k];
  ex[r.x] = __uint_as_float(r.y);
  ez[r.x] = __uint_as_float(r.z);
  flags[r.x] |= GWAOI_STRIP_END;
}

// 16 flags of thread `t` of block `b` (ids b * kSChunk + t * 16 ...), zero beyond n
__device__ __forceinline__ void load_flags16(const uint8_t* flags, uint32_t n, uint32_t i0, uint8_t (&f)[kSItems]) {
  if (i0 + kSItems <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(flags + i0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < kSItems; ++k) f[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  } else {
#pragma unroll
    for (int k = 0; k < kSItems; ++k) f[k] = (i0 + k < n) ? flags[i0 + k] : (uint8_t)0;
  }
}

__device__ __forceinline__ bool has_op(uint8_t f) { return (f & (GWAOI_STRIP_PRESENT | GWAOI_STRIP_END)) != 0; }

__device__ __forceinline__ bool is_enter(uint8_t f) { return (f & (GWAOI_STRIP_PRESENT | GWAOI_STRIP_END)) == GWAOI_STRIP_END; }

// ops per chunk (blk) and, for local slots, the tick's Enter count (enters: one atomic per block)
__global__ void __launch_bounds__(kSBlock) k_strip_count(const uint8_t* flags, uint32_t n, uint32_t* blk,
                                                         uint32_t* enters) {
  uint8_t f[kSItems];
  load_flags16(flags, n, blockIdx.x * kSChunk + threadIdx.x * kSItems, f);
  uint32_t c = 0, ce = 0;
#pragma unroll
  for (int k = 0; k < kSItems; ++k) {
    c += has_op(f[k]) ? 1u : 0u;
    ce += is_enter(f[k]) ? 1u : 0u;
  }
  uint32_t tot, tote = 0;
  block_scan_s(c, &tot);
  if (enters) block_scan_s(ce, &tote);  // grid-uniform branch
  if (threadIdx.x == 0) {
    blk[blockIdx.x] = tot;
    if (tote) atomicAdd(enters, tote);
  }
}

// One block per chunk of kSChunk ids (the chunk's op count scanned beforehand by k_strip_count), in
// kSItems rounds of one id per thread: every load and store of a round covers consecutive ids or
// consecutive op slots (a ballot ranks a wave's ops, four wave totals in LDS place the waves).
// (Sixteen consecutive ids per thread made every access a 16-element stride: 137 us at 2M ids.)
__global__ void __launch_bounds__(kSBlock) k_strip_emit(gwaoi_strip_geom g, uint8_t* flags, float* sx, float* sz,
                                                        const float* ex, const float* ez, const uint32_t* blk,
                                                        uint32_t* ids, float* ox, float* oz, uint8_t* kinds) {
  __shared__ uint32_t wsum[2][kSBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  uint32_t pos = blk[blockIdx.x];
#pragma unroll 1
  for (int r = 0; r < kSItems; ++r) {
    const uint32_t i = blockIdx.x * kSChunk + (uint32_t)r * kSBlock + threadIdx.x;
    const uint8_t f = i < g.n ? flags[i] : (uint8_t)0;
    const bool op = has_op(f);
    const unsigned long long m = __ballot(op);
    if (lane == 0) wsum[r & 1][w] = (uint32_t)__popcll(m);
    __syncthreads();  // one barrier per round: the two wsum buffers alternate
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kSBlock / 64; ++k) {
      const uint32_t v = wsum[r & 1][k];
      off += k < w ? v : 0u;
      tot += v;
    }
    if (op) {
      const uint32_t q = pos + off + (uint32_t)__popcll(m & below);
      const bool p = f & GWAOI_STRIP_PRESENT, e = f & GWAOI_STRIP_END;
      uint8_t kind = p ? (e ? GWAOI_OP_MOVE : GWAOI_OP_LEAVE) : GWAOI_OP_ENTER;
      if (!(f & GWAOI_STRIP_OWNED)) kind |= GWAOI_OP_SILENT;
      float x = 0.f, z = 0.f;
      uint8_t nf = 0;
      if (e) {
        x = ex[i];
        z = ez[i];
        sx[i] = x;
        sz[i] = z;
        nf = GWAOI_STRIP_PRESENT | (in_range(x, g.xa, g.xb) ? GWAOI_STRIP_OWNED : 0);
      }
      ids[q] = i;
      ox[q] = x;
      oz[q] = z;
      kinds[q] = kind;
      flags[i] = nf;
    } else if (i < g.n && f) {
      flags[i] = 0;
    }
    pos += tot;
  }
}

// ---- local slots ----
__global__ void __launch_bounds__(kSBlock) k_local_init(uint32_t n, uint32_t cap_l, uint32_t* g2l, uint32_t* fq,
                                                        uint32_t* ctr) {
  const uint32_t i = blockIdx.x * kSBlock + threadIdx.x;
  if (i < n) g2l[i] = GWAOI_STRIP_NO_SLOT;
  if (i < cap_l) fq[i] = i;
  if (i == 0) {
    ctr[0] = 0u;
    ctr[1] = cap_l;
    ctr[2] = 0u;
    ctr[3] = 0u;
  }
}

// the previous tick's Leave slots back into the free ring (one block; the count is on the device).
// sc[0] = free slots after the release (what this tick's Enters may take), sc[1] = 0 (k_strip_count
// adds the tick's Enters there).
__global__ void __launch_bounds__(1024) k_local_release(uint32_t* fq, const uint32_t* pend, uint32_t mask, uint32_t* ctr,
                                                        uint32_t* sc) {
  const uint32_t np = ctr[2], tail = ctr[1];
  for (uint32_t k = threadIdx.x; k < np; k += 1024) fq[(tail + k) & mask] = pend[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    ctr[1] = tail + np;
    ctr[2] = 0u;
    sc[0] = tail + np - ctr[0];
    sc[1] = 0u;
  }
}

// k_strip_emit, with the manager's slot of each op mapped: an Enter takes the next free slot of the
// ring, a Move keeps its slot, a Leave queues its slot in pend (released at the next emit).
__global__ void __launch_bounds__(kSBlock) k_strip_emit_local(gwaoi_strip_geom g, uint8_t* flags, float* sx, float* sz,
                                                              const float* ex, const float* ez, const uint32_t* blk,
                                                              uint32_t* slots, float* ox, float* oz, uint8_t* kinds,
                                                              uint32_t* g2l, uint32_t* l2g, const uint32_t* fq,
                                                              uint32_t* pend, uint32_t mask, uint32_t* ctr,
                                                              const uint32_t* sc, uint32_t nb, uint32_t* n_ops) {
  __shared__ uint32_t wsum[2][kSBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  const uint32_t tail = ctr[1];  // releases happened before this kernel; allocations must stay below
  // More Enters than free slots (a crowd drifting into the region past cap_l): the tick emits NOTHING
  // (zero ops, state not advanced), so the manager runs an empty pass and stays usable, and the error
  // bit names the cause. Decided from counts complete before this kernel (grid-uniform).
  const bool fits = sc[1] <= sc[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *n_ops = fits ? blk[nb] : 0u;
    if (!fits) atomicOr(&ctr[3], GWAOI_STRIP_ERR_SLOTS);
  }
  if (!fits) return;
  uint32_t pos = blk[blockIdx.x];
#pragma unroll 1
  for (int r = 0; r < kSItems; ++r) {
    const uint32_t i = blockIdx.x * kSChunk + (uint32_t)r * kSBlock + threadIdx.x;
    const uint8_t f = i < g.n ? flags[i] : (uint8_t)0;
    const bool op = has_op(f);
    const bool p = f & GWAOI_STRIP_PRESENT, e = f & GWAOI_STRIP_END;
    const unsigned long long m = __ballot(op);
    if (lane == 0) wsum[r & 1][w] = (uint32_t)__popcll(m);
    const uint32_t ka = wave_append_s(&ctr[0], op && !p);        // Enter: allocation index
    const uint32_t kl = wave_append_s(&ctr[2], op && p && !e);   // Leave: pending index
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kSBlock / 64; ++k) {
      const uint32_t v = wsum[r & 1][k];
      off += k < w ? v : 0u;
      tot += v;
    }
    if (op) {
      const uint32_t q = pos + off + (uint32_t)__popcll(m & below);
      uint8_t kind = p ? (e ? GWAOI_OP_MOVE : GWAOI_OP_LEAVE) : GWAOI_OP_ENTER;
      if (!(f & GWAOI_STRIP_OWNED)) kind |= GWAOI_OP_SILENT;
      uint32_t l;
      if (!p) {
        if ((int)(tail - ka) <= 0) {  // ring empty (excluded by the check above; kept as a guard)
          atomicOr(&ctr[3], GWAOI_STRIP_ERR_SLOTS);
          l = 0u;
        } else {
          l = fq[ka & mask];
          g2l[i] = l;
          l2g[l] = i;
        }
      } else {
        l = g2l[i];
        if (!e) {
          pend[kl] = l;
          g2l[i] = GWAOI_STRIP_NO_SLOT;
        }
      }
      float x = 0.f, z = 0.f;
      uint8_t nf = 0;
      if (e) {
        x = ex[i];
        z = ez[i];
        sx[i] = x;
        sz[i] = z;
        nf = GWAOI_STRIP_PRESENT | (in_range(x, g.xa, g.xb) ? GWAOI_STRIP_OWNED : 0);
      }
      slots[q] = l;
      ox[q] = x;
      oz[q] = z;
      kinds[q] = kind;
      flags[i] = nf;
    } else if (i < g.n && f) {
      flags[i] = 0;
    }
    pos += tot;
  }
}

__global__ void __launch_bounds__(kSBlock) k_translate(const uint32_t* l2g, uint32_t* ev, uint32_t n) {
  const uint32_t k = blockIdx.x * kSBlock + threadIdx.x;
  if (k >= n) return;
  const uint32_t m = ev[2 * k], o = ev[2 * k + 1];
  ev[2 * k] = l2g[m];
  ev[2 * k + 1] = l2g[o & 0x7FFFFFFFu] | (o & 0x80000000u);
}

// ---- region state (ABI 2.1): the strip's state in local-slot order, the region list in id order ----
// Region counters (gwaoi_strip_region.ctr), by list buffer p (R->cur: the list the tick starts from): [p] its
// length (Leaves included, as tombstones), [2 + p] the new ids appended to it this tick (absorb), [4 + p] its
// tombstones (the Leaves the emit that wrote it appended), [6] GWAOI_STRIP_ERR_* bits. Each emit writes only
// the other buffer's counters and the prep zeroes them beforehand, so no kernel has to move the counters on
// after the emit's last block (a per-block ticket with a device-scope fence, 10k blocks: 290 us, r06_a7).
constexpr uint32_t kRsSortMax = 16384;  // one block's LDS sort (the chunk)
constexpr uint32_t kRsChunks = 8;       // chunks of new ids (and of Leaves) per tick at most

// first index of a[0, n) (ascending) not below v
__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* a, uint32_t n, uint32_t v) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// entries below v in a[0, n), sorted ascending within each chunk
__device__ __forceinline__ uint32_t count_below(const uint32_t* a, uint32_t n, uint32_t chunk, uint32_t v) {
  uint32_t c = 0;
  for (uint32_t c0 = 0; c0 < n; c0 += chunk) c += lower_bound_u32(a + c0, min(chunk, n - c0), v);
  return c;
}
// list entries (ids with the tombstone bit) below id v
__device__ __forceinline__ uint32_t list_below(const uint32_t* rl, uint32_t n, uint32_t v) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((rl[mid] & ~GWAOI_STRIP_TOMB) < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

struct RsDev {  // the device side of gwaoi_strip_region (the list buffers resolved: cur / next)
  uint8_t* flags;
  float *sx, *sz, *ex, *ez;
  uint32_t *g2l, *l2g, *fq, *pend, *lctr;
  uint32_t *rl, *rs, *rl_next, *rs_next;
  uint32_t *nw, *lv, *srt, *ctr;
  uint32_t cap_l, cap_new, chunk, mask, p;  // p: the current list buffer (R->cur)
};

// the region's entities of tick 0, in id order, into slots 0, 1, ... (k_strip_count + scan beforehand)
__global__ void __launch_bounds__(kSBlock) k_rs_start(gwaoi_strip_geom g, RsDev R, const uint8_t* gflags,
                                                      const float* gex, const float* gez, const uint32_t* blk,
                                                      uint32_t nb, uint32_t* slots, float* ox, float* oz,
                                                      uint8_t* kinds, uint32_t* n_ops) {
  __shared__ uint32_t wsum[2][kSBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  const uint32_t m = blk[nb];
  const bool fits = m <= R.cap_l;  // grid-uniform
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *n_ops = fits ? m : 0u;
    if (!fits) {
      atomicOr(&R.lctr[3], GWAOI_STRIP_ERR_SLOTS);
    } else {
      R.lctr[0] = m;  // the ring's first m slots (0 .. m-1) taken
      R.ctr[R.p] = m;
    }
  }
  if (!fits) return;
  uint32_t pos = blk[blockIdx.x];
#pragma unroll 1
  for (int r = 0; r < kSItems; ++r) {
    const uint32_t i = blockIdx.x * kSChunk + (uint32_t)r * kSBlock + threadIdx.x;
    const uint8_t f = i < g.n ? gflags[i] : (uint8_t)0;
    const bool op = (f & GWAOI_STRIP_END) != 0;
    const unsigned long long mk = __ballot(op);
    if (lane == 0) wsum[r & 1][w] = (uint32_t)__popcll(mk);
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kSBlock / 64; ++k) {
      const uint32_t v = wsum[r & 1][k];
      off += k < w ? v : 0u;
      tot += v;
    }
    if (op) {
      const uint32_t q = pos + off + (uint32_t)__popcll(mk & below), l = q;
      const float x = gex[i], z = gez[i];
      R.g2l[i] = l;
      R.l2g[l] = i;
      R.flags[l] = GWAOI_STRIP_PRESENT | (in_range(x, g.xa, g.xb) ? GWAOI_STRIP_OWNED : 0);
      R.sx[l] = x;
      R.sz[l] = z;
      R.rl[q] = i;
      R.rs[q] = l;
      slots[q] = l;
      ox[q] = x;
      oz[q] = z;
      kinds[q] = GWAOI_OP_ENTER | ((f & GWAOI_STRIP_OWNED) ? 0 : GWAOI_OP_SILENT);
    }
    pos += tot;
  }
}

// received records into the slot state; an id new to the region takes a free slot and is appended to the
// tick's new ids (nw: ids, then their slots at nw + cap_new). Two messages in one launch (both neighbours'):
// threads [0, na) take message a, the rest message b; a count in device memory (d_n*) clamps its message.
__global__ void __launch_bounds__(kSBlock) k_rs_absorb(RsDev R, const uint4* recs_a, uint32_t na, const uint32_t* d_na,
                                                       const uint4* recs_b, uint32_t nb, const uint32_t* d_nb,
                                                       uint32_t* err) {
  const uint32_t t = blockIdx.x * kSBlock + threadIdx.x;
  if (t == 0 && err) {  // a sender past its capacity kept counting: its list was cut (the receiver fails too)
    if ((d_na && *d_na > na) || (d_nb && *d_nb > nb)) atomicOr(err, GWAOI_STRIP_ERR_OVERFLOW);
  }
  const bool second = t >= na;
  const uint32_t k = second ? t - na : t;
  const uint32_t* d_n = second ? d_nb : d_na;
  uint32_t n = second ? nb : na;
  if (d_n) n = min(n, *d_n);
  const uint32_t tail = R.lctr[1];  // (releases run in the emit, after every absorb of the tick)
  uint4 r = make_uint4(0u, 0u, 0u, 0u);
  uint32_t l = GWAOI_STRIP_NO_SLOT;
  if (k < n) {
    r = (second ? recs_b : recs_a)[k];
    l = R.g2l[r.x];
  }  const bool fresh = k < n && l == GWAOI_STRIP_NO_SLOT;
  const uint32_t ka = wave_append_s(&R.lctr[0], fresh);
  const bool got_slot = fresh && (int)(tail - ka) > 0;
  if (fresh && !got_slot) atomicOr(&R.lctr[3], GWAOI_STRIP_ERR_SLOTS);
  const uint32_t j = wave_append_s(&R.ctr[2 + R.p], got_slot);
  if (k >= n || (fresh && !got_slot)) return;
  if (got_slot) {
    l = R.fq[ka & R.mask];
    R.g2l[r.x] = l;
    R.l2g[l] = r.x;
    R.flags[l] = GWAOI_STRIP_END;
    if (j < R.cap_new) {
      R.nw[j] = r.x;
      R.nw[R.cap_new + j] = l;
    } else {
      atomicOr(&R.ctr[6], GWAOI_STRIP_ERR_NEWLIST);
    }
  } else {
    R.flags[l] |= GWAOI_STRIP_END;
  }
  R.ex[l] = __uint_as_float(r.y);
  R.ez[l] = __uint_as_float(r.z);
}

// Before the emit, one launch: blocks [0, kRsChunks) sort the tick's new ids by chunk (ids into srt, their
// slots carried to srt + cap_new), blocks [kRsChunks, 2 kRsChunks) the last emit's Leave positions (into
// srt + 2 cap_new), block 2 kRsChunks returns the last emit's Leave slots to the free ring.
__global__ void __launch_bounds__(1024) k_rs_prep(RsDev R) {
  __shared__ uint32_t sk[kRsSortMax];
  const uint32_t M = R.ctr[2 + R.p], T = R.ctr[4 + R.p];
  if (blockIdx.x == 2 * kRsChunks) {
    const uint32_t np = R.lctr[2], tail = R.lctr[1];
    for (uint32_t k = threadIdx.x; k < np; k += 1024) R.fq[(tail + k) & R.mask] = R.pend[k];
    __syncthreads();
    if (threadIdx.x == 0) {
      R.lctr[1] = tail + np;
      R.lctr[2] = 0u;
      R.ctr[4 + (R.p ^ 1u)] = 0u;  // the emit appends the tick's Leaves there
      if (M > R.cap_new || T > R.cap_new) atomicOr(&R.ctr[6], GWAOI_STRIP_ERR_NEWLIST);
    }
    return;
  }
  const bool leaves = blockIdx.x >= kRsChunks;
  const uint32_t cnt = min(leaves ? T : M, R.cap_new);
  const uint32_t c0 = (blockIdx.x - (leaves ? kRsChunks : 0u)) * R.chunk;
  if (c0 >= cnt) return;
  const uint32_t len = min(R.chunk, cnt - c0);
  const uint32_t* src = (leaves ? R.lv : R.nw) + c0;
  uint32_t* dst = R.srt + (leaves ? 2u * R.cap_new : 0u) + c0;
  uint32_t P = 64;
  while (P < len) P <<= 1;
  for (uint32_t i = threadIdx.x; i < P; i += 1024) sk[i] = i < len ? src[i] : 0xFFFFFFFFu;
  __syncthreads();
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += 1024) {
        const uint32_t o = i ^ j;
        if (o > i) {
          const uint32_t u = sk[i], v = sk[o];
          if ((u > v) == ((i & k) == 0)) sk[i] = v, sk[o] = u;
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = threadIdx.x; i < len; i += 1024) dst[i] = sk[i];
  if (!leaves)  // each new id's slot to its sorted place (ids are distinct)
    for (uint32_t i = threadIdx.x; i < len; i += 1024) dst[R.cap_new + lower_bound_u32(sk, len, src[i])] = src[R.cap_new + i];
}

// The op list: thread t < N takes list entry t (a tombstone: nothing; else Moved or Leave), thread N + k the
// k-th sorted new id (Enter). An op's place in id order = its entries below it in the other input, less the
// tombstones below it in the list (binary searches of the sorted new ids and Leave positions, a few hundred
// per tick). The next list is the op list itself: ids and slots at the op's place, the Leaves as tombstones
// (their places noted in lv for the next emit).
__global__ void __launch_bounds__(kSBlock) k_rs_emit(gwaoi_strip_geom g, RsDev R, uint32_t* slots, float* ox, float* oz,
                                                     uint8_t* kinds, uint32_t* n_ops) {
  const uint32_t t = blockIdx.x * kSBlock + threadIdx.x;
  const uint32_t N = R.ctr[R.p], M = R.ctr[2 + R.p], T = R.ctr[4 + R.p];
  const bool bad = R.ctr[6] != 0u || R.lctr[3] != 0u;  // grid-uniform (set before this launch)
  if (t == 0) {
    *n_ops = bad ? 0u : N - T + M;
    R.ctr[R.p ^ 1u] = N - T + M;  // the next list's length; no new ids yet
    R.ctr[2 + (R.p ^ 1u)] = 0u;
  }
  const uint32_t* snw = R.srt;
  const uint32_t* slv = R.srt + 2u * R.cap_new;
  bool live = false, fresh = false;
  uint32_t id = 0, l = 0, q = 0;
  uint8_t f = 0;
  if (!bad && t < N) {
    const uint32_t v = R.rl[t];
    if (!(v & GWAOI_STRIP_TOMB)) {
      live = true;
      id = v;
      l = R.rs[t];
      q = t - count_below(slv, T, R.chunk, t) + count_below(snw, M, R.chunk, id);
    }
  } else if (!bad && t < N + M) {
    fresh = true;
    id = snw[t - N];
    l = snw[R.cap_new + (t - N)];
    const uint32_t p = list_below(R.rl, N, id);
    q = count_below(snw, M, R.chunk, id) + p - count_below(slv, T, R.chunk, p);
  }
  if (live || fresh) f = R.flags[l];
  const bool leave = live && !(f & GWAOI_STRIP_END);
  const uint32_t kl = wave_append_s(&R.lctr[2], leave);  // the slot back to the ring at the next emit
  const uint32_t jl = wave_append_s(&R.ctr[4 + (R.p ^ 1u)], leave);  // the tombstone's place, for the next emit
  if (live || fresh) {
    uint8_t kind = fresh ? GWAOI_OP_ENTER : (leave ? GWAOI_OP_LEAVE : GWAOI_OP_MOVE);
    if (!(f & GWAOI_STRIP_OWNED)) kind |= GWAOI_OP_SILENT;
    float x = 0.f, z = 0.f;
    if (!leave) {
      x = R.ex[l];
      z = R.ez[l];
      R.sx[l] = x;
      R.sz[l] = z;
      R.flags[l] = GWAOI_STRIP_PRESENT | (in_range(x, g.xa, g.xb) ? GWAOI_STRIP_OWNED : 0);
      R.rl_next[q] = id;
    } else {
      R.pend[kl] = l;
      R.g2l[id] = GWAOI_STRIP_NO_SLOT;
      R.flags[l] = 0;
      R.rl_next[q] = id | GWAOI_STRIP_TOMB;
      if (jl < R.cap_new) R.lv[jl] = q;
      else atomicOr(&R.ctr[6], GWAOI_STRIP_ERR_NEWLIST);
    }
    R.rs_next[q] = l;
    slots[q] = l;
    ox[q] = x;
    oz[q] = z;
    kinds[q] = kind;
  }
}

inline dim3 blocks_for(uint32_t n) { return dim3((n + kSBlock - 1) / kSBlock); }
// the free-slot ring of cap_l local slots: the next power of two entries (index mask)
inline uint32_t ring_mask(uint32_t cap_l) {
  uint32_t r = 1;
  while (r < cap_l) r <<= 1;
  return r - 1;
}
inline uint32_t emit_blocks(uint32_t n) { return (n + kSChunk - 1) / kSChunk; }

}  // namespace
}  // namespace gw

extern "C" {

int gwaoi_strip_init_walk(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, float* ex, float* ez, uint64_t seed,
                          float L) {
  if (!g || !flags || !ex || !ez) return GWAOI_ERR_INVALID;
  if (g->n)
    hipLaunchKernelGGL(gw::k_strip_init_walk, gw::blocks_for(g->n), dim3(gw::kSBlock), 0, (hipStream_t)stream, *g,
                       flags, ex, ez, seed, L);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_walk(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, const float* sx, const float* sz,
                     float* ex, float* ez, uint64_t seed, uint64_t tick, float L, float step, uint32_t* d_err) {
  if (!g || !flags || !sx || !sz || !ex || !ez || !d_err) return GWAOI_ERR_INVALID;
  if (g->n)
    hipLaunchKernelGGL(gw::k_strip_walk, gw::blocks_for(g->n), dim3(gw::kSBlock), 0, (hipStream_t)stream, *g, flags,
                       sx, sz, ex, ez, seed, tick, L, step, d_err, g->n, (const uint32_t*)nullptr);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_ingest(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, const float* sx, float* ex, float* ez,
                       const uint32_t* d_ids, const float* d_x, const float* d_z, uint32_t n, uint32_t* d_err) {
  if (!g || !flags || !sx || !ex || !ez || !d_err || (n && (!d_ids || !d_x || !d_z))) return GWAOI_ERR_INVALID;
  if (n)
    hipLaunchKernelGGL(gw::k_strip_ingest, gw::blocks_for(n), dim3(gw::kSBlock), 0, (hipStream_t)stream, *g, flags,
                       sx, ex, ez, d_ids, d_x, d_z, n, d_err, (const uint32_t*)nullptr);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_select(void* stream, const gwaoi_strip_geom* g, const uint8_t* flags, const float* sx, const float* ex,
                       const float* ez, uint32_t* d_left, uint32_t* d_right, uint32_t cap, uint32_t* d_counts,
                       uint32_t* d_err) {
  if (!g || !flags || !sx || !ex || !ez || !d_left || !d_right || !d_counts || !d_err) return GWAOI_ERR_INVALID;
  if (hipMemsetAsync(d_counts, 0, 2 * sizeof(uint32_t), (hipStream_t)stream) != hipSuccess) return GWAOI_ERR_HIP;
  if (g->n) {
    const uint32_t items = gw::sel_items(g->n), chunk = gw::kSBlock * items;
    hipLaunchKernelGGL(gw::k_strip_select, dim3((g->n + chunk - 1) / chunk), dim3(gw::kSBlock), 0, (hipStream_t)stream,
                       *g, flags, sx, ex, ez, reinterpret_cast<uint4*>(d_left), reinterpret_cast<uint4*>(d_right), cap,
                       d_counts, d_err, items, g->n, (const uint32_t*)nullptr);
  }
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_absorb(void* stream, uint8_t* flags, float* ex, float* ez, const uint32_t* d_recs, uint32_t n) {
  if (!flags || !ex || !ez || (n && !d_recs)) return GWAOI_ERR_INVALID;
  if (n)
    hipLaunchKernelGGL(gw::k_strip_absorb, gw::blocks_for(n), dim3(gw::kSBlock), 0, (hipStream_t)stream, flags, ex, ez,
                       reinterpret_cast<const uint4*>(d_recs), n, (const uint32_t*)nullptr, (uint32_t*)nullptr);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_absorb_n(void* stream, uint8_t* flags, float* ex, float* ez, const uint32_t* d_recs, const uint32_t* d_n,
                         uint32_t n_max, uint32_t* d_err) {
  if (!flags || !ex || !ez || !d_n || (n_max && !d_recs)) return GWAOI_ERR_INVALID;
  // one block at least: the overflow check runs even for a zero-capacity message
  hipLaunchKernelGGL(gw::k_strip_absorb, gw::blocks_for(n_max ? n_max : 1u), dim3(gw::kSBlock), 0, (hipStream_t)stream,
                     flags, ex, ez, reinterpret_cast<const uint4*>(d_recs), n_max, d_n, d_err);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_init_skew(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, float* ex, float* ez, uint64_t seed,
                          float L, uint32_t nhot, float sigma, uint32_t hot_every) {
  if (!g || !flags || !ex || !ez) return GWAOI_ERR_INVALID;
  if (g->n)
    hipLaunchKernelGGL(gw::k_strip_init_skew, gw::blocks_for(g->n), dim3(gw::kSBlock), 0, (hipStream_t)stream, *g,
                       flags, ex, ez, seed, L, nhot, sigma, hot_every);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

size_t gwaoi_strip_scratch_words(uint32_t n) {
  const uint32_t nb = gw::emit_blocks(n);
  return (size_t)nb + 1 + gw::scan_part_words(nb + 1) + 4;
}

int gwaoi_strip_emit(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, float* sx, float* sz, const float* ex,
                     const float* ez, uint32_t* d_ids, float* d_x, float* d_z, uint8_t* d_kinds, uint32_t* d_scratch,
                     uint32_t* d_n_ops) {
  if (!g || !flags || !sx || !sz || !ex || !ez || !d_ids || !d_x || !d_z || !d_kinds || !d_scratch || !d_n_ops)
    return GWAOI_ERR_INVALID;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t nb = gw::emit_blocks(g->n);
  uint32_t* blk = d_scratch;  // [nb + 1]
  gw::ScanCtx sc;
  sc.status = d_scratch + nb + 1;
  if (hipMemsetAsync(blk + nb, 0, sizeof(uint32_t), st) != hipSuccess) return GWAOI_ERR_HIP;
  if (nb) {
    hipLaunchKernelGGL(gw::k_strip_count, dim3(nb), dim3(gw::kSBlock), 0, st, flags, g->n, blk, (uint32_t*)nullptr);
    gw::launch_scan(sc, blk, nb + 1, st);
    hipLaunchKernelGGL(gw::k_strip_emit, dim3(nb), dim3(gw::kSBlock), 0, st, *g, flags, sx, sz, ex, ez,
                       (const uint32_t*)blk, d_ids, d_x, d_z, d_kinds);
  }
  if (hipMemcpyAsync(d_n_ops, blk + nb, sizeof(uint32_t), hipMemcpyDeviceToDevice, st) != hipSuccess)
    return GWAOI_ERR_HIP;
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_local_init(void* stream, uint32_t n, uint32_t cap_l, uint32_t* g2l, uint32_t* fq, uint32_t* ctr) {
  if (!g2l || !fq || !ctr || !cap_l || cap_l > 0x80000000u) return GWAOI_ERR_INVALID;
  const uint32_t m = n > cap_l ? n : cap_l;
  hipLaunchKernelGGL(gw::k_local_init, gw::blocks_for(m), dim3(gw::kSBlock), 0, (hipStream_t)stream, n, cap_l, g2l, fq,
                     ctr);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_emit_local(void* stream, const gwaoi_strip_geom* g, uint8_t* flags, float* sx, float* sz,
                           const float* ex, const float* ez, uint32_t* d_slots, float* d_x, float* d_z,
                           uint8_t* d_kinds, uint32_t* d_scratch, uint32_t* d_n_ops, uint32_t* g2l, uint32_t* l2g,
                           uint32_t* fq, uint32_t* pend, uint32_t cap_l, uint32_t* ctr) {
  if (!g || !flags || !sx || !sz || !ex || !ez || !d_slots || !d_x || !d_z || !d_kinds || !d_scratch || !d_n_ops ||
      !g2l || !l2g || !fq || !pend || !ctr || !cap_l || cap_l > 0x80000000u)
    return GWAOI_ERR_INVALID;
  const uint32_t mask = gw::ring_mask(cap_l);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t nb = gw::emit_blocks(g->n);
  uint32_t* blk = d_scratch;  // [nb + 1]
  gw::ScanCtx sc;
  sc.status = d_scratch + nb + 1;
  if (hipMemsetAsync(blk + nb, 0, sizeof(uint32_t), st) != hipSuccess) return GWAOI_ERR_HIP;
  uint32_t* spare = d_scratch + nb + 1 + gw::scan_part_words(nb + 1);  // 4 words (gwaoi_strip_scratch_words)
  hipLaunchKernelGGL(gw::k_local_release, dim3(1), dim3(1024), 0, st, fq, (const uint32_t*)pend, mask, ctr, spare);
  if (nb) {
    hipLaunchKernelGGL(gw::k_strip_count, dim3(nb), dim3(gw::kSBlock), 0, st, flags, g->n, blk, spare + 1);
    gw::launch_scan(sc, blk, nb + 1, st);
    // writes *d_n_ops (0 when the Enters do not fit the free slots)
    hipLaunchKernelGGL(gw::k_strip_emit_local, dim3(nb), dim3(gw::kSBlock), 0, st, *g, flags, sx, sz, ex, ez,
                       (const uint32_t*)blk, d_slots, d_x, d_z, d_kinds, g2l, l2g, (const uint32_t*)fq, pend,
                       mask, ctr, (const uint32_t*)spare, nb, d_n_ops);
  } else if (hipMemsetAsync(d_n_ops, 0, sizeof(uint32_t), st) != hipSuccess) {
    return GWAOI_ERR_HIP;
  }
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

// ---- region state (ABI 2.1) ----
static bool region_ok(const gwaoi_strip_region* R) {
  if (!R || !R->flags || !R->sx || !R->sz || !R->ex || !R->ez || !R->g2l || !R->l2g || !R->fq || !R->pend || !R->lctr ||
      !R->rl[0] || !R->rl[1] || !R->rs[0] || !R->rs[1] || !R->nw || !R->lv || !R->srt || !R->ctr || !R->cap_l ||
      R->cap_l > 0x7fffffffu || !R->cap_new || R->cur > 1)
    return false;
  const uint32_t ch = R->chunk ? R->chunk : gw::kRsSortMax;
  return ch >= 16 && ch <= gw::kRsSortMax && !(ch & (ch - 1)) && R->cap_new <= gw::kRsChunks * ch;
}

static gw::RsDev region_dev(const gwaoi_strip_region* R) {
  gw::RsDev d;
  d.flags = R->flags;
  d.sx = R->sx;
  d.sz = R->sz;
  d.ex = R->ex;
  d.ez = R->ez;
  d.g2l = R->g2l;
  d.l2g = R->l2g;
  d.fq = R->fq;
  d.pend = R->pend;
  d.lctr = R->lctr;
  d.rl = R->rl[R->cur];
  d.rs = R->rs[R->cur];
  d.rl_next = R->rl[R->cur ^ 1u];
  d.rs_next = R->rs[R->cur ^ 1u];
  d.nw = R->nw;
  d.lv = R->lv;
  d.srt = R->srt;
  d.ctr = R->ctr;
  d.cap_l = R->cap_l;
  d.cap_new = R->cap_new;
  d.chunk = R->chunk ? R->chunk : gw::kRsSortMax;
  d.mask = gw::ring_mask(R->cap_l);
  d.p = R->cur;
  return d;
}

int gwaoi_strip_region_init(void* stream, gwaoi_strip_region* R) {
  if (!region_ok(R) || R->n > 0x7fffffffu) return GWAOI_ERR_INVALID;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(R->flags, 0, R->cap_l, st) != hipSuccess ||
      hipMemsetAsync(R->ctr, 0, 8 * sizeof(uint32_t), st) != hipSuccess)
    return GWAOI_ERR_HIP;
  R->cur = 0;
  return gwaoi_strip_local_init(stream, R->n, R->cap_l, R->g2l, R->fq, R->lctr);
}

int gwaoi_strip_region_start(void* stream, const gwaoi_strip_geom* g, gwaoi_strip_region* R, const uint8_t* flags,
                             const float* ex, const float* ez, uint32_t* d_slots, float* d_x, float* d_z,
                             uint8_t* d_kinds, uint32_t* d_n_ops) {
  if (!g || !region_ok(R) || !R->scratch || g->n != R->n || !flags || !ex || !ez || !d_slots || !d_x || !d_z ||
      !d_kinds || !d_n_ops)
    return GWAOI_ERR_INVALID;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t nb = gw::emit_blocks(g->n);
  uint32_t* blk = R->scratch;  // [nb + 1]
  gw::ScanCtx sc;
  sc.status = R->scratch + nb + 1;
  if (hipMemsetAsync(blk + nb, 0, sizeof(uint32_t), st) != hipSuccess) return GWAOI_ERR_HIP;
  if (nb) {
    hipLaunchKernelGGL(gw::k_strip_count, dim3(nb), dim3(gw::kSBlock), 0, st, flags, g->n, blk, (uint32_t*)nullptr);
    gw::launch_scan(sc, blk, nb + 1, st);
  }
  hipLaunchKernelGGL(gw::k_rs_start, dim3(nb ? nb : 1u), dim3(gw::kSBlock), 0, st, *g, region_dev(R), flags, ex, ez,
                     (const uint32_t*)blk, nb, d_slots, d_x, d_z, d_kinds, d_n_ops);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_region_walk(void* stream, const gwaoi_strip_geom* g, const gwaoi_strip_region* R, uint64_t seed,
                            uint64_t tick, float Lw, float step, uint32_t* d_err) {
  if (!g || !region_ok(R) || !d_err) return GWAOI_ERR_INVALID;
  hipLaunchKernelGGL(gw::k_strip_walk, gw::blocks_for(R->cap_l), dim3(gw::kSBlock), 0, (hipStream_t)stream, *g,
                     R->flags, (const float*)R->sx, (const float*)R->sz, R->ex, R->ez, seed, tick, Lw, step, d_err,
                     R->cap_l, (const uint32_t*)R->l2g);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_region_ingest(void* stream, const gwaoi_strip_geom* g, const gwaoi_strip_region* R,
                              const uint32_t* d_ids, const float* d_x, const float* d_z, uint32_t n, uint32_t* d_err) {
  if (!g || !region_ok(R) || !d_err || (n && (!d_ids || !d_x || !d_z))) return GWAOI_ERR_INVALID;
  if (n)
    hipLaunchKernelGGL(gw::k_strip_ingest, gw::blocks_for(n), dim3(gw::kSBlock), 0, (hipStream_t)stream, *g, R->flags,
                       (const float*)R->sx, R->ex, R->ez, d_ids, d_x, d_z, n, d_err, (const uint32_t*)R->g2l);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_region_select(void* stream, const gwaoi_strip_geom* g, const gwaoi_strip_region* R, uint32_t* d_left,
                              uint32_t* d_right, uint32_t cap, uint32_t* d_counts, uint32_t* d_err) {
  if (!g || !region_ok(R) || !d_left || !d_right || !d_counts || !d_err) return GWAOI_ERR_INVALID;
  if (hipMemsetAsync(d_counts, 0, 2 * sizeof(uint32_t), (hipStream_t)stream) != hipSuccess) return GWAOI_ERR_HIP;
  const uint32_t items = gw::sel_items(R->cap_l), chunk = gw::kSBlock * items;
  hipLaunchKernelGGL(gw::k_strip_select, dim3((R->cap_l + chunk - 1) / chunk), dim3(gw::kSBlock), 0,
                     (hipStream_t)stream, *g, (const uint8_t*)R->flags, (const float*)R->sx, (const float*)R->ex,
                     (const float*)R->ez, reinterpret_cast<uint4*>(d_left), reinterpret_cast<uint4*>(d_right), cap,
                     d_counts, d_err, items, R->cap_l, (const uint32_t*)R->l2g);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_region_absorb(void* stream, const gwaoi_strip_region* R, const uint32_t* d_recs, const uint32_t* d_n,
                              uint32_t n_max, uint32_t* d_err) {
  return gwaoi_strip_region_absorb2(stream, R, d_recs, d_n, n_max, nullptr, nullptr, 0u, d_err);
}

int gwaoi_strip_region_absorb2(void* stream, const gwaoi_strip_region* R, const uint32_t* d_left, const uint32_t* d_nl,
                               uint32_t nl_max, const uint32_t* d_right, const uint32_t* d_nr, uint32_t nr_max,
                               uint32_t* d_err) {
  if (!region_ok(R) || (nl_max && !d_left) || (nr_max && !d_right) || nl_max > 0x7fffffffu || nr_max > 0x7fffffffu)
    return GWAOI_ERR_INVALID;
  // one block at least: a count check runs even for zero-capacity messages
  const uint32_t tot = nl_max + nr_max;
  hipLaunchKernelGGL(gw::k_rs_absorb, gw::blocks_for(tot ? tot : 1u), dim3(gw::kSBlock), 0, (hipStream_t)stream,
                     region_dev(R), reinterpret_cast<const uint4*>(d_left), nl_max, d_nl,
                     reinterpret_cast<const uint4*>(d_right), nr_max, d_nr, d_err);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

int gwaoi_strip_region_emit(void* stream, const gwaoi_strip_geom* g, gwaoi_strip_region* R, uint32_t* d_slots,
                            float* d_x, float* d_z, uint8_t* d_kinds, uint32_t* d_n_ops) {
  if (!g || !region_ok(R) || !d_slots || !d_x || !d_z || !d_kinds || !d_n_ops) return GWAOI_ERR_INVALID;
  hipStream_t st = (hipStream_t)stream;
  const gw::RsDev d = region_dev(R);
  hipLaunchKernelGGL(gw::k_rs_prep, dim3(2 * gw::kRsChunks + 1), dim3(1024), 0, st, d);
  // the list and the new ids hold distinct slots: N + M <= cap_l (+ cap_new: room for a broken count)
  hipLaunchKernelGGL(gw::k_rs_emit, gw::blocks_for(R->cap_l + R->cap_new), dim3(gw::kSBlock), 0, st, *g, d, d_slots,
                     d_x, d_z, d_kinds, d_n_ops);
  if (hipGetLastError() != hipSuccess) return GWAOI_ERR_HIP;
  R->cur ^= 1u;
  return GWAOI_OK;
}

int gwaoi_strip_translate_events(void* stream, const uint32_t* l2g, uint32_t* d_events, uint32_t n) {
  if (!l2g || (n && !d_events)) return GWAOI_ERR_INVALID;
  if (n)
    hipLaunchKernelGGL(gw::k_translate, gw::blocks_for(n), dim3(gw::kSBlock), 0, (hipStream_t)stream, l2g, d_events, n);
  return hipGetLastError() == hipSuccess ? GWAOI_OK : GWAOI_ERR_HIP;
}

}  // extern "C"
