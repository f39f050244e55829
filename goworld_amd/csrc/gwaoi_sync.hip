// gwaoi_sync.hip — the callers either side of the AOI path, on the GPU (include/gwaoi_sync.h):
//
//   * tick-end sync fan-out (CollectEntitySyncInfos, engine/entity/Entity.go:1207-1267): for every
//     flagged entity, a 48-byte record to its own client and to the client of every AOI neighbour,
//     grouped per gate. The neighbour set is evaluated from the manager's grid exactly as the relation
//     export does (N(a,b) = in(L, F), L = later actor), one thread per grid record in cell order so
//     neighbouring threads walk the same cells. Count walk -> scan -> write walk (entity-major pair list)
//     -> stable counting sort by gate (per 4096-pair chunk: LDS histogram, scan, wave-ballot multisplit
//     ranks) that writes the wire records straight into their gate's packet body.
//
//   * position ingest (HandleSyncPositionYawFromClient, components/game/GameService.go:398-410): 32-byte
//     records decoded on the GPU, EntityID -> slot through an open-addressing hash table (host-owned,
//     mirrored to HBM on change), presence and syncingFromClient checked, accepted records compacted in
//     payload order into a device-counted Moved batch of the manager. A payload that names a slot twice
//     is cut at the first repeat and run as consecutive batches, so the events are those of the
//     reference's sequential loop.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "gwaoi.h"
#include "gwaoi_device.h"
#include "gwaoi_internal.h"
#include "gwaoi_sync.h"

namespace gw {

namespace {

constexpr int kSy = 256;                  // threads per block
constexpr int kGItems = 16;               // pairs per thread in the gate partition
constexpr uint32_t kGChunk = kSy * kGItems;  // pairs per chunk (block) of the gate partition
constexpr uint32_t kHEmpty = 0xFFFFFFFFu;  // hash bucket states (otherwise the bucket holds a slot)
constexpr uint32_t kHTomb = 0xFFFFFFFEu;
constexpr uint32_t kNone = 0xFFFFFFFFu;

__host__ __device__ __forceinline__ uint32_t id_hash(uint4 k) {
  const uint64_t a = ((uint64_t)k.y << 32) | k.x, b = ((uint64_t)k.w << 32) | k.z;
  uint64_t h = (a * 0x9E3779B97F4A7C15ull) ^ ((b + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full);
  h ^= h >> 31;
  h *= 0xD6E8FEB86659FD93ull;
  h ^= h >> 32;
  return (uint32_t)h;
}

__host__ __device__ __forceinline__ bool id_eq(uint4 a, uint4 b) {
  return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
}
__host__ __device__ __forceinline__ bool id_zero(uint4 a) { return !(a.x | a.y | a.z | a.w); }

// ------------------------------------------------------------------------------------------------
// setters: one thread per (deduplicated) entry
struct ScatArgs {
  const uint32_t* slot;
  uint32_t n;
  int mode;  // 0 entity ids, 1 clients, 2 syncing, 3 mark
  const uint4* id;
  const uint16_t* gate;
  const float* y;
  const float* yaw;
  const uint8_t* f;
  uint8_t* flags;
  uint16_t* t_gate;
  uint4* t_cid;
  uint4* t_eid;
  float* t_y;
  float* t_yaw;
};

__global__ void __launch_bounds__(kSy) k_sync_scatter(ScatArgs a) {
  const uint32_t i = blockIdx.x * kSy + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t s = a.slot[i];
  switch (a.mode) {
    case 0:
      a.t_eid[s] = a.id[i];
      if (a.f[i]) {  // a new entity in the slot: nothing of the previous one carries over
        a.flags[s] = 0;
        a.t_gate[s] = GWAOI_SYNC_NO_CLIENT;
        a.t_cid[s] = make_uint4(0, 0, 0, 0);
      }
      break;
    case 1:
      a.t_gate[s] = a.gate[i];
      a.t_cid[s] = a.id[i];
      break;
    case 2: a.flags[s] = (uint8_t)((a.flags[s] & ~GWAOI_SYNC_FROM_CLIENT) | (a.f[i] ? GWAOI_SYNC_FROM_CLIENT : 0u)); break;
    default:
      a.t_y[s] = a.y[i];
      a.t_yaw[s] = a.yaw[i];
      a.flags[s] = (uint8_t)(a.flags[s] | a.f[i]);
      break;
  }
}

// collect, after the fan-out: the sync bits of slots absent from the manager clear without records
// (the fan-out visits present entities only; the reference clears every collected flag, Entity.go:1226)
__global__ void __launch_bounds__(kSy) k_clear_absent(uint8_t* flags, const uint32_t* seq, uint32_t cap) {
  for (uint32_t s = blockIdx.x * kSy + threadIdx.x; s < cap; s += gridDim.x * kSy)
    if (!seq[s] && (flags[s] & (GWAOI_SYNC_OWN_CLIENT | GWAOI_SYNC_NEIGHBOR_CLIENTS)))
      flags[s] = (uint8_t)(flags[s] & ~(GWAOI_SYNC_OWN_CLIENT | GWAOI_SYNC_NEIGHBOR_CLIENTS));
}

// the device hash table: one 32-B bucket per entry, {key} then {slot, 0, 0, 0}, so a probe is one line
__global__ void __launch_bounds__(kSy) k_hash_scatter(const uint32_t* __restrict__ idx, const uint4* __restrict__ key,
                                                      const uint32_t* __restrict__ val, uint32_t n, uint4* hb) {
  const uint32_t i = blockIdx.x * kSy + threadIdx.x;
  if (i >= n) return;
  hb[2 * (size_t)idx[i]] = key[i];
  hb[2 * (size_t)idx[i] + 1] = make_uint4(val[i], 0u, 0u, 0u);
}

// ------------------------------------------------------------------------------------------------
// fan-out
struct FanArgs {
  GridView g;
  const uint32_t* rec_count;
  uint32_t rec_bound;
  const float* pos_x;
  const float* pos_z;
  const uint32_t* space_of;
  uint8_t* flags;
  const uint16_t* gate;
  int clear;            // write pass: clear the sync bits of every collected entity
  uint32_t* cnt;        // count pass: pairs per grid record ([rec_bound + 1], scanned afterwards)
  const uint32_t* off;  // write pass: the scanned counts
  uint2* pairs;         // {entity, receiver} (receiver == entity: own client)
  uint4* tstat;         // count pass: per tile {pairs (64 bits: lo, hi), entities collected, 0}, summed by
                        // k_fan_total (one atomic per wave on one word serialised the count pass: 172 us)
  // client sub-grid: the main records of entities WITH a client, in grid order (the only candidates
  // a fan-out can name), with their own cell starts over the same cell keys
  const uint32_t* ccs;  // [ncells + 1]
  const uint4* crec;    // {x, z, seq_end, slot}
  const uint8_t* cgate;
  const uint32_t* cpos;  // scanned sub-grid positions (own client: the entity's own sub-grid record)
  const uint4* ccid;    // client id of each sub-grid record (direct fan-out)
  const uint4* eid;
  const float* y;
  const float* yaw;
  uint4* info;          // write pass: per grid record of a collected entity {EntityID}, {x, y, z, yaw}
  // direct fan-out (n_gates <= kDirectGates: k_fan_dcount / k_fan_dwrite)
  uint32_t n_gates;
  uint32_t gstride;      // gcnt entries per record (n_gates rounded up to 4)
  uint32_t* gcnt;        // count pass: pairs of each record per gate, record-major [j * gstride + g]
  uint8_t* wantj;        // count pass: each record's collected bits (the flags are cleared there)
  uint32_t* tg;          // count pass: pairs per gate per tile, gate-major [g * ntiles + t] (+ 1 total);
                         // scanned: the first wire record of each (gate, tile) block
  uint32_t ntiles;
  uint4* out;            // write pass: the wire records, 3 uint4 each
  uint32_t out_cap;      // records out holds (nothing is written past it: the host grows it and re-runs)
  const uint4* pk;       // direct passes: per slot {EntityID}, {y, yaw, gate | flags << 16, 0} (k_sync_pack)
};

struct ClientGridArgs {
  const Rec* rec;
  const uint32_t* cs;
  const uint32_t* rec_count;
  uint32_t rec_bound;
  uint32_t ncells;
  const uint16_t* gate;
  uint32_t* cpos;  // [rec_bound + 1]: 0/1, scanned -> position in the sub-grid
  uint32_t* ccs;
  uint4* crec;
  uint8_t* cgate;
  const uint4* cid;
  uint4* ccid;     // client id of each sub-grid record (fan-out reads are then spatially local)
};

__device__ __forceinline__ bool cg_take(const ClientGridArgs& a, uint32_t j, uint32_t nrec) {
  if (j >= nrec) return false;
  const uint32_t z = a.rec[j].a.z;
  return !(z & REC_GHOST) && a.gate[z & REC_SLOT] != GWAOI_SYNC_NO_CLIENT;
}

__global__ void __launch_bounds__(kSy) k_cg_flag(ClientGridArgs a) {
  const uint32_t nrec = *a.rec_count;
  for (uint32_t j = blockIdx.x * kSy + threadIdx.x; j <= a.rec_bound; j += gridDim.x * kSy)
    a.cpos[j] = cg_take(a, j, nrec) ? 1u : 0u;
}

__global__ void __launch_bounds__(kSy) k_cg_build(ClientGridArgs a) {
  const uint32_t nrec = *a.rec_count;
  const uint32_t nth = gridDim.x * kSy;
  for (uint32_t j = blockIdx.x * kSy + threadIdx.x; j < nrec; j += nth) {
    // taken iff the exclusive scan steps at j (j < nrec <= rec_bound: cpos[j + 1] exists): two coalesced
    // words instead of the record and its slot's gate again
    const uint32_t p = a.cpos[j];
    if (a.cpos[j + 1] == p) continue;
    const Rec r = a.rec[j];
    const uint32_t s = r.a.z & REC_SLOT;
    a.crec[p] = make_uint4(r.a.x, r.a.y, r.b.w, s);
    a.cgate[p] = (uint8_t)a.gate[s];
    a.ccid[p] = a.cid[s];
  }
  for (uint32_t c = blockIdx.x * kSy + threadIdx.x; c <= a.ncells; c += nth) a.ccs[c] = a.cpos[a.cs[c]];
}

// Every neighbour o of the entity of main record j whose client exists: f(o). The neighbour set is
// {o : in(L, F)} with L the later actor (Entity.InterestedBy under the XZ manager, see gwaoi_kernels.hip).
template <class F>
__device__ __forceinline__ void client_neighbours(const FanArgs& a, uint32_t s, float sx, float sz, uint32_t qs, F&& f) {
  const Geom g = a.g.geom[a.space_of[s]];
  const float D = g.D;
  const CellBox B = qbox(g, sx, sz);
  for (int r = B.z0; r <= B.z1; ++r) {
    row_entries_global(g, a.ccs, r, B.x0, B.x1, [&](uint32_t j) {
      const uint4 c = a.crec[j];
      const uint32_t o = c.w;
      if (o == s) return;
      const float ox = __uint_as_float(c.x), oz = __uint_as_float(c.y);
      const bool in = (c.z > qs) ? inbox(ox, oz, D, sx, sz) : inbox(sx, sz, D, ox, oz);
      if (in) f(j, a.cgate[j]);
    });
  }
}

// Tile-staged walk: one block per grid tile; the client sub-grid's cell starts and ends of the tile
// plus a halo of `reach` cells are staged in LDS, so a row segment costs two LDS reads instead of two
// dependent global loads. Entities whose box leaves the region (reach 0, coarse grids) walk the
// global table. Same per-record outputs as k_fan (count, pairs in walk order, info, flag clear).
constexpr int kFanRegCells = kSweepRegCells;
constexpr int kFanLdsPairs = 4096;  // 32 KB: a round of 256 entities at ~16 pairs each
constexpr int kFanLdsRecs = 896;    // 14 KB of staged sub-grid records (a uniform region holds ~200); keeps
                                    // the write pass at 3 blocks per CU
template <bool kWrite>
__global__ void __launch_bounds__(kSy) k_fan_tile(FanArgs a) {
  // The region's sub-grid records are copied into LDS in row-major cell order, so one row of a box is
  // ONE contiguous LDS range: cst[i] = first staged record of region cell i (cst[W * Hh] = total).
  __shared__ uint16_t cst[kFanRegCells + 1];
  __shared__ uint4 crl[kFanLdsRecs];  // {x, z, seq_end, sub-grid index}
  __shared__ uint32_t red[kSy / 64];
  __shared__ uint32_t tot_sh;
  __shared__ uint2 lpairs[kWrite ? kFanLdsPairs : 1];
  const uint32_t t = blockIdx.x;
  const uint32_t sp = __builtin_amdgcn_readfirstlane(a.g.tile_space[t]);
  const Geom g = uniform_geom(&a.g.geom[sp]);
  const int lt = (int)(t - g.tile_base);
  const int tx = lt % g.ntx, tz = lt / g.ntx;
  const uint32_t k0 = g.base + ((uint32_t)lt << kTileCellShift);
  const uint32_t j0 = a.g.cs[k0], j1 = a.g.cs[k0 + kTileCells];
  if (j0 == j1) {
    if (!kWrite && threadIdx.x == 0) a.tstat[t] = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  const int R = g.reach;
  const int cx0 = max(tx * kTile - R, 0), cx1 = min(tx * kTile + kTile - 1 + R, g.ncx - 1);
  const int cz0 = max(tz * kTile - R, 0), cz1 = min(tz * kTile + kTile - 1 + R, g.ncz - 1);
  const int W = cx1 - cx0 + 1, Hh = cz1 - cz0 + 1;
  const int ncell = W * Hh;
  const bool lds = R > 0 && ncell <= kFanRegCells &&
                   stage_region<kSy, kFanRegCells, kFanLdsRecs>(g, a.ccs, cx0, cz0, W, ncell, cst, crl, red, &tot_sh,
                                                   [&](uint32_t q) {
                                                     const uint4 c = a.crec[q];
                                                     return make_uint4(c.x, c.y, c.z, q);
                                                   });
  uint32_t ents = 0;
  // one record: count (and, in the write pass, emit) its pairs through `put`
  auto visit = [&](uint32_t j, auto&& put) {
    uint32_t c = 0;
    const uint4 ra = a.g.rec[j].a;
    const uint32_t s = ra.z & REC_SLOT;
    const uint8_t fl = (ra.z & REC_GHOST) ? 0 : a.flags[s];
    const uint32_t want = fl & (GWAOI_SYNC_OWN_CLIENT | GWAOI_SYNC_NEIGHBOR_CLIENTS);
    if (want) {
      ++ents;
      uint32_t w = kWrite ? a.off[j] : 0u;
      const uint32_t w0 = w;
      uint4 eid = make_uint4(0, 0, 0, 0);
      float yy = 0.0f, yw = 0.0f;
      if (kWrite) {  // issued before the walk: independent of it
        eid = a.eid[s];
        yy = a.y[s];
        yw = a.yaw[s];
      }
      const uint16_t gs = a.gate[s];
      if ((want & GWAOI_SYNC_OWN_CLIENT) && gs != GWAOI_SYNC_NO_CLIENT) {
        if (kWrite) put(w++, make_uint2(j, a.cpos[j]));
        ++c;
      }
      if (want & GWAOI_SYNC_NEIGHBOR_CLIENTS) {
        const float sx = __uint_as_float(ra.x), sz = __uint_as_float(ra.y);
        const uint32_t qs = a.g.rec[j].b.w;
        const CellBox B = qbox(g, sx, sz);
        if (lds && B.x0 >= cx0 && B.x1 <= cx1 && B.z0 >= cz0 && B.z1 <= cz1) {
          const float D = g.D;
          // the entity's own sub-grid record (only an entity with a client has one)
          const uint32_t selfq = gs != GWAOI_SYNC_NO_CLIENT ? a.cpos[j] : 0xffffffffu;
          for (int r = B.z0; r <= B.z1; ++r) {
            const int rb = (r - cz0) * W - cx0;
            const uint32_t e = cst[rb + B.x1 + 1];
            for (uint32_t p = cst[rb + B.x0]; p < e; ++p) {
              const uint4 cr = crl[p];
              const float ox = __uint_as_float(cr.x), oz = __uint_as_float(cr.y);
              const bool in = cr.w != selfq && ((cr.z > qs) ? inbox(ox, oz, D, sx, sz) : inbox(sx, sz, D, ox, oz));
              if (in) {
                if (kWrite) put(w++, make_uint2(j, cr.w));
                ++c;
              }
            }
          }
        } else {
          client_neighbours(a, s, sx, sz, qs, [&](uint32_t cj, uint8_t) {
            if (kWrite) put(w++, make_uint2(j, cj));
            ++c;
          });
        }
      }
      if (kWrite) {
        if (w != w0) {
          a.info[2 * (size_t)j] = eid;
          a.info[2 * (size_t)j + 1] = make_uint4(ra.x, __float_as_uint(yy), ra.y, __float_as_uint(yw));
        }
        if (a.clear) a.flags[s] = (uint8_t)(fl & ~(GWAOI_SYNC_OWN_CLIENT | GWAOI_SYNC_NEIGHBOR_CLIENTS));
      }
    }
    return c;
  };
  unsigned long long psum = 0;  // count pass: this thread's pairs
  for (uint32_t jb = j0; jb < j1; jb += kSy) {
    const uint32_t j = jb + threadIdx.x;
    if (!kWrite) {
      if (j < j1) {
        const uint32_t c = visit(j, [](uint32_t, uint2) {});
        a.cnt[j] = c;
        psum += c;
      }
      continue;
    }
    // write pass, per round of kSy records: their output is the contiguous range [off[jb], off[je]),
    // staged in LDS and copied out coalesced when it fits (else written directly)
    const uint32_t pb = a.off[jb], pe = a.off[min(jb + kSy, j1)];
    if (pe - pb <= (uint32_t)kFanLdsPairs) {
      if (j < j1) visit(j, [&](uint32_t w, uint2 v) { lpairs[w - pb] = v; });
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < pe - pb; i += kSy) a.pairs[pb + i] = lpairs[i];
      __syncthreads();
    } else if (j < j1) {
      uint2* pairs = a.pairs;
      visit(j, [&](uint32_t w, uint2 v) { pairs[w] = v; });
    }
  }
  if (!kWrite) {  // the tile's totals, stored (no atomics)
    __shared__ unsigned long long rp[kSy / 64];
    for (int o = 32; o > 0; o >>= 1) psum += __shfl_xor(psum, o, 64);
    for (int o = 32; o > 0; o >>= 1) ents += __shfl_xor(ents, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ents, rp[threadIdx.x >> 6] = psum;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tot = 0;
      unsigned long long pt = 0;
      for (int k = 0; k < kSy / 64; ++k) tot += red[k], pt += rp[k];
      a.tstat[t] = make_uint4((uint32_t)pt, (uint32_t)(pt >> 32), tot, 0u);
    }
  }
}

// ---- direct fan-out (n_gates <= kDirectGates) ---------------------------------------------------
// The wire records are written straight into their gate's packet, in grid order, with no pair list and
// no gate partition: the count pass stores each record's pairs PER GATE (record-major) and each tile's
// pairs per gate (gate-major); one small scan over the (gate, tile) totals gives every (gate, tile)
// block its first record, and the gate offsets. The write pass block-scans a round's per-gate counts
// into per-thread cursors, walks again, and stages the round's records as 4-byte references
// {receiver, entity, gate} in LDS; the round's records of one gate are one contiguous range of the
// packet, copied out 16 B per lane over consecutive addresses. Same records and order as the
// partition path: gates in order, entities in grid order, each entity's run contiguous with its own
// client's record first.
#ifndef GW_FAN_UNROLL  // candidates of a row judged per step of the pair walk (loads in flight together)
#define GW_FAN_UNROLL 2
#endif
#ifndef GW_ABL_FAN  // ablation (timing only), write pass without: 1 its copy-out, 2 + its pair walk, 3 + the region
                    // staging, 4 + the entities' loads
#define GW_ABL_FAN 0
#endif
constexpr uint32_t kDirectGates = 8;
#ifndef GW_FAN_NT
#define GW_FAN_NT 1
#endif
// A wire record part into the packet buffer: written once per collect and read by the consumer later,
// so stored non-temporally. Plain stores left the collect's ~390 MB of records in the caches at the
// expense of what the next kernels reuse (r04_c31, gametick: write pass 190 -> 177 us, the next
// ingest's hash lookups 68 -> 59 us, the next grid build 36.5 -> 30.4 us; 0.648 -> 0.624 ms/step).
__device__ __forceinline__ void fan_store(uint4* p, const uint4 v) {
#if GW_FAN_NT
  __builtin_nontemporal_store(v.x, &p->x);
  __builtin_nontemporal_store(v.y, &p->y);
  __builtin_nontemporal_store(v.z, &p->z);
  __builtin_nontemporal_store(v.w, &p->w);
#else
  *p = v;
#endif
}

// The per-slot fields the direct passes read for each collected entity, packed into one 32-B record per
// slot at the start of the collect: {EntityID}, {y, yaw, gate | flags << 16, 0}. The passes visit the
// entities in grid order, i.e. at random slots: one 32-B gather per entity instead of a line fetched
// per field (54 of the write pass's 217 us were those gathers, r04_c17). (On a side stream beside the
// count pass instead, both ran slower: tick 0.66 -> 0.69 ms, r04_c21.) With `clear`, the sync bits of
// EVERY slot are cleared here, once packed (a collected entity's bits clear, and so do an absent slot's:
// k_clear_absent's contract); nothing after the pack reads them.
__global__ void __launch_bounds__(kSy) k_sync_pack(uint8_t* __restrict__ flags, const uint16_t* __restrict__ gate,
                                                   const uint4* __restrict__ eid, const float* __restrict__ y,
                                                   const float* __restrict__ yaw, uint32_t cap, int clear,
                                                   uint4* __restrict__ pk) {
  for (uint32_t s = blockIdx.x * kSy + threadIdx.x; s < cap; s += gridDim.x * kSy) {
    const uint8_t fl = flags[s];
    pk[2 * (size_t)s] = eid[s];
    pk[2 * (size_t)s + 1] = make_uint4(__float_as_uint(y[s]), __float_as_uint(yaw[s]),
                                       (uint32_t)gate[s] | ((uint32_t)fl << 16), 0u);
    if (clear) flags[s] = fl & (uint8_t)~(GWAOI_SYNC_OWN_CLIENT | GWAOI_SYNC_NEIGHBOR_CLIENTS);
  }
}
constexpr uint32_t kRoundRecs = 2560;   // a round's staged records (10 KB of references)
constexpr int kDirLdsRecs = 384;        // staged sub-grid records of the direct kernels (config 2: ~210 per
                                        // region); with the write pass's ClientIDs, 4 blocks per CU
constexpr uint32_t kRefSkip = 0xFFFFFFFFu;  // written directly (receiver outside the LDS region)
constexpr uint32_t kRefOwn = 1u << 28;      // the entity's own client

struct FanGeo {
  Geom g;
  int cx0, cx1, cz0, cz1, W, Hh;
  uint32_t j0, j1;
};

__device__ __forceinline__ FanGeo fan_geo(const FanArgs& a, uint32_t t) {
  FanGeo f;
  const uint32_t sp = __builtin_amdgcn_readfirstlane(a.g.tile_space[t]);
  f.g = uniform_geom(&a.g.geom[sp]);
  const int lt = (int)(t - f.g.tile_base);
  const int tx = lt % f.g.ntx, tz = lt / f.g.ntx;
  const uint32_t k0 = f.g.base + ((uint32_t)lt << kTileCellShift);
  f.j0 = a.g.cs[k0];
  f.j1 = a.g.cs[k0 + kTileCells];
  const int R = f.g.reach;
  f.cx0 = max(tx * kTile - R, 0), f.cx1 = min(tx * kTile + kTile - 1 + R, f.g.ncx - 1);
  f.cz0 = max(tz * kTile - R, 0), f.cz1 = min(tz * kTile + kTile - 1 + R, f.g.ncz - 1);
  f.W = f.cx1 - f.cx0 + 1, f.Hh = f.cz1 - f.cz0 + 1;
  return f;
}

// Every client neighbour of the entity of main record ra (the pair predicate of k_fan_tile): f(gate, lds
// index or kNone, sub-grid index). qs: the record's seq_end, selfq: the entity's own sub-grid record or
// 0xffffffff (loaded by the caller, ahead of the walk).
template <class F>
__device__ __forceinline__ void fan_pairs(const FanArgs& a, const FanGeo& fg, bool lds, const uint16_t* cst,
                                          const uint4* crl, const uint8_t* cgl, uint32_t qs, uint32_t selfq, uint4 ra,
                                          uint32_t s, F&& f) {
  const Geom& g = fg.g;
  const float sx = __uint_as_float(ra.x), sz = __uint_as_float(ra.y);
  const CellBox B = qbox(g, sx, sz);
  if (lds && B.x0 >= fg.cx0 && B.x1 <= fg.cx1 && B.z0 >= fg.cz0 && B.z1 <= fg.cz1) {
    const float D = g.D;
    auto test = [&](const uint4 cr, uint32_t p) {
      const float ox = __uint_as_float(cr.x), oz = __uint_as_float(cr.y);
      const bool in = cr.w != selfq && ((cr.z > qs) ? inbox(ox, oz, D, sx, sz) : inbox(sx, sz, D, ox, oz));
      if (in) f((uint32_t)cgl[p], p, cr.w);
    };
    for (int r = B.z0; r <= B.z1; ++r) {
      const int rb = (r - fg.cz0) * fg.W - fg.cx0;
      const uint32_t e = cst[rb + B.x1 + 1];
#if GW_FAN_UNROLL > 1
      for (uint32_t p = cst[rb + B.x0]; p < e; p += GW_FAN_UNROLL) {
        uint4 cr[GW_FAN_UNROLL];
#pragma unroll
        for (int k = 0; k < GW_FAN_UNROLL; ++k) cr[k] = crl[min(p + k, e - 1)];
#pragma unroll
        for (int k = 0; k < GW_FAN_UNROLL; ++k)
          if (p + k < e) test(cr[k], p + k);
      }
#else
      for (uint32_t p = cst[rb + B.x0]; p < e; ++p) test(crl[p], p);
#endif
    }
  } else {
    client_neighbours(a, s, sx, sz, qs, [&](uint32_t cj, uint8_t cg) { f((uint32_t)cg, kNone, cj); });
  }
}

// stage the tile's region of the client sub-grid (and each staged record's gate); false: walk global
__device__ __forceinline__ bool fan_stage(const FanArgs& a, const FanGeo& fg, uint16_t* cst, uint4* crl, uint8_t* cgl,
                                          uint32_t* red, uint32_t* tot_sh, uint4* cidl = nullptr) {
  const int ncell = fg.W * fg.Hh;
  const bool lds = fg.g.reach > 0 && ncell <= kFanRegCells &&
                   stage_region<kSy, kFanRegCells, kDirLdsRecs>(fg.g, a.ccs, fg.cx0, fg.cz0, fg.W, ncell, cst, crl, red,
                                                                 tot_sh, [&](uint32_t q) {
                                                                   const uint4 c = a.crec[q];
                                                                   return make_uint4(c.x, c.y, c.z, q);
                                                                 });
  if (lds) {
    const uint32_t ns = cst[ncell];
    for (uint32_t p = threadIdx.x; p < ns; p += kSy) {
      const uint32_t q = crl[p].w;
      cgl[p] = a.cgate[q];
      if (cidl) cidl[p] = a.ccid[q];  // (write pass: the receivers' ClientIDs, gathered once per region)
    }
    __syncthreads();
  }
  return lds;
}

// a gate's per-thread counter / cursor in registers: static indices only (a dynamic index would go
// through scratch), one select per gate
__device__ __forceinline__ uint32_t gate_bump(uint32_t (&c)[kDirectGates], uint32_t g) {
  uint32_t v = 0;
#pragma unroll
  for (uint32_t k = 0; k < kDirectGates; ++k) {
    v = g == k ? c[k] : v;
    c[k] += g == k ? 1u : 0u;
  }
  return v;
}

__global__ void __launch_bounds__(kSy) k_fan_dcount(FanArgs a) {
  __shared__ uint16_t cst[kFanRegCells + 1];
  __shared__ uint4 crl[kDirLdsRecs];
  __shared__ uint8_t cgl[kDirLdsRecs];
  __shared__ uint32_t gred[kDirectGates][kSy / 64];
  __shared__ uint32_t red[kSy / 64];
  __shared__ uint32_t tot_sh;
  __shared__ unsigned long long rp[kSy / 64];
  const uint32_t G = a.n_gates, t = blockIdx.x;
  if (t == 0 && threadIdx.x == 0) a.tg[G * a.ntiles] = 0u;  // (the scan's total lands there)
  const FanGeo fg = fan_geo(a, t);
  if (fg.j0 == fg.j1) {
    if (threadIdx.x < G) a.tg[threadIdx.x * a.ntiles + t] = 0u;
    if (threadIdx.x == 0) a.tstat[t] = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  const bool lds = fan_stage(a, fg, cst, crl, cgl, red, &tot_sh);
  __syncthreads();
  uint32_t ents = 0;
  unsigned long long psum = 0;
  uint32_t gtot[kDirectGates];  // the thread's pairs per gate over its rounds (reduced once per tile)
#pragma unroll
  for (uint32_t g = 0; g < kDirectGates; ++g) gtot[g] = 0u;
  const uint32_t tid = threadIdx.x;
  for (uint32_t jb = fg.j0; jb < fg.j1; jb += kSy) {
    const uint32_t j = jb + tid;
    if (j >= fg.j1) continue;
    uint32_t c[kDirectGates];
#pragma unroll
    for (uint32_t g = 0; g < kDirectGates; ++g) c[g] = 0u;
    const uint4 ra = a.g.rec[j].a;
    const uint32_t s = ra.z & REC_SLOT;
    const uint32_t pw = (ra.z & REC_GHOST) ? 0u : a.pk[2 * (size_t)s + 1].z;  // gate | flags << 16
    const uint8_t want = (uint8_t)(pw >> 16) & (GWAOI_SYNC_OWN_CLIENT | GWAOI_SYNC_NEIGHBOR_CLIENTS);
    if (want) {
      ++ents;
      const uint16_t gs = (uint16_t)pw;
      if ((want & GWAOI_SYNC_OWN_CLIENT) && gs < G) gate_bump(c, gs);
      if (want & GWAOI_SYNC_NEIGHBOR_CLIENTS)
        fan_pairs(a, fg, lds, cst, crl, cgl, a.g.rec[j].b.w, gs != GWAOI_SYNC_NO_CLIENT ? a.cpos[j] : 0xffffffffu, ra,
                  s, [&](uint32_t g, uint32_t, uint32_t) {
                    if (g < G) gate_bump(c, g);
                  });
    }
    a.wantj[j] = want;
    uint4* dst = reinterpret_cast<uint4*>(a.gcnt + (size_t)j * a.gstride);
    dst[0] = make_uint4(c[0], c[1], c[2], c[3]);
    if (a.gstride > 4) dst[1] = make_uint4(c[4], c[5], c[6], c[7]);
#pragma unroll
    for (uint32_t g = 0; g < kDirectGates; ++g) {
      psum += c[g];
      gtot[g] += c[g];
    }
  }
  // tile totals per gate: wave sums, then the block's (one LDS word per wave and gate)
#pragma unroll
  for (uint32_t g = 0; g < kDirectGates; ++g) {
    uint32_t v = gtot[g];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((tid & 63) == 0) gred[g][tid >> 6] = v;
  }
  for (int o = 32; o > 0; o >>= 1) psum += __shfl_xor(psum, o, 64);
  for (int o = 32; o > 0; o >>= 1) ents += __shfl_xor(ents, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = ents, rp[tid >> 6] = psum;
  __syncthreads();
  if (tid < G) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < kSy / 64; ++k) v += gred[tid][k];
    a.tg[tid * a.ntiles + t] = v;
  }
  if (tid == 0) {
    uint32_t tot = 0;
    unsigned long long pt = 0;
    for (int k = 0; k < kSy / 64; ++k) tot += red[k], pt += rp[k];
    a.tstat[t] = make_uint4((uint32_t)pt, (uint32_t)(pt >> 32), tot, 0u);
  }
}

__global__ void __launch_bounds__(kSy) __attribute__((amdgpu_waves_per_eu(3))) k_fan_dwrite(FanArgs a) {
  __shared__ uint16_t cst[kFanRegCells + 1];
  __shared__ uint4 crl[kDirLdsRecs];
  __shared__ uint8_t cgl[kDirLdsRecs];
  __shared__ uint32_t gbase[kDirectGates];      // out index of the round's first record of each gate
  __shared__ uint32_t wred[kDirectGates][kSy / 64];
  __shared__ uint32_t groff[kDirectGates];      // round position of each gate's first record
  __shared__ uint32_t gtot[kDirectGates];       // the round's records of each gate
  __shared__ uint32_t ref[kRoundRecs];
  __shared__ uint4 cidl[kDirLdsRecs];           // the staged receivers' ClientIDs
  __shared__ uint4 ent[kSy][2];                 // the round's entities: EntityID, {x, y, z, yaw}
  __shared__ uint4 ocid[kSy];                   // and their own client's id
  __shared__ uint32_t red[kSy / 64];
  __shared__ uint32_t tot_sh;
  const uint32_t G = a.n_gates, t = blockIdx.x, tid = threadIdx.x;
  const FanGeo fg = fan_geo(a, t);
  if (fg.j0 == fg.j1) return;
  if (tid < G) gbase[tid] = a.tg[tid * a.ntiles + t];
  const bool lds = GW_ABL_FAN < 3 && fan_stage(a, fg, cst, crl, cgl, red, &tot_sh, cidl);
  __syncthreads();  // gbase
  const int lane = tid & 63, w = tid >> 6;
  // A round's per-entity inputs. The next round's are loaded during this one (software pipelined:
  // the record-order loads at the round's start, the slot gathers after its walk, the own client's id
  // after its copy-out), so each round's walk and copy-out cover the gathers' latency.
  struct RoundIn {
    uint32_t want, qs, cp, c[kDirectGates];
    uint4 ra, eid, pw, own;
  };
  auto load_rec = [&](uint32_t j, RoundIn& in) {  // record order: coalesced
    const bool live = j < fg.j1;
    in.want = live ? a.wantj[j] : 0u;
#pragma unroll
    for (uint32_t g = 0; g < kDirectGates; ++g) in.c[g] = 0u;
    in.ra = make_uint4(0, 0, 0, 0);
    in.qs = in.cp = 0u;
    if (live) {
      const uint4* src = reinterpret_cast<const uint4*>(a.gcnt + (size_t)j * a.gstride);
#pragma unroll
      for (uint32_t g4 = 0; g4 < kDirectGates; g4 += 4) {
        if (g4 < a.gstride) {
          const uint4 v = src[g4 / 4];
          in.c[g4] = v.x, in.c[g4 + 1] = v.y, in.c[g4 + 2] = v.z, in.c[g4 + 3] = v.w;
        }
      }
      in.ra = a.g.rec[j].a;
      in.qs = a.g.rec[j].b.w;
      in.cp = a.cpos[j];
    }
  };
  auto load_slot = [&](RoundIn& in) {  // the entity's slot: one 32-B gather
    in.eid = in.pw = make_uint4(0, 0, 0, 0);
    in.pw.z = GWAOI_SYNC_NO_CLIENT;
    if (GW_ABL_FAN < 4 && in.want) {
      const size_t s2 = 2 * (size_t)(in.ra.z & REC_SLOT);
      in.eid = a.pk[s2];
      in.pw = a.pk[s2 + 1];
    }
  };
  auto load_own = [&](RoundIn& in) {
    in.own = make_uint4(0, 0, 0, 0);
    if ((in.want & GWAOI_SYNC_OWN_CLIENT) && (in.pw.z & 0xFFFFu) < G) in.own = a.ccid[in.cp];
  };
  RoundIn rin, rnx;
  load_rec(fg.j0 + tid, rin);
  load_slot(rin);
  load_own(rin);
  for (uint32_t jb = fg.j0; jb < fg.j1; jb += kSy) {  // block-uniform
    const uint32_t j = jb + tid;
    const bool more = jb + kSy < fg.j1;  // block-uniform
    if (more) load_rec(j + kSy, rnx);
    const uint32_t want = rin.want;
    uint32_t c[kDirectGates];
#pragma unroll
    for (uint32_t g = 0; g < kDirectGates; ++g) c[g] = rin.c[g];
    const uint4 ra = rin.ra, eid = rin.eid, own = rin.own;
    const uint4 info = make_uint4(ra.x, rin.pw.x, ra.y, rin.pw.y);
    const uint32_t s = ra.z & REC_SLOT;
    const uint16_t gs = (uint16_t)rin.pw.z;
    // block scan of the per-gate counts: wave scans, then the waves' totals
    uint32_t inc[kDirectGates];
#pragma unroll
    for (uint32_t g = 0; g < kDirectGates; ++g) {
      const uint32_t v = wave_incl_scan(c[g]);  // (DPP; every lane of the block reaches it)
      inc[g] = v;
      if (lane == 63) wred[g][w] = v;
    }
    __syncthreads();
    uint32_t roff = 0;  // round position of gate g's first record
    uint32_t cur[kDirectGates];  // the thread's next record per gate (round position, or out index)
    bool staged;
    {
      uint32_t R = 0;
#pragma unroll
      for (uint32_t g = 0; g < kDirectGates; ++g) {
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < kSy / 64; ++k) {
          const uint32_t x = wred[g][k];
          before += k < w ? x : 0u;
          tot += x;
        }
        inc[g] = before + inc[g] - c[g];  // exclusive prefix within the round
        c[g] = tot;                       // the round's records of gate g
        R += tot;
      }
      staged = R <= kRoundRecs;  // block-uniform
#pragma unroll
      for (uint32_t g = 0; g < kDirectGates; ++g) {
        cur[g] = staged ? roff + inc[g] : gbase[g] + inc[g];
        if (tid == 0) groff[g] = roff, gtot[g] = c[g];
        roff += c[g];
      }
    }
    if (want) {  // (the previous round's copy-out read ent / ocid before its last barrier)
      ent[tid][0] = eid;
      ent[tid][1] = info;
      ocid[tid] = own;
    }
    __syncthreads();  // groff / gtot
    auto put_direct = [&](uint32_t dst, const uint4& cid) {
      if (dst < a.out_cap) {
        fan_store(&a.out[3 * (size_t)dst], cid);
        fan_store(&a.out[3 * (size_t)dst + 1], eid);
        fan_store(&a.out[3 * (size_t)dst + 2], info);
      }
    };
    if (want) {
      if ((want & GWAOI_SYNC_OWN_CLIENT) && gs < G) {
        const uint32_t pos = gate_bump(cur, gs);
        if (!staged) put_direct(pos, own);
        else if (pos < kRoundRecs) ref[pos] = kRefOwn | (tid << 12) | ((uint32_t)gs << 20);
      }
      auto pair = [&](uint32_t g, uint32_t p, uint32_t q) {
        if (g >= G) return;
        const uint32_t pos = gate_bump(cur, g);
        if (!staged) {
          put_direct(pos, p != kNone ? cidl[p] : a.ccid[q]);
        } else if (pos < kRoundRecs) {
          if (p != kNone) {
            ref[pos] = p | (tid << 12) | (g << 20);
          } else {  // a receiver outside the staged region: written now, skipped by the copy-out
            ref[pos] = kRefSkip;
            put_direct(gbase[g] + (pos - groff[g]), a.ccid[q]);
          }
        }
      };
      if (GW_ABL_FAN < 2 && (want & GWAOI_SYNC_NEIGHBOR_CLIENTS))
        fan_pairs(a, fg, lds, cst, crl, cgl, rin.qs, gs != GWAOI_SYNC_NO_CLIENT ? rin.cp : 0xffffffffu, ra, s, pair);
    }
    if (more) load_slot(rnx);
    __syncthreads();
    if (staged && GW_ABL_FAN == 0) {  // copy-out: record r of the round, 16-B part k, over consecutive addresses per gate;
                   // four parts per thread in flight (the ClientID gathers are global loads)
      const uint32_t nq = 3 * roff;
      constexpr size_t kNoDst = ~(size_t)0;
      auto fetch = [&](uint32_t i, size_t& dst) -> uint4 {  // part i of the round: its value and out index
        const bool on = i < nq;
        const uint32_t r = on ? i / 3 : 0u, k = i - 3 * r;
        const uint32_t v = on ? ref[r] : kRefSkip;
        const uint32_t g = (v >> 20) & 0xFFu, owner = (v >> 12) & 0xFFu;
        const bool live = v != kRefSkip;
        const uint32_t d = live ? gbase[g] + (r - groff[g]) : 0u;
        dst = live && d < a.out_cap ? 3 * (size_t)d + k : kNoDst;
        if (!live) return make_uint4(0, 0, 0, 0);
        if (k != 0) return ent[owner][k - 1];
        return (v & kRefOwn) ? ocid[owner] : cidl[v & 0xFFFu];
      };
      for (uint32_t i0 = tid; i0 < nq; i0 += 4 * kSy) {
        size_t d0, d1, d2, d3;
        const uint4 v0 = fetch(i0, d0), v1 = fetch(i0 + kSy, d1), v2 = fetch(i0 + 2 * kSy, d2),
                    v3 = fetch(i0 + 3 * kSy, d3);
        if (d0 != kNoDst) fan_store(&a.out[d0], v0);
        if (d1 != kNoDst) fan_store(&a.out[d1], v1);
        if (d2 != kNoDst) fan_store(&a.out[d2], v2);
        if (d3 != kNoDst) fan_store(&a.out[d3], v3);
      }
    }
    if (more) load_own(rnx);
    __syncthreads();
    if (tid < G) gbase[tid] += gtot[tid];
    __syncthreads();
    rin = rnx;
  }
}

// two small device ranges into the mapped host words the host reads after the stream synchronises (no
// DMA copy per range: each cost a copy-engine round trip on the collect / ingest critical path)
__global__ void k_to_host(const uint32_t* __restrict__ a, uint32_t na, uint32_t oa, const uint32_t* __restrict__ b,
                          uint32_t nb, uint32_t ob, uint32_t* h) {
  for (uint32_t i = threadIdx.x; i < na; i += blockDim.x) h[oa + i] = a[i];
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) h[ob + i] = b[i];
  __threadfence_system();
}

// gate offsets of the direct fan-out: the scanned (gate, tile) blocks' first records (g = G: the total)
__global__ void __launch_bounds__(1024) k_fan_total(const uint4* __restrict__ tstat, uint32_t ntiles, uint32_t* n_ent,
                                                    unsigned long long* npairs64) {
  __shared__ unsigned long long sp[1024 / 64];
  __shared__ uint32_t se[1024 / 64];
  unsigned long long p = 0;
  uint32_t e = 0;
  for (uint32_t i = threadIdx.x; i < ntiles; i += 1024) {
    const uint4 v = tstat[i];
    p += (unsigned long long)v.x | ((unsigned long long)v.y << 32);
    e += v.z;
  }
  for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o, 64), e += __shfl_xor(e, o, 64);
  if ((threadIdx.x & 63) == 0) sp[threadIdx.x >> 6] = p, se[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 1024 / 64; ++k) p += sp[k], e += se[k];
    *npairs64 = p;
    *n_ent = e;
  }
}
__global__ void k_fan_goff(const uint32_t* __restrict__ tg, uint32_t ntiles, uint32_t G, uint32_t* goff) {
  const uint32_t g = threadIdx.x;
  if (g <= G) goff[g] = tg[(size_t)g * ntiles];
}

struct GateArgs {
  const uint2* pairs;
  const uint8_t* cgate;  // gate of a pair = gate of its receiver's sub-grid record
  uint32_t n;        // pairs
  uint32_t nchunks;
  uint32_t n_gates;
  int bits;          // ceil(log2(n_gates)), >= 1
  uint32_t* ghist;   // [n_gates * nchunks + 1], gate-major; scanned between the two kernels
  const uint4* ccid;
  const uint4* info;
  uint4* out;        // 3 uint4 per record
  uint32_t* goff;    // [n_gates + 1]
};

__global__ void __launch_bounds__(kSy) k_gate_hist(GateArgs a) {
  __shared__ uint32_t h[GWAOI_SYNC_MAX_GATES];
  for (uint32_t g = threadIdx.x; g < a.n_gates; g += kSy) h[g] = 0;
  __syncthreads();
  const uint32_t b0 = blockIdx.x * kGChunk;
#pragma unroll 4
  for (int k = 0; k < kGItems; ++k) {
    const uint32_t i = b0 + k * kSy + threadIdx.x;
    if (i < a.n) atomicAdd(&h[a.cgate[a.pairs[i].y]], 1u);
  }
  __syncthreads();
  for (uint32_t g = threadIdx.x; g < a.n_gates; g += kSy) a.ghist[g * a.nchunks + blockIdx.x] = h[g];
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ghist[a.n_gates * a.nchunks] = 0;
}

// Stable partition of one chunk by gate: rounds of 256 pairs; inside a wave, lanes of the same gate
// are found with one ballot per gate bit; across the block's 4 waves, per-wave gate counts in LDS.
// A round's records are staged in LDS in partition order (its records of one gate are one run, and
// land in one contiguous output range), then copied out 16 B per lane over consecutive addresses,
// so the stores cover whole lines instead of one 48-B record per lane.
__global__ void __launch_bounds__(kSy) k_gate_scatter(GateArgs a) {
  __shared__ uint32_t run[GWAOI_SYNC_MAX_GATES];         // pairs of each gate placed by earlier rounds
  __shared__ uint32_t wc[kSy / 64][GWAOI_SYNC_MAX_GATES];  // this round: pairs of each gate per wave
  __shared__ uint32_t gst[GWAOI_SYNC_MAX_GATES];         // this round: first staged record of each gate
  __shared__ uint32_t red[kSy / 64];
  __shared__ uint32_t nlive_sh;
  __shared__ uint4 lrec[3 * kSy];                          // staged records (3 x 16 B each)
  __shared__ uint32_t lpos[kSy];                           // output record index of each staged record
  static_assert(GWAOI_SYNC_MAX_GATES <= kSy, "one thread per gate in the round scan");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint32_t g = threadIdx.x; g < a.n_gates; g += kSy) {
    run[g] = a.ghist[g * a.nchunks + blockIdx.x];  // chunk's base in the gate-major output
#pragma unroll
    for (int k = 0; k < kSy / 64; ++k) wc[k][g] = 0;
  }
  __syncthreads();
  const uint32_t b0 = blockIdx.x * kGChunk;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int k = 0; k < kGItems; ++k) {
    const uint32_t i = b0 + k * kSy + threadIdx.x;
    const bool live = i < a.n;
    const uint2 p = live ? a.pairs[i] : make_uint2(0u, 0u);
    const uint32_t g = live ? a.cgate[p.y] : 0u;
    unsigned long long same = __ballot(live);
    for (int b = 0; b < a.bits; ++b) {
      const unsigned long long v = __ballot(live && ((g >> b) & 1u));
      same &= ((g >> b) & 1u) ? v : ~v;
    }
    const bool leader = live && !(same & lt);
    if (leader) wc[w][g] = (uint32_t)__popcll(same);
    __syncthreads();
    // exclusive scan of the round's per-gate totals (thread t = gate t)
    uint32_t tot = 0;
    if (threadIdx.x < a.n_gates) {
#pragma unroll
      for (int q = 0; q < kSy / 64; ++q) tot += wc[q][threadIdx.x];
    }
    uint32_t inc = tot;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) red[w] = inc;
    __syncthreads();
    for (int q = 0; q < w; ++q) inc += red[q];
    if (threadIdx.x < a.n_gates) gst[threadIdx.x] = inc - tot;
    if (threadIdx.x == kSy - 1) nlive_sh = inc;
    __syncthreads();
    if (live) {
      // p = {grid record of the entity, sub-grid record of the receiver}
      uint32_t r = (uint32_t)__popcll(same & lt);
      for (int q = 0; q < w; ++q) r += wc[q][g];
      const uint32_t li = gst[g] + r;
      lpos[li] = run[g] + r;
      lrec[3 * li] = a.ccid[p.y];
      lrec[3 * li + 1] = a.info[2 * (size_t)p.x];
      lrec[3 * li + 2] = a.info[2 * (size_t)p.x + 1];
    }
    __syncthreads();
    if (leader) {
      atomicAdd(&run[g], (uint32_t)__popcll(same));  // one leader per (wave, gate)
      wc[w][g] = 0;
    }
    const uint32_t nq = 3 * nlive_sh;
    for (uint32_t q = threadIdx.x; q < nq; q += kSy) {
      const uint32_t li = q / 3;
      fan_store(&a.out[(size_t)lpos[li] * 3 + (q - 3 * li)], lrec[q]);
    }
    __syncthreads();
  }
}

__global__ void k_gate_offsets(GateArgs a) {
  const uint32_t g = threadIdx.x + blockIdx.x * blockDim.x;
  if (g <= a.n_gates) a.goff[g] = a.ghist[g * a.nchunks];
}

// ------------------------------------------------------------------------------------------------
// ingest
struct IngArgs {
  const uint4* rec;  // 2 uint4 per record
  uint32_t n;        // records in the payload
  uint32_t seg;      // first record of this batch
  uint32_t hmask;
  const uint4* hb;       // buckets: [2b] key, [2b + 1].x slot (kHEmpty / kHTomb)
  const uint32_t* seq;
  uint8_t* flags;
  float* y;
  float* yaw;
  uint32_t* res;     // per record: slot, or kNone (not accepted)
  uint32_t* first;   // per slot: first record of this batch naming it (kNone between batches)
  uint32_t* ctr;     // [0] cut, [1] unknown, [2] rejected, [3] non-finite x or z
  uint32_t* bcnt;    // per block: accepted records of the batch, scanned -> offsets; [nb] = total
  uint32_t* op_slot;
  float* op_x;
  float* op_z;
};

__device__ __forceinline__ void wave_add(uint32_t* p, uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(p, v);
}

// resolve every record once: slot or kNone, with the unknown / rejected counts. The first batch's
// repeat search rides along (k_ing_first / k_ing_cut for the later batches): each accepted record
// lowers first[slot] by an atomicMin, and when the value it replaced is a record too, the later of the
// two repeats the slot; every slot's second record is found that way whichever atomic ran first, so
// the smallest such index (ctr[0], preset to n) is the batch's cut.
__global__ void __launch_bounds__(kSy) k_ing_resolve(IngArgs a) {
  const uint32_t i = blockIdx.x * kSy + threadIdx.x;
  uint32_t unk = 0, rej = 0, nonf = 0, rep = kNone;
  if (i < a.n) {
    const uint4 id = a.rec[2 * i];
    uint32_t b = id_hash(id) & a.hmask, slot = kNone;
    for (;;) {
      const uint4 k = a.hb[2 * (size_t)b];  // key and slot of a bucket: one 32-B line, both loads together
      const uint32_t v = a.hb[2 * (size_t)b + 1].x;
      if (v == kHEmpty) break;
      if (v != kHTomb && id_eq(k, id)) {
        slot = v;
        break;
      }
      b = (b + 1) & a.hmask;
    }
    if (slot == kNone) {
      unk = 1;
    } else if (!a.seq[slot] || !(a.flags[slot] & GWAOI_SYNC_FROM_CLIENT)) {
      rej = 1;
      slot = kNone;
    } else {
      const uint4 v = a.rec[2 * i + 1];  // a client float that is NaN / +-Inf is dropped
      if (!finite_bits(v.x) || !finite_bits(v.z)) {
        nonf = 1;
        slot = kNone;
      }
    }
    a.res[i] = slot;
    if (slot != kNone) {
      const uint32_t old = atomicMin(&a.first[slot], i);
      if (old != kNone) rep = max(old, i);
    }
  }
  for (int o = 32; o > 0; o >>= 1) rep = min(rep, (uint32_t)__shfl_xor(rep, o, 64));
  if ((threadIdx.x & 63) == 0 && rep != kNone) atomicMin(&a.ctr[0], rep);
  wave_add(&a.ctr[1], unk);
  wave_add(&a.ctr[2], rej);
  wave_add(&a.ctr[3], nonf);
}

__global__ void k_ing_init(uint32_t* ctr, uint32_t n) {
  if (threadIdx.x < 4) ctr[threadIdx.x] = threadIdx.x ? 0u : n;
}

// first record of the batch [seg, n) naming each slot
__global__ void __launch_bounds__(kSy) k_ing_first(IngArgs a) {
  const uint32_t i = a.seg + blockIdx.x * kSy + threadIdx.x;
  if (i < a.n) {
    const uint32_t s = a.res[i];
    if (s != kNone) atomicMin(&a.first[s], i);
  }
}

// cut = the first record that repeats a slot (ctr[0], preset to n)
__global__ void __launch_bounds__(kSy) k_ing_cut(IngArgs a) {
  const uint32_t i = a.seg + blockIdx.x * kSy + threadIdx.x;
  uint32_t c = kNone;
  if (i < a.n) {
    const uint32_t s = a.res[i];
    if (s != kNone && a.first[s] != i) c = i;
  }
  for (int o = 32; o > 0; o >>= 1) c = min(c, (uint32_t)__shfl_xor(c, o, 64));
  if ((threadIdx.x & 63) == 0 && c != kNone) atomicMin(&a.ctr[0], c);
}

__device__ __forceinline__ bool ing_take(const IngArgs& a, uint32_t i, uint32_t cut) {
  return i < cut && a.res[i] != kNone;
}

__global__ void __launch_bounds__(kSy) k_ing_count(IngArgs a) {
  const uint32_t i = a.seg + blockIdx.x * kSy + threadIdx.x;
  const bool t = ing_take(a, i, min(a.ctr[0], a.n));
  const unsigned long long m = __ballot(t);
  __shared__ uint32_t wsum[kSy / 64];
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = (uint32_t)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int k = 0; k < kSy / 64; ++k) s += wsum[k];
    a.bcnt[blockIdx.x] = s;
  }
}

// accepted records of [seg, cut) -> the Moved batch in payload order, plus setPositionYaw's y/yaw and
// sifSyncNeighborClients (Entity.go:1195-1202, fromClient). Every record of [seg, n) resets `first`.
__global__ void __launch_bounds__(kSy) k_ing_emit(IngArgs a) {
  const uint32_t i = a.seg + blockIdx.x * kSy + threadIdx.x;
  const uint32_t cut = min(a.ctr[0], a.n);
  const bool t = ing_take(a, i, cut);
  const unsigned long long m = __ballot(t);
  __shared__ uint32_t wsum[kSy / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t pos = a.bcnt[blockIdx.x] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
  for (int k = 0; k < w; ++k) pos += wsum[k];
  if (i < a.n) {
    const uint32_t s = a.res[i];
    if (s != kNone) a.first[s] = kNone;
    if (t) {
      const uint4 v = a.rec[2 * i + 1];
      a.op_slot[pos] = s;
      a.op_x[pos] = __uint_as_float(v.x);
      a.op_z[pos] = __uint_as_float(v.z);
      a.y[s] = __uint_as_float(v.y);
      a.yaw[s] = __uint_as_float(v.w);
      a.flags[s] = (uint8_t)(a.flags[s] | GWAOI_SYNC_NEIGHBOR_CLIENTS);
    }
  }
}

__global__ void k_fill_u32(uint32_t* p, uint32_t v, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}

__global__ void __launch_bounds__(kSy) k_wl_pack_ingest(const uint4* __restrict__ ids, const float* __restrict__ x,
                                                        const float* __restrict__ z, uint32_t n, float yaw, uint4* out) {
  const uint32_t i = blockIdx.x * kSy + threadIdx.x;
  if (i >= n) return;
  out[2 * i] = ids[i];
  out[2 * i + 1] = make_uint4(__float_as_uint(x[i]), 0u, __float_as_uint(z[i]), __float_as_uint(yaw));
}

uint32_t blocks_for(uint64_t n) { return (uint32_t)std::max<uint64_t>(1, (n + kSy - 1) / kSy); }

}  // namespace

// ------------------------------------------------------------------------------------------------
struct SyncState {
  int device = 0;
  uint32_t cap = 0, n_gates = 0;
  uint8_t* flags = nullptr;
  uint16_t* gate = nullptr;
  uint4* cid = nullptr;
  uint4* eid = nullptr;
  float* y = nullptr;
  float* yaw = nullptr;
  // EntityID -> slot: host-owned open addressing table, mirrored to HBM
  uint32_t hcap = 0, n_tomb = 0;
  uint4* d_hb = nullptr;  // 2 x hcap: the buckets (k_ing_resolve)
  std::vector<uint4> h_hkey;
  std::vector<uint32_t> h_hval;
  std::vector<uint4> h_id_of;      // slot -> registered id (zero: none)
  std::vector<uint32_t> h_bucket;  // slot -> its bucket
  std::vector<uint32_t> dirty;
  std::vector<uint8_t> is_dirty;
  bool dirty_all = true;
  std::vector<uint32_t> h_mark;  // setters' last-wins dedup (generation stamps)
  uint32_t mark_gen = 0;
  // collect scratch
  uint32_t* cnt = nullptr;
  uint32_t cnt_n = 0;
  uint32_t* cpos = nullptr;
  uint32_t cpos_n = 0;
  uint32_t* ccs = nullptr;
  uint32_t ccs_n = 0;
  uint4* crec = nullptr;
  uint8_t* cgate = nullptr;
  uint32_t crec_n = 0, cgate_n = 0;
  uint4* ccid = nullptr;
  uint4* pk = nullptr;  // [2 cap]: k_sync_pack (direct fan-out)
  uint32_t ccid_n = 0;
  uint4* info = nullptr;
  uint64_t info_cap = 0;
  uint4* tstat = nullptr;  // per tile count-pass totals
  uint32_t tstat_n = 0;
  // direct fan-out (k_fan_dcount / k_fan_dwrite)
  uint32_t* gcnt = nullptr;
  uint64_t gcnt_cap = 0;
  uint8_t* wantj = nullptr;
  uint64_t wantj_cap = 0;
  uint32_t* tg = nullptr;
  uint64_t tg_cap = 0;
  int fan_mode = 0;  // gwaoi_debug_set_fanout_mode: 0 direct when n_gates <= kDirectGates, 1 pair list + partition
  uint64_t direct_reruns = 0;
  uint2* pairs = nullptr;
  uint64_t pairs_cap = 0;
  uint32_t* ghist = nullptr;
  uint64_t ghist_cap = 0;
  uint4* out = nullptr;
  uint64_t out_cap = 0;  // records
  uint8_t* h_out = nullptr;
  uint64_t h_out_cap = 0;
  uint32_t* d_goff = nullptr;
  uint32_t* h_small = nullptr;  // pinned (mapped): [0..3] counters, [4..] gate offsets
  uint32_t* d_small = nullptr;  // its device address (k_to_host), null: DMA copies instead
  std::vector<uint64_t> goff64;
  ScanCtx scan;
  uint32_t scan_words = 0;
  // ingest scratch
  uint8_t* d_payload = nullptr;
  uint64_t payload_cap = 0;
  uint32_t* res = nullptr;
  uint32_t res_cap = 0;
  uint32_t* first = nullptr;
  uint32_t* ictr = nullptr;
  uint32_t* bcnt = nullptr;
  uint32_t bcnt_cap = 0;
  uint32_t* op_slot = nullptr;
  float* op_x = nullptr;
  float* op_z = nullptr;
  // stage timing (gwaoi_set_timing)
  hipEvent_t tev[6] = {};
  gwaoi_sync_stats stats = {};
};

void sync_free(SyncState* s) {
  if (!s) return;
  void* p[] = {s->flags, s->gate, s->cid, s->eid, s->y, s->yaw, s->d_hb, s->cnt, s->cpos, s->ccs,
               s->crec, s->cgate, s->ccid, s->info, s->tstat, s->pairs, s->gcnt, s->wantj, s->tg,
               s->ghist, s->out, s->d_goff, s->scan.status, s->d_payload, s->res, s->first, s->ictr, s->bcnt,
               s->op_slot, s->op_x, s->op_z, s->pk};
  for (void* q : p)
    if (q) hipFree(q);
  if (s->h_out) hipHostFree(s->h_out);
  if (s->h_small) hipHostFree(s->h_small);
  for (hipEvent_t e : s->tev)
    if (e) hipEventDestroy(e);
  delete s;
}

namespace {

#define SCHK(x)                                                                               \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      gw::set_error("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_));           \
      return GWAOI_ERR_HIP;                                                                   \
    }                                                                                         \
  } while (0)
#define SRCHK(x)                   \
  do {                             \
    int r_ = (x);                  \
    if (r_ != GWAOI_OK) return r_; \
  } while (0)

template <class T>
int dgrow(T** p, uint64_t* cap, uint64_t need) {
  if (*p && *cap >= need) return GWAOI_OK;
  if (*p) hipFree(*p);
  *p = nullptr;
  const uint64_t n = std::max<uint64_t>(need + need / 4, 1024);
  if (hipMalloc((void**)p, n * sizeof(T)) != hipSuccess) {
    *p = nullptr;
    *cap = 0;
    set_error("hipMalloc(%llu bytes) failed", (unsigned long long)(n * sizeof(T)));
    return GWAOI_ERR_NOMEM;
  }
  *cap = n;
  return GWAOI_OK;
}

template <class T>
int dgrow32(T** p, uint32_t* cap, uint64_t need) {
  uint64_t c = *cap;
  SRCHK(dgrow(p, &c, need));
  *cap = (uint32_t)std::min<uint64_t>(c, 0xFFFFFFFFull);
  return GWAOI_OK;
}

int ensure_scan(SyncState* s, uint32_t n) {
  const uint32_t w = scan_part_words(n) + 2;
  if (s->scan.status && s->scan_words >= w) return GWAOI_OK;
  if (s->scan.status) hipFree(s->scan.status);
  s->scan.status = nullptr;
  uint64_t c = 0;
  SRCHK(dgrow(&s->scan.status, &c, std::max<uint32_t>(w, 1026)));
  s->scan_words = (uint32_t)c;
  return GWAOI_OK;
}

int get_state(gwaoi_mgr* m, MgrView* v, SyncState** s) {
  SRCHK(mgr_view(m, v));
  *s = *v->sync;
  if (!*s) {
    set_error("sync state not enabled (gwaoi_sync_enable)");
    return GWAOI_ERR_STATE;
  }
  return GWAOI_OK;
}

// indices of the entries that win for their slot (the last one), in array order
int last_wins(SyncState* s, const uint32_t* slots, uint32_t n, std::vector<uint32_t>* idx) {
  for (uint32_t i = 0; i < n; ++i)
    if (slots[i] >= s->cap) {
      set_error("slot %u >= capacity %u", slots[i], s->cap);
      return GWAOI_ERR_INVALID;
    }
  if (++s->mark_gen == 0) {
    std::fill(s->h_mark.begin(), s->h_mark.end(), 0u);
    s->mark_gen = 1;
  }
  idx->clear();
  for (uint32_t i = n; i-- > 0;) {
    if (s->h_mark[slots[i]] == s->mark_gen) continue;
    s->h_mark[slots[i]] = s->mark_gen;
    idx->push_back(i);
  }
  std::reverse(idx->begin(), idx->end());
  return GWAOI_OK;
}

// upload host arrays, run k_sync_scatter, free (setters are the rare path)
struct Up {
  std::vector<void*> bufs;
  ~Up() {
    for (void* p : bufs) hipFree(p);
  }
  template <class T>
  int put(const std::vector<T>& h, const T** d) {
    *d = nullptr;
    if (h.empty()) return GWAOI_OK;
    void* p = nullptr;
    if (hipMalloc(&p, h.size() * sizeof(T)) != hipSuccess) {
      set_error("hipMalloc failed");
      return GWAOI_ERR_NOMEM;
    }
    bufs.push_back(p);
    SCHK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    *d = (const T*)p;
    return GWAOI_OK;
  }
};

int run_scatter(const MgrView& v, SyncState* s, ScatArgs a) {
  a.flags = s->flags;
  a.t_gate = s->gate;
  a.t_cid = s->cid;
  a.t_eid = s->eid;
  a.t_y = s->y;
  a.t_yaw = s->yaw;
  if (a.n) hipLaunchKernelGGL(k_sync_scatter, dim3(blocks_for(a.n)), dim3(kSy), 0, v.stream, a);
  SCHK(hipGetLastError());
  SCHK(hipStreamSynchronize(v.stream));
  return GWAOI_OK;
}

void mark_dirty(SyncState* s, uint32_t b) {
  if (s->dirty_all || s->is_dirty[b]) return;
  s->is_dirty[b] = 1;
  s->dirty.push_back(b);
  if (s->dirty.size() > s->hcap / 16) s->dirty_all = true;
}

// rebuild the host table without tombstones
void rehash(SyncState* s) {
  std::fill(s->h_hval.begin(), s->h_hval.end(), kHEmpty);
  const uint32_t mask = s->hcap - 1;
  for (uint32_t slot = 0; slot < s->cap; ++slot) {
    const uint4 k = s->h_id_of[slot];
    if (id_zero(k)) continue;
    uint32_t b = id_hash(k) & mask;
    while (s->h_hval[b] != kHEmpty) b = (b + 1) & mask;
    s->h_hkey[b] = k;
    s->h_hval[b] = slot;
    s->h_bucket[slot] = b;
  }
  s->n_tomb = 0;
  s->dirty_all = true;
}

int upload_hash(const MgrView& v, SyncState* s) {
  if (s->dirty_all) {
    std::vector<uint4> hb(2 * (size_t)s->hcap);
    for (uint32_t b = 0; b < s->hcap; ++b) {
      hb[2 * (size_t)b] = s->h_hkey[b];
      hb[2 * (size_t)b + 1] = make_uint4(s->h_hval[b], 0u, 0u, 0u);
    }
    SCHK(hipMemcpyAsync(s->d_hb, hb.data(), hb.size() * sizeof(uint4), hipMemcpyHostToDevice, v.stream));
    SCHK(hipStreamSynchronize(v.stream));
    for (uint32_t b : s->dirty) s->is_dirty[b] = 0;
    s->dirty.clear();
    s->dirty_all = false;
    return GWAOI_OK;
  }
  if (s->dirty.empty()) return GWAOI_OK;
  std::vector<uint32_t> idx(s->dirty), val(idx.size());
  std::vector<uint4> key(idx.size());
  for (size_t i = 0; i < idx.size(); ++i) {
    key[i] = s->h_hkey[idx[i]];
    val[i] = s->h_hval[idx[i]];
    s->is_dirty[idx[i]] = 0;
  }
  s->dirty.clear();
  Up up;
  const uint32_t *d_idx, *d_val;
  const uint4* d_key;
  SRCHK(up.put(idx, &d_idx));
  SRCHK(up.put(val, &d_val));
  SRCHK(up.put(key, &d_key));
  hipLaunchKernelGGL(k_hash_scatter, dim3(blocks_for(idx.size())), dim3(kSy), 0, v.stream, d_idx, d_key, d_val,
                     (uint32_t)idx.size(), s->d_hb);
  SCHK(hipGetLastError());
  SCHK(hipStreamSynchronize(v.stream));
  return GWAOI_OK;
}

void add_collect_stats(SyncState* s, uint64_t records, uint32_t entities) {
  float t01, t12, t34, t45;
  if (hipEventElapsedTime(&t01, s->tev[0], s->tev[1]) != hipSuccess ||
      hipEventElapsedTime(&t12, s->tev[1], s->tev[2]) != hipSuccess ||
      hipEventElapsedTime(&t34, s->tev[3], s->tev[4]) != hipSuccess ||
      hipEventElapsedTime(&t45, s->tev[4], s->tev[5]) != hipSuccess)
    return;
  s->stats.collects++;
  s->stats.ms_client_grid += t01;
  s->stats.ms_count += t12;
  s->stats.ms_write += t34;
  s->stats.ms_gate += t45;
  s->stats.records += records;
  s->stats.entities += entities;
}

// The direct fan-out (n_gates <= kDirectGates), after the client sub-grid: count pass (per-gate counts,
// flags cleared) -> scan of the (gate, tile) totals -> write pass straight into the gate packets. The
// packet buffer keeps the previous collect's size: no host round trip between the passes; a collect
// with more records re-runs the write pass into a grown buffer.
int collect_direct(const MgrView& v, SyncState* s, FanArgs f, uint32_t opts, gwaoi_sync_out* out) {
  hipStream_t st = v.stream;
  const uint32_t ntiles = v.ntiles, G = s->n_gates, bound = v.rec_bound;
  const uint32_t gstride = (G + 3u) & ~3u;
  SRCHK(dgrow(&s->gcnt, &s->gcnt_cap, ((uint64_t)bound + 1) * gstride));
  SRCHK(dgrow(&s->wantj, &s->wantj_cap, (uint64_t)bound + 1));
  const uint64_t tgn = (uint64_t)G * ntiles + 1;
  SRCHK(dgrow(&s->tg, &s->tg_cap, tgn));
  SRCHK(ensure_scan(s, (uint32_t)tgn));
  if (!s->out) SRCHK(dgrow(&s->out, &s->out_cap, 3u * 65536u));
  if (!s->pk) {
    if (hipMalloc((void**)&s->pk, (size_t)s->cap * 32) != hipSuccess) {
      s->pk = nullptr;
      set_error("collect_sync: hipMalloc(%llu) failed", (unsigned long long)s->cap * 32);
      return GWAOI_ERR_NOMEM;
    }
  }
  f.pk = s->pk;
  f.n_gates = G;
  f.gstride = gstride;
  f.gcnt = s->gcnt;
  f.wantj = s->wantj;
  f.tg = s->tg;
  f.ntiles = ntiles;
  if (v.timing) SCHK(hipEventRecord(s->tev[1], st));
  hipLaunchKernelGGL(k_sync_pack, dim3(std::min<uint32_t>(blocks_for(s->cap), 4096)), dim3(kSy), 0, st, s->flags,
                     (const uint16_t*)s->gate, (const uint4*)s->eid, (const float*)s->y, (const float*)s->yaw, s->cap,
                     f.clear, s->pk);
  hipLaunchKernelGGL(k_fan_dcount, dim3(ntiles), dim3(kSy), 0, st, f);
  // (fused into one single-block kernel, the totals, scan and gate offsets measured slower: the count
  // stage 0.115 -> 0.119 ms, r04_c26)
  hipLaunchKernelGGL(k_fan_total, dim3(1), dim3(1024), 0, st, (const uint4*)s->tstat, ntiles, s->ictr + 8,
                     (unsigned long long*)(s->ictr + 10));
  launch_scan(s->scan, s->tg, (uint32_t)tgn, st);
  hipLaunchKernelGGL(k_fan_goff, dim3(1), dim3(kDirectGates + 1), 0, st, (const uint32_t*)s->tg, ntiles, G, s->d_goff);
  if (v.timing) SCHK(hipEventRecord(s->tev[2], st));
  auto write = [&]() -> int {
    f.out = s->out;
    f.out_cap = (uint32_t)std::min<uint64_t>(s->out_cap / 3, 0xFFFFFFFFull);
    if (v.timing) SCHK(hipEventRecord(s->tev[3], st));
    hipLaunchKernelGGL(k_fan_dwrite, dim3(ntiles), dim3(kSy), 0, st, f);
    if (v.timing) {
      SCHK(hipEventRecord(s->tev[4], st));
      SCHK(hipEventRecord(s->tev[5], st));
    }
    SCHK(hipGetLastError());
    if (s->d_small) {
      hipLaunchKernelGGL(k_to_host, dim3(1), dim3(64), 0, st, (const uint32_t*)s->d_goff, G + 1, 8u,
                         (const uint32_t*)(s->ictr + 8), 4u, 4u, s->d_small);
    } else {
      SCHK(hipMemcpyAsync(s->h_small + 8, s->d_goff, (G + 1) * 4, hipMemcpyDeviceToHost, st));
      SCHK(hipMemcpyAsync(s->h_small + 4, s->ictr + 8, 16, hipMemcpyDeviceToHost, st));
    }
    SCHK(hipStreamSynchronize(st));
    return GWAOI_OK;
  };
  SRCHK(write());
  uint64_t M64;
  memcpy(&M64, s->h_small + 6, sizeof M64);
  if (M64 > v.index_limit) {  // record indices are uint32: the scanned offsets wrapped
    set_error("collect_sync: %llu records exceed the fan-out's uint32 offsets (limit %llu)", (unsigned long long)M64,
              (unsigned long long)v.index_limit);
    return GWAOI_ERR_NOMEM;
  }
  const uint32_t M = s->h_small[8 + G];
  if ((uint64_t)M * 3 > s->out_cap) {  // more records than the previous collect's buffer: grown, written again
    SRCHK(dgrow(&s->out, &s->out_cap, (uint64_t)M * 3));
    s->direct_reruns++;
    SRCHK(write());
  }
  out->n_entities = s->h_small[4];
  for (uint32_t k = 0; k <= G; ++k) s->goff64[k] = s->h_small[8 + k];
  out->n_records = M;
  out->d_records = (const uint8_t*)s->out;
  if (M && (opts & GWAOI_COLLECT_HOST)) {
    const uint64_t bytes = (uint64_t)M * GWAOI_SYNC_RECORD_BYTES;
    if (s->h_out_cap < bytes) {
      if (s->h_out) hipHostFree(s->h_out);
      s->h_out = nullptr;
      s->h_out_cap = 0;
      const uint64_t nb = bytes + bytes / 4;
      if (hipHostMalloc((void**)&s->h_out, nb, hipHostMallocDefault) != hipSuccess) {
        s->h_out = nullptr;
        set_error("collect_sync: hipHostMalloc(%llu) failed", (unsigned long long)nb);
        return GWAOI_ERR_NOMEM;
      }
      s->h_out_cap = nb;
    }
    SCHK(hipMemcpyAsync(s->h_out, s->out, bytes, hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    out->records = s->h_out;
  }
  if (v.timing) add_collect_stats(s, M, out->n_entities);
  return GWAOI_OK;
}

}  // namespace
}  // namespace gw

using gw::SyncState;

extern "C" {

int gwaoi_sync_enable(gwaoi_mgr* m, uint32_t n_gates) {
  gw::MgrView v;
  SRCHK(gw::mgr_view(m, &v));
  if (*v.sync) {
    gw::set_error("sync_enable: already enabled");
    return GWAOI_ERR_STATE;
  }
  if (n_gates == 0 || n_gates > GWAOI_SYNC_MAX_GATES) {
    gw::set_error("sync_enable: n_gates %u not in [1, %u]", n_gates, GWAOI_SYNC_MAX_GATES);
    return GWAOI_ERR_INVALID;
  }
  SyncState* s = new (std::nothrow) SyncState();
  if (!s) return GWAOI_ERR_NOMEM;
  s->device = v.device;
  s->cap = v.cap;
  s->n_gates = n_gates;
  const size_t C = v.cap;
  s->hcap = 1024;
  while (s->hcap < 2 * C) s->hcap <<= 1;
  bool ok = hipMalloc((void**)&s->flags, C) == hipSuccess && hipMalloc((void**)&s->gate, C * 2) == hipSuccess &&
            hipMalloc((void**)&s->cid, C * 16) == hipSuccess && hipMalloc((void**)&s->eid, C * 16) == hipSuccess &&
            hipMalloc((void**)&s->y, C * 4) == hipSuccess && hipMalloc((void**)&s->yaw, C * 4) == hipSuccess &&
            hipMalloc((void**)&s->d_hb, (size_t)s->hcap * 32) == hipSuccess &&
            hipMalloc((void**)&s->first, C * 4) == hipSuccess && hipMalloc((void**)&s->ictr, 64) == hipSuccess &&
            hipHostMalloc((void**)&s->h_small, (8 + GWAOI_SYNC_MAX_GATES + 1) * 4,
                          hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
            hipMalloc((void**)&s->d_goff, (GWAOI_SYNC_MAX_GATES + 1) * 4) == hipSuccess;
  if (ok) {
    ok = hipMemsetAsync(s->flags, 0, C, v.stream) == hipSuccess &&
         hipMemsetAsync(s->gate, 0xFF, C * 2, v.stream) == hipSuccess &&
         hipMemsetAsync(s->cid, 0, C * 16, v.stream) == hipSuccess &&
         hipMemsetAsync(s->eid, 0, C * 16, v.stream) == hipSuccess &&
         hipMemsetAsync(s->y, 0, C * 4, v.stream) == hipSuccess && hipMemsetAsync(s->yaw, 0, C * 4, v.stream) == hipSuccess &&
         hipMemsetAsync(s->first, 0xFF, C * 4, v.stream) == hipSuccess &&
         hipMemsetAsync(s->d_hb, 0xFF, (size_t)s->hcap * 32, v.stream) == hipSuccess &&
         hipStreamSynchronize(v.stream) == hipSuccess;
  }
  if (ok) {
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, s->h_small, 0) == hipSuccess) s->d_small = (uint32_t*)dp;
    else (void)hipGetLastError();
  }
  if (!ok) {
    gw::set_error("sync_enable: device allocation failed");
    gw::sync_free(s);
    return GWAOI_ERR_NOMEM;
  }
  s->h_hkey.assign(s->hcap, make_uint4(0, 0, 0, 0));
  s->h_hval.assign(s->hcap, gw::kHEmpty);
  s->h_id_of.assign(C, make_uint4(0, 0, 0, 0));
  s->h_bucket.assign(C, gw::kNone);
  s->is_dirty.assign(s->hcap, 0);
  s->h_mark.assign(C, 0);
  s->dirty_all = false;  // device table already empty
  for (hipEvent_t& e : s->tev)
    if (hipEventCreate(&e) != hipSuccess) {
      gw::set_error("sync_enable: hipEventCreate failed");
      gw::sync_free(s);
      return GWAOI_ERR_HIP;
    }
  *v.sync = s;
  return GWAOI_OK;
}

int gwaoi_sync_get_tables(gwaoi_mgr* m, gwaoi_sync_tables* out) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::get_state(m, &v, &s));
  if (!out) return GWAOI_ERR_INVALID;
  out->flags = s->flags;
  out->gate = s->gate;
  out->client_id = (uint8_t*)s->cid;
  out->entity_id = (uint8_t*)s->eid;
  out->y = s->y;
  out->yaw = s->yaw;
  out->capacity = s->cap;
  out->n_gates = s->n_gates;
  return GWAOI_OK;
}

int gwaoi_sync_set_entities(gwaoi_mgr* m, const uint32_t* slots, const uint8_t* ids, uint32_t n) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::get_state(m, &v, &s));
  if (n && (!slots || !ids)) {
    gw::set_error("sync_set_entities: null array");
    return GWAOI_ERR_INVALID;
  }
  std::vector<uint32_t> idx;
  SRCHK(gw::last_wins(s, slots, n, &idx));
  const uint32_t mask = s->hcap - 1;
  auto lookup = [&](const uint4& k) -> uint32_t {  // slot holding id k now, or kNone
    for (uint32_t b = gw::id_hash(k) & mask;; b = (b + 1) & mask) {
      const uint32_t hv = s->h_hval[b];
      if (hv == gw::kHEmpty) return gw::kNone;
      if (hv != gw::kHTomb && gw::id_eq(s->h_hkey[b], k)) return hv;
    }
  };
  // validate first, so a failing call changes nothing: in the state after the call no id may be
  // held by two slots (an id may move to another slot in the same call if its old slot changes too)
  {
    std::unordered_map<uint64_t, std::vector<std::pair<uint4, uint32_t>>> fresh;  // new ids of the call
    std::unordered_map<uint32_t, bool> in_call;
    for (uint32_t i : idx) in_call[slots[i]] = true;
    for (uint32_t i : idx) {
      uint4 k;
      memcpy(&k, ids + (size_t)16 * i, 16);
      if (gw::id_zero(k)) continue;
      auto& bucket = fresh[((uint64_t)k.y << 32 | k.x) ^ ((uint64_t)k.w << 32 | k.z)];
      for (auto& e : bucket)
        if (gw::id_eq(e.first, k)) {
          gw::set_error("sync_set_entities: slots %u and %u are given the same entity id", e.second, slots[i]);
          return GWAOI_ERR_INVALID;
        }
      bucket.push_back({k, slots[i]});
      const uint32_t owner = lookup(k);
      if (owner != gw::kNone && owner != slots[i] && !in_call.count(owner)) {
        gw::set_error("sync_set_entities: entity id of slot %u is already registered to slot %u", slots[i], owner);
        return GWAOI_ERR_INVALID;
      }
    }
  }
  std::vector<uint32_t> us;
  std::vector<uint4> uk;
  std::vector<uint8_t> reset;  // the slot's entity changes: its flags and client are reset
  // pass 1: unregister the slots' old ids (so ids may move between slots within one call)
  for (uint32_t i : idx) {
    const uint32_t slot = slots[i];
    uint4 k;
    memcpy(&k, ids + (size_t)16 * i, 16);
    const uint4 old = s->h_id_of[slot];
    if (!gw::id_zero(old) && !gw::id_eq(old, k)) {
      const uint32_t b = s->h_bucket[slot];
      s->h_hval[b] = gw::kHTomb;
      ++s->n_tomb;
      gw::mark_dirty(s, b);
      s->h_id_of[slot] = make_uint4(0, 0, 0, 0);
      s->h_bucket[slot] = gw::kNone;
    }
  }
  // pass 2: register the new ones
  int rc = GWAOI_OK;
  for (uint32_t i : idx) {
    const uint32_t slot = slots[i];
    uint4 k;
    memcpy(&k, ids + (size_t)16 * i, 16);
    us.push_back(slot);
    uk.push_back(k);
    reset.push_back(gw::id_eq(s->h_id_of[slot], k) ? 0 : 1);
    if (gw::id_zero(k) || gw::id_eq(s->h_id_of[slot], k)) continue;
    uint32_t b = gw::id_hash(k) & mask, free_b = gw::kNone;
    bool dup = false;
    for (;;) {
      const uint32_t hv = s->h_hval[b];
      if (hv == gw::kHEmpty) break;
      if (hv == gw::kHTomb) {
        if (free_b == gw::kNone) free_b = b;
      } else if (gw::id_eq(s->h_hkey[b], k)) {
        dup = true;
        break;
      }
      b = (b + 1) & mask;
    }
    if (dup) {  // excluded by the validation above
      gw::set_error("sync_set_entities: internal: entity id of slot %u is already registered to slot %u", slot,
                    s->h_hval[b]);
      rc = GWAOI_ERR_INVALID;
      uk.back() = make_uint4(0, 0, 0, 0);
      continue;
    }
    if (free_b != gw::kNone) {
      b = free_b;
      --s->n_tomb;
    }
    s->h_hkey[b] = k;
    s->h_hval[b] = slot;
    s->h_id_of[slot] = k;
    s->h_bucket[slot] = b;
    gw::mark_dirty(s, b);
  }
  if (s->n_tomb > s->hcap / 4) gw::rehash(s);
  gw::Up up;
  gw::ScatArgs a = {};
  a.mode = 0;
  a.n = (uint32_t)us.size();
  SRCHK(up.put(us, &a.slot));
  SRCHK(up.put(uk, &a.id));
  SRCHK(up.put(reset, &a.f));
  SRCHK(gw::run_scatter(v, s, a));
  return rc;
}

int gwaoi_sync_set_clients(gwaoi_mgr* m, const uint32_t* slots, const uint16_t* gates, const uint8_t* cids,
                           uint32_t n) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::get_state(m, &v, &s));
  if (n && (!slots || !gates || !cids)) {
    gw::set_error("sync_set_clients: null array");
    return GWAOI_ERR_INVALID;
  }
  for (uint32_t i = 0; i < n; ++i)
    if (gates[i] != GWAOI_SYNC_NO_CLIENT && gates[i] >= s->n_gates) {
      gw::set_error("sync_set_clients: gate index %u >= n_gates %u", gates[i], s->n_gates);
      return GWAOI_ERR_INVALID;
    }
  std::vector<uint32_t> idx;
  SRCHK(gw::last_wins(s, slots, n, &idx));
  std::vector<uint32_t> us;
  std::vector<uint16_t> ug;
  std::vector<uint4> uc;
  for (uint32_t i : idx) {
    uint4 k;
    memcpy(&k, cids + (size_t)16 * i, 16);
    us.push_back(slots[i]);
    ug.push_back(gates[i]);
    uc.push_back(k);
  }
  gw::Up up;
  gw::ScatArgs a = {};
  a.mode = 1;
  a.n = (uint32_t)us.size();
  SRCHK(up.put(us, &a.slot));
  SRCHK(up.put(ug, &a.gate));
  SRCHK(up.put(uc, &a.id));
  return gw::run_scatter(v, s, a);
}

int gwaoi_sync_set_syncing(gwaoi_mgr* m, const uint32_t* slots, const uint8_t* on, uint32_t n) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::get_state(m, &v, &s));
  if (n && (!slots || !on)) {
    gw::set_error("sync_set_syncing: null array");
    return GWAOI_ERR_INVALID;
  }
  std::vector<uint32_t> idx;
  SRCHK(gw::last_wins(s, slots, n, &idx));
  std::vector<uint32_t> us;
  std::vector<uint8_t> uf;
  for (uint32_t i : idx) {
    us.push_back(slots[i]);
    uf.push_back(on[i] ? 1 : 0);
  }
  gw::Up up;
  gw::ScatArgs a = {};
  a.mode = 2;
  a.n = (uint32_t)us.size();
  SRCHK(up.put(us, &a.slot));
  SRCHK(up.put(uf, &a.f));
  return gw::run_scatter(v, s, a);
}

int gwaoi_sync_mark(gwaoi_mgr* m, const uint32_t* slots, const float* y, const float* yaw, const uint8_t* flags,
                    uint32_t n) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::get_state(m, &v, &s));
  if (n && (!slots || !y || !yaw || !flags)) {
    gw::set_error("sync_mark: null array");
    return GWAOI_ERR_INVALID;
  }
  for (uint32_t i = 0; i < n; ++i)
    if (flags[i] & ~(GWAOI_SYNC_OWN_CLIENT | GWAOI_SYNC_NEIGHBOR_CLIENTS)) {
      gw::set_error("sync_mark: flags 0x%x: only GWAOI_SYNC_OWN_CLIENT | GWAOI_SYNC_NEIGHBOR_CLIENTS", flags[i]);
      return GWAOI_ERR_INVALID;
    }
  std::vector<uint32_t> idx;
  SRCHK(gw::last_wins(s, slots, n, &idx));
  // flags accumulate over every entry of a slot (|=), y/yaw: the last entry
  std::vector<uint8_t> acc(idx.size());
  {
    std::vector<std::pair<uint32_t, uint32_t>> sp;
    sp.reserve(idx.size());
    for (uint32_t k = 0; k < idx.size(); ++k) sp.push_back({slots[idx[k]], k});
    std::sort(sp.begin(), sp.end());
    for (uint32_t i = 0; i < n; ++i) {
      auto it = std::lower_bound(sp.begin(), sp.end(), std::make_pair(slots[i], 0u));
      acc[it->second] |= flags[i];
    }
  }
  std::vector<uint32_t> us;
  std::vector<float> uy, uyaw;
  for (uint32_t k = 0; k < idx.size(); ++k) {
    us.push_back(slots[idx[k]]);
    uy.push_back(y[idx[k]]);
    uyaw.push_back(yaw[idx[k]]);
  }
  gw::Up up;
  gw::ScatArgs a = {};
  a.mode = 3;
  a.n = (uint32_t)us.size();
  SRCHK(up.put(us, &a.slot));
  SRCHK(up.put(uy, &a.y));
  SRCHK(up.put(uyaw, &a.yaw));
  SRCHK(up.put(acc, &a.f));
  return gw::run_scatter(v, s, a);
}

int gwaoi_collect_sync(gwaoi_mgr* m, uint32_t opts, gwaoi_sync_out* out) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::mgr_grid_current(m));  // the walks read the grid
  SRCHK(gw::get_state(m, &v, &s));
  if (!out) return GWAOI_ERR_INVALID;
  if (v.pending) {
    gw::set_error("collect_sync: ops are staged; run gwaoi_tick first (the reference collects after the tick)");
    return GWAOI_ERR_STATE;
  }
  memset(out, 0, sizeof *out);
  out->n_gates = s->n_gates;
  s->goff64.assign(s->n_gates + 1, 0);
  out->gate_off = s->goff64.data();
  hipStream_t st = v.stream;
  const bool direct = s->n_gates <= gw::kDirectGates && s->fan_mode == 0 && v.g.rec && v.ntiles;
  if (!(opts & GWAOI_COLLECT_KEEP_FLAGS) && !direct) {  // absent slots: their sync bits clear without records
    hipLaunchKernelGGL(gw::k_clear_absent, dim3(std::min<uint32_t>(gw::blocks_for(s->cap), 4096)), dim3(gw::kSy), 0, st,
                       s->flags, v.seq, s->cap);
    SCHK(hipGetLastError());
  }
  if (!v.g.rec) {  // no pass has run: nothing is present
    SCHK(hipStreamSynchronize(st));
    return GWAOI_OK;
  }
  const uint32_t bound = v.rec_bound;
  SRCHK(gw::ensure_scan(s, bound + 1));
  // client sub-grid
  SRCHK(gw::dgrow32(&s->cpos, &s->cpos_n, (uint64_t)bound + 1));
  SRCHK(gw::dgrow32(&s->ccs, &s->ccs_n, (uint64_t)v.ncells + 1));
  SRCHK(gw::dgrow32(&s->crec, &s->crec_n, s->cap));
  SRCHK(gw::dgrow32(&s->cgate, &s->cgate_n, s->cap));
  SRCHK(gw::dgrow32(&s->ccid, &s->ccid_n, s->cap));
  gw::ClientGridArgs cg = {};
  cg.rec = v.g.rec;
  cg.cs = v.g.cs;
  cg.rec_count = v.rec_count;
  cg.rec_bound = bound;
  cg.ncells = v.ncells;
  cg.gate = s->gate;
  cg.cpos = s->cpos;
  cg.ccs = s->ccs;
  cg.crec = s->crec;
  cg.cgate = s->cgate;
  cg.cid = s->cid;
  cg.ccid = s->ccid;
  const uint32_t fan_blocks = std::min<uint32_t>(gw::blocks_for((uint64_t)bound + 1), 8192);
  SRCHK(gw::ensure_scan(s, std::max(bound, v.ncells) + 1));
  if (v.timing) SCHK(hipEventRecord(s->tev[0], st));
  hipLaunchKernelGGL(gw::k_cg_flag, dim3(fan_blocks), dim3(gw::kSy), 0, st, cg);
  gw::launch_scan(s->scan, s->cpos, bound + 1, st);
  hipLaunchKernelGGL(gw::k_cg_build, dim3(fan_blocks), dim3(gw::kSy), 0, st, cg);
  gw::FanArgs f = {};
  f.ccs = s->ccs;
  f.crec = s->crec;
  f.cgate = s->cgate;
  f.cpos = s->cpos;
  f.ccid = s->ccid;
  f.eid = s->eid;
  f.y = s->y;
  f.yaw = s->yaw;
  f.g = v.g;
  f.rec_count = v.rec_count;
  f.rec_bound = bound;
  f.pos_x = v.pos_x;
  f.pos_z = v.pos_z;
  f.space_of = v.space_of;
  f.flags = s->flags;
  f.gate = s->gate;
  f.clear = !(opts & GWAOI_COLLECT_KEEP_FLAGS);
  const uint32_t ntiles = v.ntiles;
  if (!ntiles) return GWAOI_OK;
  SRCHK(gw::dgrow32(&s->tstat, &s->tstat_n, ntiles));
  f.tstat = s->tstat;
  if (direct) return gw::collect_direct(v, s, f, opts, out);
  // pair list + gate partition
  SRCHK(gw::dgrow32(&s->cnt, &s->cnt_n, (uint64_t)bound + 1));
  SRCHK(gw::dgrow(&s->info, &s->info_cap, 2 * ((uint64_t)bound + 1)));
  f.info = s->info;
  f.cnt = s->cnt;
  SCHK(hipMemsetAsync(s->cnt, 0, ((size_t)bound + 1) * 4, st));
  if (v.timing) SCHK(hipEventRecord(s->tev[1], st));
  hipLaunchKernelGGL(gw::k_fan_tile<false>, dim3(ntiles), dim3(gw::kSy), 0, st, f);
  hipLaunchKernelGGL(gw::k_fan_total, dim3(1), dim3(1024), 0, st, (const uint4*)s->tstat, ntiles, s->ictr + 8,
                     (unsigned long long*)(s->ictr + 10));
  gw::launch_scan(s->scan, s->cnt, bound + 1, st);
  if (v.timing) SCHK(hipEventRecord(s->tev[2], st));
  SCHK(hipMemcpyAsync(s->h_small, s->cnt + bound, 4, hipMemcpyDeviceToHost, st));
  // [4] entities collected, [6..7] the 64-bit pair total
  SCHK(hipMemcpyAsync(s->h_small + 4, s->ictr + 8, 16, hipMemcpyDeviceToHost, st));
  SCHK(hipStreamSynchronize(st));
  uint64_t M64;
  memcpy(&M64, s->h_small + 6, sizeof M64);
  if (M64 > v.index_limit) {  // pair offsets are uint32: the scanned counts would have wrapped
    gw::set_error("collect_sync: %llu records exceed the fan-out's uint32 offsets (limit %llu)",
                  (unsigned long long)M64, (unsigned long long)v.index_limit);
    return GWAOI_ERR_NOMEM;
  }
  const uint32_t M = s->h_small[0];
  out->n_entities = s->h_small[4];
  if (M == 0) {
    if (f.clear) {  // nothing to write, but the flags of the collected entities still clear
      f.off = s->cnt;
      hipLaunchKernelGGL(gw::k_fan_tile<true>, dim3(ntiles), dim3(gw::kSy), 0, st, f);
      SCHK(hipStreamSynchronize(st));
    }
    return GWAOI_OK;
  }
  SRCHK(gw::dgrow(&s->pairs, &s->pairs_cap, M));
  f.off = s->cnt;
  f.pairs = s->pairs;
  if (v.timing) SCHK(hipEventRecord(s->tev[3], st));
  hipLaunchKernelGGL(gw::k_fan_tile<true>, dim3(ntiles), dim3(gw::kSy), 0, st, f);
  if (v.timing) SCHK(hipEventRecord(s->tev[4], st));

  gw::GateArgs g = {};
  g.pairs = s->pairs;
  g.cgate = s->cgate;
  g.n = M;
  g.nchunks = (M + gw::kGChunk - 1) / gw::kGChunk;
  g.n_gates = s->n_gates;
  g.bits = 1;
  while ((1u << g.bits) < s->n_gates) ++g.bits;
  const uint64_t hn = (uint64_t)g.nchunks * s->n_gates + 1;
  SRCHK(gw::dgrow(&s->ghist, &s->ghist_cap, hn));
  SRCHK(gw::ensure_scan(s, (uint32_t)hn));
  g.ghist = s->ghist;
  g.ccid = s->ccid;
  g.info = s->info;
  SRCHK(gw::dgrow(&s->out, &s->out_cap, (uint64_t)M * 3));
  g.out = s->out;
  g.goff = s->d_goff;
  hipLaunchKernelGGL(gw::k_gate_hist, dim3(g.nchunks), dim3(gw::kSy), 0, st, g);
  gw::launch_scan(s->scan, s->ghist, (uint32_t)hn, st);
  hipLaunchKernelGGL(gw::k_gate_scatter, dim3(g.nchunks), dim3(gw::kSy), 0, st, g);
  hipLaunchKernelGGL(gw::k_gate_offsets, dim3(1), dim3(GWAOI_SYNC_MAX_GATES + 64), 0, st, g);
  if (v.timing) SCHK(hipEventRecord(s->tev[5], st));
  SCHK(hipGetLastError());
  SCHK(hipMemcpyAsync(s->h_small + 8, s->d_goff, (s->n_gates + 1) * 4, hipMemcpyDeviceToHost, st));
  const uint64_t bytes = (uint64_t)M * GWAOI_SYNC_RECORD_BYTES;
  if (opts & GWAOI_COLLECT_HOST) {
    if (s->h_out_cap < bytes) {
      if (s->h_out) hipHostFree(s->h_out);
      s->h_out = nullptr;
      s->h_out_cap = 0;
      const uint64_t nb = bytes + bytes / 4;
      if (hipHostMalloc((void**)&s->h_out, nb, hipHostMallocDefault) != hipSuccess) {
        s->h_out = nullptr;
        gw::set_error("collect_sync: hipHostMalloc(%llu) failed", (unsigned long long)nb);
        return GWAOI_ERR_NOMEM;
      }
      s->h_out_cap = nb;
    }
    SCHK(hipMemcpyAsync(s->h_out, s->out, bytes, hipMemcpyDeviceToHost, st));
    out->records = s->h_out;
  }
  SCHK(hipStreamSynchronize(st));
  for (uint32_t k = 0; k <= s->n_gates; ++k) s->goff64[k] = s->h_small[8 + k];
  out->n_records = M;
  out->d_records = (const uint8_t*)s->out;
  if (v.timing) {  // the stream was synchronised above: every event is complete
    float t01, t12, t34, t45;
    SCHK(hipEventElapsedTime(&t01, s->tev[0], s->tev[1]));
    SCHK(hipEventElapsedTime(&t12, s->tev[1], s->tev[2]));
    SCHK(hipEventElapsedTime(&t34, s->tev[3], s->tev[4]));
    SCHK(hipEventElapsedTime(&t45, s->tev[4], s->tev[5]));
    s->stats.collects++;
    s->stats.ms_client_grid += t01;
    s->stats.ms_count += t12;
    s->stats.ms_write += t34;
    s->stats.ms_gate += t45;
    s->stats.records += M;
    s->stats.entities += out->n_entities;
  }
  return GWAOI_OK;
}

int gwaoi_ingest_positions(gwaoi_mgr* m, const uint8_t* payload, uint64_t bytes, uint32_t opts,
                           gwaoi_ingest_result* out) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::get_state(m, &v, &s));
  if (out) memset(out, 0, sizeof *out);
  if (bytes % GWAOI_INGEST_RECORD_BYTES) {
    gw::set_error("ingest_positions: %llu bytes is not a whole number of 32-byte records", (unsigned long long)bytes);
    return GWAOI_ERR_INVALID;
  }
  if (bytes / GWAOI_INGEST_RECORD_BYTES > 0x7FFFFFFFull) {
    gw::set_error("ingest_positions: payload too large");
    return GWAOI_ERR_INVALID;
  }
  const uint32_t n = (uint32_t)(bytes / GWAOI_INGEST_RECORD_BYTES);
  if (n && !payload) {
    gw::set_error("ingest_positions: null payload");
    return GWAOI_ERR_INVALID;
  }
  if (!(opts & GWAOI_INGEST_HOST_PAYLOAD) && ((uintptr_t)payload & 15)) {
    gw::set_error("ingest_positions: device payload must be 16-byte aligned");
    return GWAOI_ERR_INVALID;
  }
  if (out) out->n_records = n;
  if (!n) return GWAOI_OK;
  // the records come after every op already staged: presence is read on the device
  SRCHK(gw::mgr_flush(m));
  SRCHK(gw::mgr_view(m, &v));
  SRCHK(gw::upload_hash(v, s));
  hipStream_t st = v.stream;
  const uint8_t* src = payload;
  if (opts & GWAOI_INGEST_HOST_PAYLOAD) {
    SRCHK(gw::dgrow(&s->d_payload, &s->payload_cap, bytes));
    SCHK(hipMemcpyAsync(s->d_payload, payload, bytes, hipMemcpyHostToDevice, st));
    src = s->d_payload;
  }
  const uint32_t nb = gw::blocks_for(n);
  SRCHK(gw::dgrow32(&s->res, &s->res_cap, n));
  SRCHK(gw::dgrow32(&s->bcnt, &s->bcnt_cap, (uint64_t)nb + 1));
  SRCHK(gw::ensure_scan(s, nb + 1));
  if (!s->op_slot) {
    const size_t C = s->cap;
    if (hipMalloc((void**)&s->op_slot, C * 4) != hipSuccess || hipMalloc((void**)&s->op_x, C * 4) != hipSuccess ||
        hipMalloc((void**)&s->op_z, C * 4) != hipSuccess) {
      gw::set_error("ingest_positions: device allocation failed");
      return GWAOI_ERR_NOMEM;
    }
  }
  gw::IngArgs a = {};
  a.rec = (const uint4*)src;
  a.n = n;
  a.hmask = s->hcap - 1;
  a.hb = s->d_hb;
  a.seq = v.seq;
  a.flags = s->flags;
  a.y = s->y;
  a.yaw = s->yaw;
  a.res = s->res;
  a.first = s->first;
  a.ctr = s->ictr;
  a.bcnt = s->bcnt;
  a.op_slot = s->op_slot;
  a.op_x = s->op_x;
  a.op_z = s->op_z;
  if (v.timing) SCHK(hipEventRecord(s->tev[0], st));
  hipLaunchKernelGGL(gw::k_ing_init, dim3(1), dim3(64), 0, st, s->ictr, n);  // cut = n, counts 0
  hipLaunchKernelGGL(gw::k_ing_resolve, dim3(nb), dim3(gw::kSy), 0, st, a);  // (and the first batch's cut)
  uint32_t seg = 0, passes = 0, moved = 0;
  float ing_ms = 0.f;
  for (;;) {
    const uint32_t nseg = gw::blocks_for(n - seg);
    a.seg = seg;
    if (seg) {
      hipLaunchKernelGGL(gw::k_fill_u32, dim3(1), dim3(64), 0, st, s->ictr, n, 1u);
      hipLaunchKernelGGL(gw::k_ing_first, dim3(nseg), dim3(gw::kSy), 0, st, a);
      hipLaunchKernelGGL(gw::k_ing_cut, dim3(nseg), dim3(gw::kSy), 0, st, a);
    }
    hipLaunchKernelGGL(gw::k_ing_count, dim3(nseg), dim3(gw::kSy), 0, st, a);
    hipLaunchKernelGGL(gw::k_fill_u32, dim3(1), dim3(64), 0, st, s->bcnt + nseg, 0u, 1u);
    gw::launch_scan(s->scan, s->bcnt, nseg + 1, st);
    hipLaunchKernelGGL(gw::k_ing_emit, dim3(nseg), dim3(gw::kSy), 0, st, a);
    if (v.timing) SCHK(hipEventRecord(s->tev[1], st));
    SCHK(hipGetLastError());
    const uint32_t bound = std::min<uint32_t>(n - seg, s->cap);
    SRCHK(gw::mgr_stage_moves_device_n(m, s->op_slot, s->op_x, s->op_z, s->bcnt + nseg, bound));
    if (s->d_small) {
      hipLaunchKernelGGL(gw::k_to_host, dim3(1), dim3(64), 0, st, (const uint32_t*)s->ictr, 4u, 0u,
                         (const uint32_t*)(s->bcnt + nseg), 1u, 4u, s->d_small);
    } else {
      SCHK(hipMemcpyAsync(s->h_small, s->ictr, 16, hipMemcpyDeviceToHost, st));
      SCHK(hipMemcpyAsync(s->h_small + 4, s->bcnt + nseg, 4, hipMemcpyDeviceToHost, st));
    }
    SCHK(hipStreamSynchronize(st));
    if (v.timing) {
      float t;
      SCHK(hipEventElapsedTime(&t, s->tev[0], s->tev[1]));
      ing_ms += t;
    }
    ++passes;
    moved += s->h_small[4];
    const uint32_t cut = std::min(s->h_small[0], n);
    if (cut >= n) break;
    SRCHK(gw::mgr_flush(m));  // run this batch now; the next starts at the repeat
    seg = cut;
    if (v.timing) SCHK(hipEventRecord(s->tev[0], st));
  }
  if (v.timing) {
    s->stats.ingests++;
    s->stats.ms_ingest += ing_ms;
    s->stats.ingest_records += n;
  }
  if (out) {
    out->n_moved = moved;
    out->n_unknown = s->h_small[1];
    out->n_rejected = s->h_small[2];
    out->n_passes = passes;
    out->n_nonfinite = s->h_small[3];
  }
  return GWAOI_OK;
}

int gwaoi_sync_get_stats(gwaoi_mgr* m, gwaoi_sync_stats* out) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::get_state(m, &v, &s));
  if (!out) {
    gw::set_error("sync_get_stats: null output");
    return GWAOI_ERR_INVALID;
  }
  *out = s->stats;
  return GWAOI_OK;
}

int gwaoi_debug_set_fanout_mode(gwaoi_mgr* m, int mode, uint64_t* direct_reruns) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::get_state(m, &v, &s));
  if (mode > 1) {
    gw::set_error("debug_set_fanout_mode: mode %d not in {-1, 0, 1}", mode);
    return GWAOI_ERR_INVALID;
  }
  if (mode >= 0) s->fan_mode = mode;
  if (direct_reruns) *direct_reruns = s->direct_reruns;
  return GWAOI_OK;
}

int gwaoi_sync_reset_stats(gwaoi_mgr* m) {
  gw::MgrView v;
  SyncState* s;
  SRCHK(gw::get_state(m, &v, &s));
  s->stats = gwaoi_sync_stats{};
  return GWAOI_OK;
}

int gwaoi_wl_pack_ingest(int device, const uint8_t* d_ids, const float* d_x, const float* d_z, uint32_t n,
                         uint32_t tick, uint8_t* d_out) {
  SCHK(hipSetDevice(device));
  if (!n) return GWAOI_OK;
  if (!d_ids || !d_x || !d_z || !d_out || ((uintptr_t)d_ids & 15) || ((uintptr_t)d_out & 15)) {
    gw::set_error("wl_pack_ingest: null or unaligned array");
    return GWAOI_ERR_INVALID;
  }
  hipLaunchKernelGGL(gw::k_wl_pack_ingest, dim3(gw::blocks_for(n)), dim3(gw::kSy), 0, nullptr, (const uint4*)d_ids,
                     d_x, d_z, n, (float)tick * 0.01f, (uint4*)d_out);
  SCHK(hipGetLastError());
  SCHK(hipDeviceSynchronize());
  return GWAOI_OK;
}

}  // extern "C"
