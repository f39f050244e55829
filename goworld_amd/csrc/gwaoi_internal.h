// gwaoi_internal.h — data layout shared by the gfx950 kernels (gwaoi_kernels.hip) and the host
// runtime (gwaoi_runtime.hip). See DESIGN.md "Data layout in HBM".
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gw {

// Op kinds staged by the host (the reference's three AOIManager calls, Space.go:211/221, 243, 259).
enum : uint8_t { OP_MOVE = 0, OP_ENTER = 1, OP_LEAVE = 2, OP_KIND = 3, OP_SILENT = 0x80 };

// Device-side error bits (device-staged batches are validated on the GPU).
enum : uint32_t { ERR_DUP_SLOT = 1u, ERR_ABSENT_SLOT = 2u, ERR_BAD_SLOT = 4u, ERR_PRESENT_SLOT = 8u, ERR_BAD_SPACE = 16u,
                  ERR_BAD_COUNT = 32u, ERR_BAD_COORD = 64u };

// IEEE binary32 bit test: not NaN, not +-Inf (the ABI rejects non-finite coordinates)
__host__ __device__ __forceinline__ bool finite_bits(uint32_t b) { return (b & 0x7f800000u) != 0x7f800000u; }

// Counters block in device memory.
enum { CTR_EVENTS = 0, CTR_ERR = 1, CTR_ENTER = 2, CTR_UNITS = 3, CTR_RECORDS = 4, CTR_PRESENT = 5, CTR_LEAVES = 6,
       CTR_DENSE = 7, CTR_HOLES = 8, CTR_NOPS = 9,  // ops of the pass (device-counted batches)
       CTR_BOVF = 10,   // the one-pass build overflowed a tile's bucket: the pass is re-run (counting build)
       CTR_NEV = 11,    // events of the pass (scan total of the per-op counts; k_place)
       CTR_UNSORTED = 12,  // set when ops' events were numbered out of canonical order (k_slice_sort sorts every op)
       CTR_UNS_SOME = 13,  // set when some ops are flagged in the unsorted bitmask (k_slice_sort sorts those)
       CTR_BAND_MV = 14,     // dense movers that took the band walk (k_sweep_dense)
       CTR_SMALL_OVF = 15,   // k_order_small: the pass's events exceed its LDS (the host re-runs the order stage)
       CTR_BDONE = 16,  // blocks of the one-pass build done (not published)
       CTR_SDONE = 17,  // blocks of k_slice_sort done (the last one publishes the counters)
       CTR_RING_MV = 18,  // movers k_sweep_band handed to the ring walk (k_sweep_dense<true> exits at 0)
       CTR_N = 32 };
constexpr int kPubWords = 16;  // counters [0, 16) are what the host reads after a pass
// CTR_EVENTS counts SLOTS of ev_tmp's shared region (after the per-tile regions, SweepArgs.ev_fix);
// k_sweep_dense reserves them in per-wave chunks and marks the unused tail of its last chunk as holes
// (x == kEvHole), counted in CTR_HOLES. The pass's event count is CTR_NEV.
constexpr uint32_t kEvHole = 0xFFFFFFFFu;

// Cells are grouped in square tiles of kTile x kTile cells; cell keys are tile-major,
//   key = base + (tz * ntx + tx) * 1024 + lz * 32 + lx   (cx = 32 tx + lx, cz = 32 tz + lz),
// so a tile's entities are contiguous (the unit of work and of LDS staging in the sweep) and a cell
// row inside a tile is contiguous.
constexpr int kTileShift = 5;
constexpr int kTile = 1 << kTileShift;       // 32
constexpr int kTileCellShift = 2 * kTileShift;
constexpr int kTileCells = kTile * kTile;    // 1024
// The sweep stages a tile plus a halo of `reach` cells in LDS; the region may hold at most this many
// cells (a Space whose (kTile + 2 reach)^2 exceeds it takes the global-memory sweep path).
#ifndef GW_REG_CELLS
#define GW_REG_CELLS 2304
#endif
constexpr int kSweepRegCells = GW_REG_CELLS;  // 48 x 48
// the big LDS sweep (one 1024-thread block per CU): regions of up to 68 x 68 cells
constexpr int kSweepBigRows = 68;
constexpr int kSweepBigCells = kSweepBigRows * kSweepBigRows;
// the mid sweep (two 512-thread blocks per CU: one stages while the other walks) for regions of up to
// kSweepMidRows rows and its records' LDS (Geom.pad with kPadMid set)
#ifndef GW_MID_ROWS
#define GW_MID_ROWS 56
#endif
constexpr int kSweepMidRows = GW_MID_ROWS;
constexpr int kSweepMidCells = kSweepMidRows * kSweepMidRows;
// records the mid and big sweeps stage at most (the planner keeps a region's planned population below them)
#ifndef GW_BIG_CAP
#define GW_BIG_CAP 2800
#endif
#ifndef GW_MID_CAP
#define GW_MID_CAP 1850
#endif
constexpr int kSweepBigCap = GW_BIG_CAP, kSweepMidCap = GW_MID_CAP;
constexpr uint32_t kPadMid = 0x80000000u;  // Geom.pad: the Space takes the mid sweep (the halo in the low bits)

// Cell geometry of one Space inside one grid snapshot.
struct Geom {
  float x0, z0;       // origin of cell (0,0)
  float inv_c;        // 1 / cell side
  float D;            // AOI distance of the Space (manager-wide per Space, as NewXZListAOIManager)
  int32_t ncx, ncz;   // cells per axis (multiples of kTile)
  int32_t ntx, ntz;   // tiles per axis
  uint32_t base;      // first cell key of this Space
  uint32_t tile_base; // first tile index of this Space (base / kTileCells)
  int32_t reach;      // halo (cells) staged around a tile in the sweep (0: the region does not fit k_sweep)
  uint32_t pad;       // reach 0: the halo of the big sweep (k_sweep<SwBig>; 0: neither, the dense walk)
};

// The pass's grid: every record sorted by cell key (counting sort). Per slot: a MAIN record at its
// end-of-pass cell (if present at the end) and a GHOST record at its start-of-pass cell (if present
// at the start and that cell differs, or it left in this pass).
//   rec[j].a = {x_bin bits, z_bin bits, slot | flags, opq}   (binned position; opq = op seq of this pass)
//   rec[j].b = {x_start bits, z_start bits, seq_start, seq_end}
enum : uint32_t { REC_GHOST = 0x80000000u, REC_HASG = 0x40000000u, REC_SLOT = 0x3fffffffu };
constexpr uint32_t kNoKey = 0xffffffffu;

struct Rec {  // one grid record, 32 B contiguous (one write per record, one 32-B read in the sweep)
  uint4 a;
  uint4 b;
};

struct GridView {
  const Rec* rec;
  const uint32_t* cs;          // cell_start[ncells + 1]
  const Geom* geom;            // [nspaces]
  const uint32_t* tile_space;  // [ntiles] tile -> space
};

struct ApplyArgs {
  const uint32_t* n_dev;     // non-null: the batch's op count is *n_dev (<= n_ops, the launch bound)
  const uint32_t* op_slot;
  const float* op_x;
  const float* op_z;
  const uint8_t* op_kind;    // null => all OP_MOVE (device-staged moves); may carry OP_SILENT
  const uint32_t* op_space;  // space of OP_ENTER ops (null: Space 0)
  uint32_t nspaces;          // op_space values are checked against it (device-staged)
  uint32_t* leaves;          // device-staged mixed batch: Leave op indices are appended here
  uint32_t n_ops;
  uint32_t base;             // seq of op 0; op i gets seq base + i
  uint32_t cap;
  int check;                 // validate (device-staged)
  float* pos_x;
  float* pos_z;
  uint32_t* seq;             // 0 = absent
  uint32_t* space_of;
  float* old_x;
  float* old_z;
  uint32_t* old_seq;
  uint32_t* opq;             // op seq of this pass (stale for slots without an op)
  uint32_t* ctr;
  uint32_t* rank_cnt;        // [n_ops + 1]: zeroed here (the sweep stores non-zero counts; [n_ops] = scan total)
  // small pass (ov_rec non-null): every op's slot joins the overlay (the slots with an op since the grid
  // was built): ov_tag[slot] = gen marks it, ov_idx[slot] its entry, ov_rec[entry] its record as a grid
  // build would write it (main record, or a ghost for a Leave)
  uint32_t gen;
  uint32_t* ov_tag;
  uint32_t* ov_idx;
  Rec* ov_rec;
  uint32_t* ov_count;        // device: overlay entries
  uint32_t ov_cap;
  // small pass with host ops: op_* are the device aliases of the pinned staging arrays (read over PCIe,
  // no copies); each op's slot and raw kind byte are written here for the kernels after k_apply
  uint32_t* cp_slot;
  uint8_t* cp_kind;
};



struct BinArgs {
  const float* pos_x;
  const float* pos_z;
  const uint32_t* seq;
  const uint32_t* space_of;
  const float* old_x;
  const float* old_z;
  const uint32_t* old_seq;
  const uint32_t* opq;
  uint32_t base, n_ops;
  const Geom* geom;
  uint32_t nspaces;
  uint32_t cap;
  uint32_t* key_of;    // [2 cap]: main / ghost key per slot (kNoKey = none)
  uint32_t* local_of;  // [2 cap]
  uint32_t* cs;        // counts, then (after scan) cell_start
  Rec* rec;
  // tile-bucketed build (launch_bin_tiles): per-(tile, slot chunk) histogram, bucket buffers
  uint32_t ntiles, nblk;
  uint32_t chunk;             // slots per block: kBinChunk, larger for big capacities (nblk <= ~256)
  uint32_t* thist;            // [ntiles * nblk]: bucket offset of (tile, chunk) inside its tile
  uint32_t* ttot;             // [kMaxLdsTiles] tile totals (zero on entry; summed by k_bin_tcount)
  uint32_t* ttot_next;        // [kMaxLdsTiles] the next build's totals (zeroed by k_bin_tscatter)
  uint32_t* tstart;           // [ntiles + 1] tile starts (this build's)
  const uint32_t* tprev;      // [ntiles + 1] the previous tile build's starts: the one-pass build's plan
  uint32_t fused;             // 1: one-pass build (k_bin_tfused), records bucketed at plan_start(tprev, tile)
  uint32_t trec_cap;          // records trec holds
  uint32_t* ctr;              // pass counters (CTR_BOVF, CTR_BDONE)
  const uint32_t* tile_space;  // tile -> space
  Rec* trec;                  // records bucketed by tile (the other grid's buffer: unused this pass)
  const uint8_t* op_kind;     // the pass's op kinds (null: all moves), for tile_walk
  uint32_t* tile_walk;        // [ntiles] out: 1 = the tile holds a reported mover (k_sweep skips the rest)
  uint32_t* tile_acted;       // [ntiles] out: slots with an op in this pass, counted once per slot (k_bin_tsort)
};

// Slots per block of the tile-bucketed build (at least; a capacity over 256 chunks gets larger
// chunks, so the tile x chunk histogram stays ~256 x tiles), and the largest tile count its LDS
// histogram holds (larger grids use the cell-atomic build).
#ifndef GW_BIN_CHUNK
#define GW_BIN_CHUNK 4096
#endif
#ifndef GW_BIN_MAX_BLOCKS
#define GW_BIN_MAX_BLOCKS 256
#endif
constexpr uint32_t kBinChunk = GW_BIN_CHUNK;
constexpr uint32_t kBinMaxBlocks = GW_BIN_MAX_BLOCKS;
inline uint32_t bin_chunk(uint32_t cap) {
  const uint64_t per = ((uint64_t)cap + kBinMaxBlocks - 1) / kBinMaxBlocks;
  const uint64_t c = (per + kBinChunk - 1) / kBinChunk * kBinChunk;
  return (uint32_t)(c > kBinChunk ? c : kBinChunk);
}
#ifndef GW_MAX_LDS_TILES
#define GW_MAX_LDS_TILES 12288
#endif
constexpr uint32_t kMaxLdsTiles = GW_MAX_LDS_TILES;

struct SweepArgs {
  GridView g;
  const float* old_x;  // start-of-pass state of Leave ops' slots
  const float* old_z;
  const uint32_t* old_seq;
  const uint32_t* space_of;
  const float* pos_x;  // current (end-of-pass) state: movers of the dense list (slots)
  const float* pos_z;
  const uint32_t* opq;
  uint32_t base;       // seq of op 0 of this pass
  uint32_t n_ops;
  uint32_t n_rec;      // upper bound on records in the grid (flat variant grid size)
  uint32_t ncells;     // cells of the grid (cs[ncells] = record count)
  uint32_t ntiles;     // tiles of the grid: blocks [0, ntiles) take one tile each, the rest Leave ops
  uint32_t big_t0, big_n;  // the tiles of the Spaces of the big sweep (Geom.pad): [big_t0, big_t0 + big_n)
  uint32_t mid_t0, mid_n;  // the tiles of the Spaces of the mid sweep (Geom.pad & kPadMid)
  int use_lds;         // 1: LDS-staged sweep; 0: every mover to k_sweep_dense (tests); 2: staging only (timing)
  const uint32_t* op_slot;    // for the leave path
  const uint8_t* op_kind;     // per op (null: all moves); OP_SILENT movers are applied, not walked
  const uint32_t* leave_ops;  // op indices of OP_LEAVE ops
  uint32_t n_leaves;          // host-staged: the count; device-staged mixed batch: see leaves_dev
  const uint32_t* n_leaves_dev;  // non-null: the count is on the device (ctr[CTR_LEAVES])
  uint32_t leave_blocks;      // blocks after the tiles that walk the Leave ops
  uint4* ev_tmp;    // shared region, slots from ctr[CTR_EVENTS]: {rank, local index within rank, mover, other|kind}
  uint32_t ev_cap;
  // k_sweep's tile blocks (tile builds): tile t's queued events at ev_fix[t * kEvLds ...], their count in
  // tile_ev[t] and its enter events in tile_ent[t] (stores, no atomics); null: the shared region only
  uint4* ev_fix;
  uint32_t* tile_ev;
  uint32_t* tile_ent;
  uint32_t* rank_cnt;
  uint32_t* uns;        // [n_ops / 32 + 1] bitmask: ops whose events are out of canonical order (CTR_UNS_SOME)
  uint32_t* ctr;
  uint32_t* dense;      // slots of movers for k_sweep_dense (boxes beyond the tile's LDS region)
  uint32_t* dense2;     // band walk on: the movers k_sweep_band leaves to the ring walk
  uint32_t dense_cap;
  uint32_t dense_hint;  // dense movers of the previous pass (0: k_sweep_dense not launched)
  const uint32_t* tile_walk;  // per tile: holds a reported mover (null: k_sweep scans the tile's records)
  // the band walk of k_sweep_dense: the grid's records sorted per cell by search key (null:
  // not built this pass, every dense mover walks its ring), and per Space the key spread
  const float* band_xk;   // x key of each record (the grid's records sorted by x key inside each cell)
  const float* band_zk;   // per cell by z key: the key, and
  const uint32_t* band_zi;  // the record
  const uint32_t* band_hd;
  const uint8_t* band_tab;   // key tables (BandArgs.tab), or null: the key windows are searched
  uint32_t band_tab_half;
  uint32_t nspaces;      // Spaces of the grid (geom[nspaces])
  uint32_t* size_tiles;  // debug (gwaoi_debug_sweep_sizes): tiles walked in LDS by the small / mid / big sweep, or null
};

// Band keys of the pass's grid for k_sweep_dense's band walk. A record's judge position p is
// its binned position, or, for a main record without a ghost whose entity acted, its start OR its end
// position (both in the binned cell), depending on the mover. Its search key is the midpoint of the two
// (the binned position otherwise), and hd bounds |p - key| per Space and axis, so a band of p values is a
// window of keys widened by hd.
struct BandArgs {
  GridView g;
  const uint32_t* space_of;
  uint32_t nspaces;
  uint32_t rec_bound;    // launch bound on the grid's records
  const uint32_t* nrec;  // device: the grid's records (cs[ncells])
  Rec* rec_out;          // [records] the grid's records sorted by x key inside each cell (cells over
                         // kBandCellMax records copied as they are); replaces the grid's records
  float* xk;             // [records] their x keys, in rec_out order
  float* zk;             // [records] per cell by z key: the key,
  uint32_t* zi;          // and the record's index in rec_out
  uint32_t* hd;          // [2 nspaces] per Space: max |p - key| (float bits; zeroed by the caller), x then z
  uint8_t* tab;          // key tables (GW_BAND_TABLE): x tables, then z tables at tab + tab_half; a sorted cell
  uint32_t tab_half;     // of kBandSearchMin.. records starting at record s owns bytes [(s / 4) * 64, + 64)
};
// cells of more records than this are not sorted: the band walk reads them whole (255: a key table's
// offsets are bytes)
constexpr uint32_t kBandCellMax = 255;
// key table of a sorted cell, per axis: byte b (1..63) = the number of the cell's keys k whose bucket
// band_bucket(k) is below b, i.e. the sorted position of the first key of bucket b (buckets: 64 equal parts of
// the cell's side); the band walk reads the keys of a window [w0, w1] as positions [tab[b(w0)], tab[b(w1) + 1])
constexpr int kBandBuckets = 64;
void launch_band_keys(const BandArgs& b, hipStream_t st);

struct RelArgs {
  GridView g;
  const float* pos_x;
  const float* pos_z;
  const uint32_t* seq;
  const uint32_t* space_of;
  uint32_t cap;
  const uint32_t* row_ptr;  // null in the count pass
  uint32_t* row_cnt;        // count pass output (zeroed beforehand: absent slots have no record)
  uint32_t* cols;
  uint32_t ntiles;          // tiles of the grid (one block each)
  unsigned long long* total64;  // count pass: sum of the row lengths in 64 bits (uint32 overflow guard)
  uint4* tstat;             // count pass: per tile {row lengths' sum lo, hi, longest row, 0} (summed after)
  uint32_t* maxlen;         // count pass: longest row
  uint32_t* slab;           // count pass, optional: the rows by grid record, interleaved (k_row_sort_slab)
  uint32_t slab_s;          // entries per row kept in the slab (rows longer than this: not kept)
  uint32_t slab_recs;       // grid records the slab has rows for: a record past them writes no slab row and
                            // reports a row longer than slab_s (the host then takes the two-walk path)
};

// Incremental relation view (gwaoi_relation_device after a tick whose events are all in ev_out).
struct RelDeltaArgs {
  const uint2* ev;        // the tick's events {mover, other | ENTER}
  uint32_t nev;
  uint32_t cap;
  const uint32_t* rp_old;  // [cap + 1] the view before the tick
  const uint32_t* cols_old;
  uint32_t* dn;            // [cap + 1] changes per row (zeroed), then their exclusive scan
  uint32_t* dcur;          // [cap] fill cursors (zeroed)
  uint32_t* dch;           // [2 nev] changes by row: col | ENTER
  uint32_t* dchrow;        // [2 nev] the row of each change
  uint32_t* rp_new;        // [cap + 1]
  uint32_t* cols_new;
  uint64_t cols_cap;       // entries cols_new holds (every store is bounded by it)
  uint32_t* flag;          // set: the update cannot be done (a row's changes exceed the sort's LDS)
  int32_t* psum;           // [2 nev] rows with many changes: inclusive prefix of the signs of the sorted list
  uint32_t* longrows;      // rows with more than kRdShort changes (sorted by k_rd_sort_long)
  uint32_t* nlong;         // their count (zeroed)
  uint32_t long_cap;
};

// Relation delta export: net changes of the relation over one tick's events (k_dx_*).
struct DeltaExportArgs {
  const uint2* ev;               // the tick's events {mover, other | ENTER}
  uint32_t nev;
  uint32_t mask;                 // hash table slots - 1 (slots >= 2 nev, a power of two)
  unsigned long long* keys;      // [slots] unordered pair (min << 32 | max); ~0 = empty
  uint32_t* cnt;                 // [slots] events of the pair (zeroed)
  uint32_t* last;                // [slots] largest event index of the pair (zeroed)
  uint32_t* slot_of;             // [nev]
  uint32_t* flags;               // [nev + 1] kept, then their exclusive scan
  uint2* out;                    // [2 nev] {row, col | ENTER (added) or col (removed)}
};

// Scan scratch (the chunk sums of launch_scan), owned by the stream's manager.
struct ScanCtx {
  uint32_t* status = nullptr;  // scan_part_words(max n) words
};

// ---- launchers (gwaoi_kernels.hip) ----
void launch_apply(const ApplyArgs& a, hipStream_t st);
void launch_bin_count(const BinArgs& a, hipStream_t st);
void launch_bin_scatter(const BinArgs& a, hipStream_t st);
// Tile-bucketed build: LDS tile histograms per slot chunk -> (scan thist) -> bucket scatter -> per-tile
// LDS cell sort that writes the records and every cell start. part: scan scratch.
void launch_bin_tiles(const BinArgs& a, hipStream_t st);
// (the one-pass build when a.fused: the previous build's tile starts as the bucket plan, a bucket past
// its tile's room raises ctr[CTR_BOVF]; else the counting build)
// In-place exclusive scan of d[0..n); d[n-1] must be 0 on entry if the total is wanted there.
void launch_scan(ScanCtx& c, uint32_t* d, uint32_t n, hipStream_t st);
uint32_t scan_part_words(uint32_t n);
void launch_sweep(const SweepArgs& a, hipStream_t st);
uint32_t sweep_ev_lds();  // events queued per tile block (the per-tile region size)
size_t sweep_lds_bytes();
uint32_t sweep_block();  // threads per sweep block
void sweep_init();  // once per process (dynamic LDS limit of the sweep)
int read_stamps(void* host, size_t bytes);
int sweep_occupancy(int* blocks);  // resident sweep blocks per CU (HIP occupancy API)  // GW_STAMPS diagnostic builds only (else -1)
// Event ordering runs without a host round trip: each step checks on the device that the sweep's
// event count fit both buffers (else it does nothing and the host re-runs after growing them).
struct EvGuard {
  const uint32_t* ctr;
  uint32_t tmp_cap;
  uint64_t keep;     // events already in ev_out from earlier passes of this tick
  uint64_t out_cap;
};
struct OrderArgs {
  EvGuard g;                 // g.tmp_cap: slots of the shared region
  const uint4* ev_tmp;       // the shared region
  const uint4* ev_fix;       // per-tile regions (null: none), ntiles_fix x kEvLds
  const uint32_t* tile_ev;
  const uint32_t* tile_ent;
  uint32_t ntiles_fix;
  uint2* scratch;            // k_slice_sort's scratch (the whole ev_tmp: 2 x its slots >= events)
  const uint32_t* rank_off;  // exclusive scan of per-op event counts, [n_ops + 1]
  uint32_t* uns;             // the sweep's unsorted-op bitmask (CTR_UNS_SOME): k_slice_sort sorts and clears
  uint2* ev_out;             // this pass's slice of the output (offset by g.keep)
  uint2* host_out;           // mapped pinned host slice, or null (events stay in HBM)
  uint32_t n_ops;
  uint32_t* zero_cs;         // cell counts of the grid the next pass builds
  uint32_t zero_n;
  uint32_t* ctr_next;        // the next pass's counter block
  const uint32_t* grid_total;  // cs[ncells] of this pass's grid (record count, reported in the stats)
  const uint32_t* op_slot;   // device-staged batch check: every op's slot carries that op's seq
  const uint32_t* opq;
  uint32_t base, cap;
  int check_ops;             // k_slice_sort checks every op's slot carries its seq (non-tile builds)
  const uint32_t* n_dev;  // device-counted batch: ranks >= *n_dev are not ops
  // tile builds of device batches: k_place compares the slots that acted (k_bin_tsort's per-tile counts)
  // with the op count instead (a duplicate slot leaves one slot for two ops)
  const uint32_t* tile_acted;
  uint32_t ntiles_acted;     // 0: no such check
  uint32_t* pub;             // mapped host publication buffer (null: the host copies the counters itself)
  uint32_t pub_seq;          // sequence word published with the counters
  int sorted_hint;           // the previous pass needed no slice sort: k_slice_sort runs as a few blocks,
                             // the last of which publishes (else one thread per op, then k_publish)
  uint32_t place_blocks;     // k_place's grid (0: 1024)
};
// Small pass: the movers of a pass with few ops judged against the last full build's grid (records of
// slots without an op since then; their state is the record's end state) plus the overlay (every slot
// with an op since then, one record each), without rebuilding the grid (k_sweep_small).
struct SmallArgs {
  GridView g;                // the grid of the last full build
  uint32_t base, n_ops;
  const uint32_t* n_dev;     // device-counted batch (null: n_ops)
  const uint32_t* op_slot;
  const uint8_t* op_kind;    // null: all moves
  const uint32_t* space_of;
  const float* pos_x;
  const float* pos_z;
  const float* old_x;
  const float* old_z;
  const uint32_t* old_seq;
  const uint32_t* opq;
  uint32_t gen;
  const uint32_t* ov_tag;
  const Rec* ov_rec;
  const uint32_t* ov_count;
  uint4* ev_tmp;             // shared region (slots from ctr[CTR_EVENTS], reserved per wave)
  uint32_t ev_cap;
  uint32_t* rank_cnt;
  uint32_t* ctr;
  // one_op: a pass of ONE host op (the Go wrapper's flushed Enter or Leave) runs as one kernel: the op
  // applied (ap; no k_apply launch), swept, and its slice ordered and published (od) from LDS. A slice
  // over the kernel's LDS, or over the event buffers, leaves the order stage to the host as
  // k_order_small's overflow does (ctr[CTR_SMALL_OVF] / the buffer re-run); a re-run of the sweep is a
  // plain k_sweep_small (the op is applied once).
  int one_op;
  ApplyArgs ap;
  OrderArgs od;
  // one_op: the op itself by value (the host staged it: no PCIe read of the pinned staging arrays), and the
  // slice also written into the mapped host event buffer (od.host_out) before the publication, so a
  // host-delivered pass needs no copy-out kernel and no stream synchronisation
  uint32_t one_slot, one_space, one_kind;
  float one_x, one_z;
};
void launch_sweep_small(const SmallArgs& a, hipStream_t st);
// k_place (+ zeroing side jobs, duplicate-slot check) -> k_slice_sort (+ batch check, publication of
// the counters by its last block when o.pub) -> k_copy_out (if host_out)
void launch_order(const OrderArgs& o, hipStream_t st);
// The order stage of a small pass in one single-block kernel (scan of the per-op counts, placement and
// slice sort in LDS, publication): when the pass has at most kOrderSmallOps ops. A pass whose events
// exceed the kernel's LDS sets ctr[CTR_SMALL_OVF] (published); the host then runs launch_order on the
// scanned counts.
constexpr uint32_t kOrderSmallOps = 1024;
void launch_order_small(const OrderArgs& o, hipStream_t st);
void launch_copy_out(const OrderArgs& o, hipStream_t st);  // k_copy_out alone (host event delivery)
void launch_publish(const uint32_t* ctr, uint32_t* pub, uint32_t seq, hipStream_t st);
// a[0, na) then b[0, nb) (na + nb <= kPubWords) into pub, then seq into pub[kPubWords]
void launch_publish_words(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb, uint32_t* pub,
                          uint32_t seq, hipStream_t st);
void launch_relation(const RelArgs& a, hipStream_t st);
// Rows of cols (filled by the fill pass) sorted in place.
void launch_row_sort(const uint32_t* row_ptr, uint32_t cap, uint32_t* cols, uint32_t* tmp, hipStream_t st);
// Rows from the count pass's slab (every row <= slab_s) into cols, sorted. fix: room for one entry per
// record; *nfix zeroed beforehand.
void launch_row_sort_slab(const Rec* rec, const uint32_t* nrec, uint32_t rec_bound, const uint32_t* row_ptr,
                          const uint32_t* slab, uint32_t slab_s, uint32_t* cols, uint32_t* tmp, uint4* fix,
                          uint32_t* nfix, hipStream_t st);
// Incremental view: count the changes per row (dn), then (after the caller scans dn) fill, new row
// lengths, scan, and place old and new entries.
void launch_rel_delta_count(const RelDeltaArgs& a, hipStream_t st);
void launch_rel_delta_apply(const RelDeltaArgs& a, ScanCtx& sc, hipStream_t st);
void launch_delta_export(const DeltaExportArgs& a, ScanCtx& sc, hipStream_t st);  // count: flags[nev] (x2)
void launch_wl_init(float* x, float* z, uint32_t n, uint64_t seed, float L, hipStream_t st);
void launch_wl_init_spaces(float* x, float* z, uint32_t n_per, uint32_t nspaces, uint64_t seed0, float L,
                           uint32_t nhot, float sigma, uint32_t hot_every, hipStream_t st);
void launch_wl_step_spaces(const float* xp, const float* zp, float* xo, float* zo, uint32_t n_per, uint32_t nspaces,
                           uint64_t seed0, uint64_t tick, float L, float s, hipStream_t st);
void launch_wl_step(const float* xp, const float* zp, float* xo, float* zo, uint32_t n, uint64_t seed,
                    uint64_t tick, float L, float s, hipStream_t st);
void launch_iota(uint32_t* d, uint32_t n, hipStream_t st);

// Pinned host staging (gwaoi_stage_moves_pinned): validation and repeat detection of a Moved batch
// already copied to the device, without touching the manager's state.
struct PinCheckArgs {
  const uint32_t* slot;
  const float* x;
  const float* z;
  uint32_t seg, n;             // ops [seg, n) of the batch
  uint32_t cap;
  int validate;                // 1: slot present + finite coordinates (the first call of a batch)
  const uint32_t* seq;         // 0 = absent
  const uint32_t* space_of;
  unsigned long long* first;   // [cap]: (id << 32 | ~first op index) of the last call naming the slot
  uint32_t id;                 // this call's id (> every id stored before)
  const float4* ext;           // per Space {gx0, gz0, gx1, gz1} of auto-extent Spaces (null: none)
  uint32_t* seen;              // per Space 4 order keys: min x, min z, max x, max z of coordinates beyond ext
  uint32_t* out;               // [0] error bits, [1] first repeat (n: none), [2] first bad op, [3] beyond ext
};
void launch_pin_check(const PinCheckArgs& a, bool reset_seen, uint32_t nspaces, hipStream_t st);
// the verdict of a pin check kept on the device (gwaoi_stage_moves_pinned_async): *n_dev = the op count of
// the sub-pass [seg, cut) (0 for a refused batch), the four out words copied into mapped host memory
void launch_pin_count(const uint32_t* out, uint32_t n, uint32_t seg, int validate, uint32_t* n_dev,
                      uint32_t* host_out, hipStream_t st);
float ord_float(uint32_t k);

// ---- manager view for the callers either side of the path (gwaoi_sync.hip) ----
struct SyncState;  // gwaoi_sync.hip
struct MgrView {
  int device;
  hipStream_t stream;
  uint32_t cap;
  GridView g;                // the grid of the last pass (main records = current state)
  const uint32_t* rec_count;  // device: records of that grid (cs[ncells])
  uint32_t rec_bound;         // host upper bound on them
  uint32_t ncells;            // cells of that grid (cs has ncells + 1 entries)
  uint32_t ntiles;            // tiles of that grid (over all Spaces)
  const float* pos_x;
  const float* pos_z;
  const uint32_t* seq;        // 0 = absent
  const uint32_t* space_of;
  ScanCtx* scan;
  SyncState** sync;          // the manager's sync state slot (owned by the manager)
  bool pending;              // ops staged and not yet run
  uint64_t index_limit;      // largest uint32-indexed output accepted (2^32 - 1; lowered by a test hook)
  bool timing;               // gwaoi_set_timing: the sync calls time their stages with hipEvents too
};
}  // namespace gw
struct gwaoi_mgr;
namespace gw {
int mgr_view(gwaoi_mgr* m, MgrView* out);
int mgr_grid_current(gwaoi_mgr* m);  // bring the grid up to date after small passes (readers of the grid)
int mgr_flush(gwaoi_mgr* m);  // run the staged ops now (their events are kept for the next gwaoi_tick)
// stage a device-counted batch of moves (*d_n <= n_max ops; slots distinct and present, checked on device)
int mgr_stage_moves_device_n(gwaoi_mgr* m, const uint32_t* d_slots, const float* d_x, const float* d_z,
                             const uint32_t* d_n, uint32_t n_max);
void sync_free(SyncState* s);
void set_error(const char* fmt, ...);

}  // namespace gw
