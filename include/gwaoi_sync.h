/*
 * gwaoi_sync.h — the two callers either side of the AOI path, on the
 * GPU, over the manager's device state:
 *
 *  1. Tick-end sync fan-out, the reference's CollectEntitySyncInfos (engine/entity/Entity.go:1207-1267):
 *     for every entity whose syncInfoFlag is set, one 48-byte record to its own client
 *     (sifSyncOwnClient) and one to the client of every entity in its InterestedBy set
 *     (sifSyncNeighborClients), grouped into one packet per gate. InterestedBy(e) is e's AOI
 *     neighbour set (the XZ manager raises both callbacks of a pair, Entity.go:227-246), which the GPU
 *     evaluates from the manager's state (positions + last-op order) without stored lists.
 *
 *  2. Position ingest, the reference's HandleSyncPositionYawFromClient (components/game/GameService.go:398-410)
 *     -> OnSyncPositionYawFromClient (EntityManager.go:480-489) -> syncPositionYawFromClient
 *     (Entity.go:430-435) -> setPositionYaw (Entity.go:1189-1205): a payload of 32-byte records
 *     [EntityID 16 B | x y z yaw float32 LE] (proto.go:136-138) is decoded on the GPU, each EntityID
 *     resolved to its slot through a device hash table, and every accepted record becomes a Moved of
 *     the AOI manager (staged, applied by the next gwaoi_tick) plus the y/yaw/flag updates of
 *     setPositionYaw. Record order is preserved exactly: a payload naming an entity twice is split into
 *     consecutive passes at the repeat (the same sub-pass rule as host staging), so the events are those
 *     of the reference's sequential loop.
 *
 * Identity: the Go side registers each AOI entity's EntityID and client (gateid, ClientID) per slot.
 * Gate ids are passed as DENSE gate indices < n_gates <= GWAOI_SYNC_MAX_GATES (the Go binding maps
 * the deployment's uint16 gate ids, GateService.go, to indices once). Entities outside AOI managers
 * (Spaces without AOI) have no InterestedBy and stay on the Go side.
 *
 * Every function returns GWAOI_OK or a negative GWAOI_ERR_* (gwaoi.h); gwaoi_last_error() explains.
 */
#ifndef GWAOI_SYNC_H
#define GWAOI_SYNC_H

#include <stdint.h>

#include "gwaoi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GWAOI_SYNC_OWN_CLIENT 0x01u       /* sifSyncOwnClient (Entity.go:94) */
#define GWAOI_SYNC_NEIGHBOR_CLIENTS 0x02u /* sifSyncNeighborClients (Entity.go:95) */
#define GWAOI_SYNC_FROM_CLIENT 0x80u      /* Entity.syncingFromClient (SetClientSyncing, Entity.go:437-440) */
#define GWAOI_SYNC_NO_CLIENT 0xFFFFu      /* gate index of a slot without a client (e.client == nil) */
#define GWAOI_SYNC_MAX_GATES 256u
#define GWAOI_ID_BYTES 16u                /* common.ENTITYID_LENGTH / CLIENTID_LENGTH */
#define GWAOI_SYNC_RECORD_BYTES 48u       /* ClientID 16 | EntityID 16 | x y z yaw f32 LE (Entity.go:1233-1238) */
#define GWAOI_INGEST_RECORD_BYTES 32u     /* EntityID 16 | x y z yaw f32 LE (GameService.go:402-407) */

/* Device tables of the sync state, capacity-sized, owned by the manager (valid until it is destroyed).
 * A GPU producer may write y/yaw/flags directly (e.g. server-side movement); client ids and entity
 * ids go through the setters below (the EntityID -> slot hash is kept in step with them). */
typedef struct {
  uint8_t* flags;      /* [cap] GWAOI_SYNC_* bits */
  uint16_t* gate;      /* [cap] dense gate index of the slot's client, or GWAOI_SYNC_NO_CLIENT */
  uint8_t* client_id;  /* [cap][16] */
  uint8_t* entity_id;  /* [cap][16] */
  float* y;            /* [cap] Position.Y (the AOI manager holds X and Z) */
  float* yaw;          /* [cap] */
  uint32_t capacity;
  uint32_t n_gates;
} gwaoi_sync_tables;

/* Allocate the sync state of a manager (flags 0, no clients, no ids). Once per manager. */
int gwaoi_sync_enable(gwaoi_mgr* mgr, uint32_t n_gates);
int gwaoi_sync_get_tables(gwaoi_mgr* mgr, gwaoi_sync_tables* out);

/* Host-array setters (n entries, applied in array order; a later entry for the same slot wins). */
/* EntityID of each slot (entity creation / restore; EntityManager.go:268-270,325-328). An all-zero id
 * unregisters the slot. Two slots may not hold the same id (GWAOI_ERR_INVALID). */
int gwaoi_sync_set_entities(gwaoi_mgr* mgr, const uint32_t* slots, const uint8_t* entity_ids, uint32_t n);
/* Client of each slot: gate index (or GWAOI_SYNC_NO_CLIENT) and ClientID (SetClient, Entity.go). */
int gwaoi_sync_set_clients(gwaoi_mgr* mgr, const uint32_t* slots, const uint16_t* gates, const uint8_t* client_ids,
                           uint32_t n);
/* SetClientSyncing(on) (Entity.go:437-440): only syncing entities accept ingested positions. */
int gwaoi_sync_set_syncing(gwaoi_mgr* mgr, const uint32_t* slots, const uint8_t* on, uint32_t n);
/* Server-side setPositionYaw bookkeeping (Entity.go:1189-1205): Y and yaw of each slot, and flag bits
 * OR-ed into its syncInfoFlag. (X/Z go to the AOI manager through gwaoi_moved as before.) */
int gwaoi_sync_mark(gwaoi_mgr* mgr, const uint32_t* slots, const float* y, const float* yaw, const uint8_t* flags,
                    uint32_t n);

/* ---- 1. CollectEntitySyncInfos ---- */
#define GWAOI_COLLECT_HOST 0x1u      /* also copy the records into host-pinned memory (out->records) */
#define GWAOI_COLLECT_KEEP_FLAGS 0x2u /* do not clear the flags (the reference clears them) */
typedef struct {
  uint64_t n_records;
  uint32_t n_gates;
  const uint64_t* gate_off;   /* host, [n_gates + 1]: gate g's records are [gate_off[g], gate_off[g+1]) */
  const uint8_t* d_records;   /* device, n_records * 48 B, gate-major; valid until the next collect */
  const uint8_t* records;     /* host-pinned copy (GWAOI_COLLECT_HOST), else null */
  uint32_t n_entities;        /* entities with a flag that were collected */
} gwaoi_sync_out;
/* Collect every flagged entity of the manager. The staged ops must have been run (gwaoi_tick) —
 * the reference collects after the tick's moves (GameService.go:185-191); else GWAOI_ERR_STATE.
 * Inside one gate, records are grouped by entity (own client first, then neighbours); the order of
 * entities and of neighbours is deterministic but unspecified (the reference's is Go map order). */
int gwaoi_collect_sync(gwaoi_mgr* mgr, uint32_t opts, gwaoi_sync_out* out);

/* Per-stage device time of the sync calls (hipEvents on the manager's stream), accumulated while the
 * manager's timing is on (gwaoi_set_timing). */
typedef struct {
  uint64_t collects;         /* gwaoi_collect_sync calls timed */
  double ms_client_grid;     /* client sub-grid build (k_cg_flag, scan, k_cg_build) */
  double ms_count;           /* fan-out count walk + scan (k_fan_tile<false>) */
  double ms_write;           /* fan-out write walk (k_fan_tile<true>): pairs + per-entity info */
  double ms_gate;            /* gate partition: k_gate_hist, scan, k_gate_scatter, k_gate_offsets */
  uint64_t records;          /* 48-B records written */
  uint64_t entities;         /* entities collected */
  uint64_t ingests;          /* gwaoi_ingest_positions calls timed */
  double ms_ingest;          /* decode + resolve + cut + compaction into the Moved batch */
  uint64_t ingest_records;   /* records decoded */
} gwaoi_sync_stats;
int gwaoi_sync_get_stats(gwaoi_mgr* mgr, gwaoi_sync_stats* out);
int gwaoi_sync_reset_stats(gwaoi_mgr* mgr);

/* ---- 2. position ingest ---- */
#define GWAOI_INGEST_HOST_PAYLOAD 0x1u /* payload is host memory (copied to the device first) */
typedef struct {
  uint32_t n_records;   /* records in the payload */
  uint32_t n_moved;     /* records that became Moved ops */
  uint32_t n_unknown;   /* EntityID not registered (entity not found: ignored, EntityManager.go:482-486) */
  uint32_t n_rejected;  /* registered but not in the manager or not syncing from its client (ignored) */
  uint32_t n_passes;    /* pipeline batches used (> 1 when an entity repeats in the payload) */
  uint32_t n_nonfinite; /* accepted id, but x or z is NaN / +-Inf: dropped (deliberate divergence: the
                           reference's list manager takes it, and a NaN node then cuts other entities'
                           Mark walks) */
} gwaoi_ingest_result;
/* Decode bytes/32 records and stage them (after any ops already staged). All but the last batch are
 * run immediately (their events are kept for the next gwaoi_tick, like any sub-pass); the last is
 * staged. The payload must stay valid until the call returns. */
int gwaoi_ingest_positions(gwaoi_mgr* mgr, const uint8_t* payload, uint64_t bytes, uint32_t opts,
                           gwaoi_ingest_result* out);

#ifdef __cplusplus
}
#endif

#endif /* GWAOI_SYNC_H */
