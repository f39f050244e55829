"""TEST INFRASTRUCTURE ONLY — CPU restatement of the callers either side of the AOI path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product (goworld_amd, libgwaoi) never does.

  collect_entity_sync_infos  restates entity.CollectEntitySyncInfos
                             (/root/reference/engine/entity/Entity.go:1221-1267, getSyncInfo 1268-1275):
      for every entity with syncInfoFlag != 0 (flag cleared):
        sifSyncOwnClient and e.client != nil  -> record(e.client.clientid, eid, X, Y, Z, Yaw) to e.client.gateid
        sifSyncNeighborClients                -> for neighbor in e.InterestedBy with neighbor.client != nil:
                                                 record(neighbor.client.clientid, eid, X, Y, Z, Yaw)
      record = ClientID 16 B | EntityID 16 B | 4 x float32 little endian (Packet.go:301-303, 378-397).
      InterestedBy(e) is e's neighbour set (both callbacks of a pair fire, Entity.go:227-246), taken
      from the AOI oracle's relation.
  ingest_positions           restates GameService.HandleSyncPositionYawFromClient (GameService.go:398-410)
                             -> OnSyncPositionYawFromClient (EntityManager.go:480-489: unknown id ignored)
                             -> syncPositionYawFromClient (Entity.go:430-435: only if syncingFromClient)
                             -> setPositionYaw (Entity.go:1189-1205: Space.move -> Moved(x, z); yaw;
                                syncInfoFlag |= sifSyncNeighborClients, fromClient so no OwnClient).

Order inside a gate's packet follows Go map iteration in the reference (random): compare per-gate
record MULTISETS (sorted rows), which is what `canonical_records` produces.
"""
from __future__ import annotations

import numpy as np

OWN_CLIENT = 0x01
NEIGHBOR_CLIENTS = 0x02
FROM_CLIENT = 0x80
NO_CLIENT = 0xFFFF

SYNC_RECORD = np.dtype([("client_id", "V16"), ("entity_id", "V16"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"),
                        ("yaw", "<f4")])
INGEST_RECORD = np.dtype([("entity_id", "V16"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("yaw", "<f4")])


def canonical_records(recs: np.ndarray) -> np.ndarray:
    """Records as sorted rows of 48 raw bytes (order-independent comparison)."""
    raw = np.ascontiguousarray(recs).view(np.uint8).reshape(-1, 48)
    if len(raw) == 0:
        return raw
    order = np.lexsort(raw.T[::-1])
    return raw[order]


def collect_entity_sync_infos(row_ptr, cols, present, flags, gate, client_id, entity_id, x, y, z, yaw, n_gates):
    """Returns ({gate: records}, flags_after). Vectorised over the CSR relation (rows = entities)."""
    flags = np.asarray(flags, np.uint8).copy()
    cap = len(flags)
    present = np.asarray(present, bool)
    want = (flags & (OWN_CLIENT | NEIGHBOR_CLIENTS)) * present
    client_id = np.asarray(client_id, np.uint8).reshape(cap, 16)
    entity_id = np.asarray(entity_id, np.uint8).reshape(cap, 16)
    gate = np.asarray(gate, np.uint16)
    # own-client records
    own = np.nonzero((want & OWN_CLIENT).astype(bool) & (gate != NO_CLIENT))[0]
    # neighbour records: every (e, o) with o in N(e), e flagged NEIGHBOR, o with a client
    row_ptr = np.asarray(row_ptr, np.int64)
    deg = np.diff(row_ptr)
    e_of = np.repeat(np.arange(cap), deg)
    o_of = np.asarray(cols, np.int64)
    keep = ((want[e_of] & NEIGHBOR_CLIENTS) != 0) & (gate[o_of] != NO_CLIENT)
    e_all = np.concatenate([own, e_of[keep]])
    r_all = np.concatenate([own, o_of[keep]])
    recs = np.zeros(len(e_all), SYNC_RECORD)
    raw = recs.view(np.uint8).reshape(-1, 48)
    raw[:, 0:16] = client_id[r_all]
    raw[:, 16:32] = entity_id[e_all]
    recs["x"] = np.asarray(x, np.float32)[e_all]
    recs["y"] = np.asarray(y, np.float32)[e_all]
    recs["z"] = np.asarray(z, np.float32)[e_all]
    recs["yaw"] = np.asarray(yaw, np.float32)[e_all]
    g_all = gate[r_all]
    out = {}
    for g in range(n_gates):
        sel = g_all == g
        if sel.any():
            out[g] = canonical_records(recs[sel])
    flags[want != 0] &= ~np.uint8(OWN_CLIENT | NEIGHBOR_CLIENTS)
    return out, flags


def ingest_positions(payload: np.ndarray, id_to_slot: dict, present, flags, y, yaw):
    """Decode a payload; returns (moves [(slot, x, z)] in order, n_unknown, n_rejected) and updates
    flags / y / yaw in place, record by record as the reference's loop does."""
    recs = np.frombuffer(np.ascontiguousarray(payload).tobytes(), INGEST_RECORD)
    moves = []
    unknown = rejected = 0
    for r in recs:
        slot = id_to_slot.get(bytes(r["entity_id"]))
        if slot is None:
            unknown += 1
            continue
        if not present[slot] or not (flags[slot] & FROM_CLIENT):
            rejected += 1
            continue
        moves.append((slot, float(r["x"]), float(r["z"])))
        y[slot] = r["y"]
        yaw[slot] = r["yaw"]
        flags[slot] |= NEIGHBOR_CLIENTS
    return moves, unknown, rejected
