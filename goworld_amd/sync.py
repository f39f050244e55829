"""Host-side mirror of the two callers either side of the AOI path (include/gwaoi_sync.h), named after
the reference functions they replace:

  EntitySync.collect_entity_sync_infos()   <- entity.CollectEntitySyncInfos   (Entity.go:1221-1267)
  EntitySync.handle_sync_position_yaw_from_client(payload)
                                           <- GameService.HandleSyncPositionYawFromClient
                                              (components/game/GameService.go:398-410)

Both run on the GPU through libgwaoi; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Dict

import numpy as np

from . import _lib
from ._lib import check

OWN_CLIENT = _lib.GWAOI_SYNC_OWN_CLIENT
NEIGHBOR_CLIENTS = _lib.GWAOI_SYNC_NEIGHBOR_CLIENTS
NO_CLIENT = _lib.GWAOI_SYNC_NO_CLIENT
RECORD_BYTES = 48   # ClientID 16 | EntityID 16 | x y z yaw f32 LE
INGEST_BYTES = 32   # EntityID 16 | x y z yaw f32 LE

SYNC_RECORD = np.dtype([("client_id", "V16"), ("entity_id", "V16"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"),
                        ("yaw", "<f4")])
INGEST_RECORD = np.dtype([("entity_id", "V16"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("yaw", "<f4")])


def _vp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class EntitySync:
    """Sync state of one Engine (AOI manager): entity ids, clients, Y/yaw and syncInfoFlag per slot."""

    def __init__(self, engine, n_gates: int):
        self.eng = engine
        self._L = engine._L
        self.n_gates = int(n_gates)
        check(self._L.gwaoi_sync_enable(engine.handle, self.n_gates))
        self.last = None

    def tables(self) -> _lib.SyncTables:
        t = _lib.SyncTables()
        check(self._L.gwaoi_sync_get_tables(self.eng.handle, ctypes.byref(t)))
        return t

    def stats(self) -> dict:
        """Per-stage device time (ms, summed) of the collect/ingest calls made while the engine's timing
        was on (Engine.set_timing)."""
        st = _lib.SyncStats()
        check(self._L.gwaoi_sync_get_stats(self.eng.handle, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in _lib.SyncStats._fields_}

    def reset_stats(self):
        check(self._L.gwaoi_sync_reset_stats(self.eng.handle))

    def debug_fanout_mode(self, mode: int = -1) -> int:
        """gwaoi_debug_set_fanout_mode: 0 direct gate writes when n_gates <= 8, 1 pair list + gate partition,
        -1 keep; returns the direct collects re-run into a grown packet buffer."""
        n = ctypes.c_uint64(0)
        check(self._L.gwaoi_debug_set_fanout_mode(self.eng.handle, int(mode), ctypes.byref(n)))
        return n.value

    @staticmethod
    def _ids(ids, n) -> np.ndarray:
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.uint8).reshape(n, 16))
        return a

    def set_entities(self, slots, entity_ids):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        ids = self._ids(entity_ids, len(s))
        check(self._L.gwaoi_sync_set_entities(self.eng.handle, _vp(s), _vp(ids), len(s)))

    def set_clients(self, slots, gates, client_ids):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        g = np.ascontiguousarray(gates, dtype=np.uint16)
        ids = self._ids(client_ids, len(s))
        check(self._L.gwaoi_sync_set_clients(self.eng.handle, _vp(s), _vp(g), _vp(ids), len(s)))

    def set_client_syncing(self, slots, on):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        o = np.ascontiguousarray(on, dtype=np.uint8)
        check(self._L.gwaoi_sync_set_syncing(self.eng.handle, _vp(s), _vp(o), len(s)))

    def mark(self, slots, y, yaw, flags):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        yy = np.ascontiguousarray(y, dtype=np.float32)
        yw = np.ascontiguousarray(yaw, dtype=np.float32)
        f = np.ascontiguousarray(flags, dtype=np.uint8)
        check(self._L.gwaoi_sync_mark(self.eng.handle, _vp(s), _vp(yy), _vp(yw), _vp(f), len(s)))

    def collect_raw(self, opts: int = 0) -> _lib.SyncOut:
        out = _lib.SyncOut()
        check(self._L.gwaoi_collect_sync(self.eng.handle, opts, ctypes.byref(out)))
        self.last = out
        return out

    def collect_entity_sync_infos(self, keep_flags: bool = False) -> Dict[int, np.ndarray]:
        """{gate index: structured array of SYNC_RECORD} — the packet body per gate."""
        opts = _lib.GWAOI_COLLECT_HOST | (_lib.GWAOI_COLLECT_KEEP_FLAGS if keep_flags else 0)
        out = self.collect_raw(opts)
        n = int(out.n_records)
        off = [int(out.gate_off[g]) for g in range(self.n_gates + 1)]
        if n:
            buf = (ctypes.c_uint8 * (n * RECORD_BYTES)).from_address(out.records)
            recs = np.frombuffer(buf, dtype=SYNC_RECORD).copy()
        else:
            recs = np.zeros(0, SYNC_RECORD)
        return {g: recs[off[g]:off[g + 1]] for g in range(self.n_gates) if off[g + 1] > off[g]}

    def handle_sync_position_yaw_from_client(self, payload) -> _lib.IngestResult:
        """Decode a host payload of 32-byte records and stage the Moved ops (applied by the next tick)."""
        p = np.ascontiguousarray(np.frombuffer(bytes(payload), np.uint8) if isinstance(payload, (bytes, bytearray))
                                 else payload.view(np.uint8))
        res = _lib.IngestResult()
        check(self._L.gwaoi_ingest_positions(self.eng.handle, _vp(p), p.nbytes, _lib.GWAOI_INGEST_HOST_PAYLOAD,
                                             ctypes.byref(res)))
        return res

    def ingest_device(self, d_payload: int, nbytes: int) -> _lib.IngestResult:
        res = _lib.IngestResult()
        check(self._L.gwaoi_ingest_positions(self.eng.handle, ctypes.c_void_p(d_payload), nbytes, 0,
                                             ctypes.byref(res)))
        return res

    def read_tables(self):
        """(flags u8, gate u16, y f32, yaw f32) copied from the device (tests)."""
        t = self.tables()
        cap = int(t.capacity)
        out = []
        for ptr, dt in ((t.flags, np.uint8), (t.gate, np.uint16), (t.y, np.float32), (t.yaw, np.float32)):
            a = np.empty(cap, dt)
            check(self._L.gwaoi_dev_dtoh(self.eng.device, _vp(a), ctypes.c_void_p(ptr), a.nbytes))
            out.append(a)
        return tuple(out)
