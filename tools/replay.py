"""ctypes front end of tools/replay_sets.c (bench tool): the Go-side callback sink — four hash-set
operations per pair event (Entity.interest / uninterest, /root/reference/engine/entity/Entity.go:227-246)."""
import ctypes
import os

import numpy as np

_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_bin", "libreplay.so")


class ReplaySets:
    def __init__(self, expect_entries: int):
        L = ctypes.CDLL(_SO)
        vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        L.rs_create.argtypes, L.rs_create.restype = [u64], vp
        L.rs_destroy.argtypes = [vp]
        L.rs_load_relation.argtypes = [vp, vp, vp, u32]
        L.rs_replay.argtypes, L.rs_replay.restype = [vp, vp, u64], u64
        L.rs_size.argtypes, L.rs_size.restype = [vp], u64
        self._L = L
        self._h = L.rs_create(int(expect_entries))
        if not self._h:
            raise MemoryError("rs_create")

    def load_relation(self, row_ptr: np.ndarray, cols: np.ndarray):
        rp = np.ascontiguousarray(row_ptr, np.uint32)
        c = np.ascontiguousarray(cols, np.uint32)
        self._L.rs_load_relation(self._h, rp.ctypes.data, c.ctypes.data, len(rp) - 1)

    def replay(self, events_ptr: int, count: int) -> int:
        """Replay `count` events at host address events_ptr ({mover, other|ENTER} u32 pairs); returns
        the number of inconsistent set operations (0 = the events are exactly the relation's changes)."""
        return int(self._L.rs_replay(self._h, ctypes.c_void_p(events_ptr), int(count)))

    def size(self) -> int:
        return int(self._L.rs_size(self._h))

    def close(self):
        if self._h:
            self._L.rs_destroy(self._h)
            self._h = None


class ShardedReplaySets:
    """The same sink split by owning entity over `shards` worker threads (rs_sharded_*)."""

    def __init__(self, expect_entries: int, shards: int):
        L = ctypes.CDLL(_SO)
        vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        L.rs_sharded_create.argtypes, L.rs_sharded_create.restype = [u64, u32], vp
        L.rs_sharded_destroy.argtypes = [vp]
        L.rs_sharded_load_relation.argtypes = [vp, vp, vp, u32]
        L.rs_sharded_replay.argtypes, L.rs_sharded_replay.restype = [vp, vp, u64], u64
        L.rs_sharded_size.argtypes, L.rs_sharded_size.restype = [vp], u64
        self._L = L
        self.shards = int(shards)
        self._h = L.rs_sharded_create(int(expect_entries), self.shards)
        if not self._h:
            raise MemoryError("rs_sharded_create")

    def load_relation(self, row_ptr: np.ndarray, cols: np.ndarray):
        rp = np.ascontiguousarray(row_ptr, np.uint32)
        c = np.ascontiguousarray(cols, np.uint32)
        self._L.rs_sharded_load_relation(self._h, rp.ctypes.data, c.ctypes.data, len(rp) - 1)

    def replay(self, events_ptr: int, count: int) -> int:
        return int(self._L.rs_sharded_replay(self._h, ctypes.c_void_p(events_ptr), int(count)))

    def size(self) -> int:
        return int(self._L.rs_sharded_size(self._h))

    def close(self):
        if self._h:
            self._L.rs_sharded_destroy(self._h)
            self._h = None


_DR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_bin", "libdeltarows.so")


class DeltaRows:
    """ctypes front end of tools/delta_rows.c: per-slot sorted neighbour arrays patched with the
    entries of gwaoi_export_relation_delta (the Go `Sets` consumer of INTEGRATION.md §2)."""

    def __init__(self, row_ptr: np.ndarray, cols: np.ndarray):
        L = ctypes.CDLL(_DR)
        vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        L.dr_create.argtypes, L.dr_create.restype = [vp, vp, u32], vp
        L.dr_destroy.argtypes = [vp]
        L.dr_apply.argtypes, L.dr_apply.restype = [vp, vp, u64], u64
        L.dr_apply_mt.argtypes, L.dr_apply_mt.restype = [vp, vp, u64, u32], u64
        L.dr_diff.argtypes, L.dr_diff.restype = [vp, vp, vp], u64
        self._L = L
        rp = np.ascontiguousarray(row_ptr, np.uint32)
        c = np.ascontiguousarray(cols, np.uint32)
        self._h = L.dr_create(rp.ctypes.data, c.ctypes.data, len(rp) - 1)
        if not self._h:
            raise MemoryError("dr_create")

    def apply(self, delta: np.ndarray, threads: int = 1) -> int:
        """Patch the rows with the delta entries; threads > 1: rows split over worker threads."""
        d = np.ascontiguousarray(delta, np.uint32)
        if threads > 1:
            return int(self._L.dr_apply_mt(self._h, d.ctypes.data, len(d), int(threads)))
        return int(self._L.dr_apply(self._h, d.ctypes.data, len(d)))

    def diff(self, row_ptr: np.ndarray, cols: np.ndarray) -> int:
        rp = np.ascontiguousarray(row_ptr, np.uint32)
        c = np.ascontiguousarray(cols, np.uint32)
        return int(self._L.dr_diff(self._h, rp.ctypes.data, c.ctypes.data))

    def close(self):
        if self._h:
            self._L.dr_destroy(self._h)
            self._h = None
