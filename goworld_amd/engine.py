"""Thin numpy-facing handle over one libgwaoi manager (include/gwaoi.h).

`Engine` is what tests and bench.py drive; `goworld_amd.aoi` builds the go-aoi-shaped interface
(AOI / AOICallback / AOIManager) on top of it.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check


def _u32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def _f32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class Engine:
    """One AOI manager on one GPU: a single Space (dist) or several Spaces (spaces=[(dist, bounds)])."""

    def __init__(self, dist: Optional[float] = None, capacity: int = 1 << 16, device: int = 0,
                 bounds: Optional[Sequence[float]] = None, spaces: Optional[Sequence] = None):
        L = _lib.load()
        self._L = L
        self.capacity = int(capacity)
        self.device = int(device)
        h = ctypes.c_void_p()
        if spaces is None:
            if dist is None:
                raise ValueError("dist or spaces required")
            spaces = [(dist, bounds)]
        descs = (_lib.SpaceDesc * len(spaces))()
        for i, (d, b) in enumerate(spaces):
            descs[i].dist = float(d)
            if b is not None:
                descs[i].min_x, descs[i].min_z, descs[i].max_x, descs[i].max_z = [float(v) for v in b]
        check(L.gwaoi_create_spaces(descs, len(spaces), self.capacity, self.device, ctypes.byref(h)))
        self._h = h
        self.nspaces = len(spaces)

    # ---- lifecycle ----
    def close(self):
        self._pin = None  # views of memory the manager owns
        if getattr(self, "_h", None) and self._h.value:
            self._L.gwaoi_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    # ---- ops (the reference's Enter / Leave / Moved) ----
    def enter(self, slot: int, x: float, z: float, space: int = 0):
        check(self._L.gwaoi_enter_space(self._h, space, slot, x, z))

    def stage_enters(self, slots, x, z, space: int = 0):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        xa = np.ascontiguousarray(x, dtype=np.float32)
        za = np.ascontiguousarray(z, dtype=np.float32)
        check(self._L.gwaoi_stage_enters(self._h, space, _u32p(s), _f32p(xa), _f32p(za), len(s)))

    def leave(self, slot: int):
        check(self._L.gwaoi_leave(self._h, slot))

    def moved(self, slot: int, x: float, z: float):
        check(self._L.gwaoi_moved(self._h, slot, x, z))

    def stage_moves(self, slots, x, z):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        xa = np.ascontiguousarray(x, dtype=np.float32)
        za = np.ascontiguousarray(z, dtype=np.float32)
        check(self._L.gwaoi_stage_moves(self._h, _u32p(s), _f32p(xa), _f32p(za), len(s)))

    def stage_buffers(self):
        """The manager's pinned staging arrays (gwaoi_stage_buffers) as numpy views: (slots, x, z), each
        of `capacity` entries. Write n moves into their heads, then stage_moves_pinned(n)."""
        if getattr(self, "_pin", None) is None:
            ps, px, pz = ctypes.POINTER(ctypes.c_uint32)(), ctypes.POINTER(ctypes.c_float)(), ctypes.POINTER(ctypes.c_float)()
            cap = ctypes.c_uint32(0)
            check(self._L.gwaoi_stage_buffers(self._h, ctypes.byref(ps), ctypes.byref(px), ctypes.byref(pz),
                                              ctypes.byref(cap)))
            n = int(cap.value)
            self._pin = (np.ctypeslib.as_array(ps, shape=(n,)), np.ctypeslib.as_array(px, shape=(n,)),
                         np.ctypeslib.as_array(pz, shape=(n,)))
        return self._pin

    def stage_moves_pinned(self, n: int):
        """The first n entries of the pinned staging arrays as n Moved calls (validated on the device)."""
        check(self._L.gwaoi_stage_moves_pinned(self._h, int(n)))

    def stage_moves_pinned_partial(self, upto: int):
        """Push entries [pushed, upto) of the pinned arrays to the device now (ABI 2.1: asynchronous DMA,
        nothing staged); the final stage_moves_pinned[_async](n) copies only the rest."""
        check(self._L.gwaoi_stage_moves_pinned_partial(self._h, int(upto)))

    def stage_moves_pinned_async(self, n: int):
        """stage_moves_pinned without the host round trip (ABI 2.1): a refused batch applies nothing and is
        reported by the next call that runs the pass (tick, or a flushing call)."""
        check(self._L.gwaoi_stage_moves_pinned_async(self._h, int(n)))

    def stage_moves_device(self, d_slots: int, d_x: int, d_z: int, n: int):
        check(self._L.gwaoi_stage_moves_device(self._h, ctypes.c_void_p(d_slots), ctypes.c_void_p(d_x),
                                                ctypes.c_void_p(d_z), n))

    def stage_ops_device(self, d_slots: int, d_x: int, d_z: int, d_kinds: int, n: int, d_spaces: int = 0,
                         d_count: int = 0):
        """Mixed Enter/Leave/Moved batch from device arrays (kinds: GWAOI_OP_*, | GWAOI_OP_SILENT);
        d_spaces (optional): the Space of each Enter; d_count (optional): device address of the op
        count (then n is only its upper bound)."""
        check(self._L.gwaoi_stage_ops_device_n(self._h, ctypes.c_void_p(d_slots), ctypes.c_void_p(d_x),
                                                ctypes.c_void_p(d_z), ctypes.c_void_p(d_kinds),
                                                ctypes.c_void_p(d_spaces or None), ctypes.c_void_p(d_count or None), n))

    def adopt_device_state(self):
        """Host-staged calls are accepted again after mixed device batches (gwaoi_adopt_device_state)."""
        check(self._L.gwaoi_adopt_device_state(self._h))

    def set_population_hint(self, space: int, expected: int):
        """About `expected` entities present in Space `space`: plans its cell size (gwaoi_set_population_hint)."""
        check(self._L.gwaoi_set_population_hint(self._h, int(space), int(expected)))

    def set_stream(self, stream_ptr: int):
        check(self._L.gwaoi_set_stream(self._h, ctypes.c_void_p(stream_ptr)))

    # ---- tick ----
    def tick(self) -> np.ndarray:
        """Apply staged ops; returns the events as an (n, 2) uint32 array [mover, other|kind] in
        canonical replay order (copied out of the manager's pinned buffer)."""
        ev = _lib.Events()
        check(self._L.gwaoi_tick(self._h, ctypes.byref(ev)))
        self.last = ev
        n = int(ev.count)
        if n == 0:
            return np.zeros((0, 2), dtype=np.uint32)
        p = ctypes.cast(ev.events, ctypes.POINTER(ctypes.c_uint32))
        return np.ctypeslib.as_array(p, shape=(2 * n,)).reshape(n, 2).copy()

    def tick_raw(self) -> _lib.Events:
        """Apply staged ops, events copied to the manager's pinned host buffer (not to numpy)."""
        ev = _lib.Events()
        check(self._L.gwaoi_tick(self._h, ctypes.byref(ev)))
        self.last = ev
        return ev

    def tick_device(self) -> _lib.Events:
        """Apply staged ops, leave the events in device memory; returns the Events record."""
        ev = _lib.Events()
        check(self._L.gwaoi_tick_ex(self._h, _lib.GWAOI_TICK_DEVICE_EVENTS, ctypes.byref(ev)))
        self.last = ev
        return ev

    def count(self):
        p = ctypes.c_uint32()
        s = ctypes.c_uint32()
        check(self._L.gwaoi_count(self._h, ctypes.byref(p), ctypes.byref(s)))
        return p.value, s.value

    def relation(self):
        """CSR (row_ptr[capacity+1], cols) of the current neighbour relation, rows ascending."""
        rp = np.zeros(self.capacity + 1, dtype=np.uint32)
        nnz = ctypes.c_uint64(0)
        cap = 1 << 16
        while True:
            cols = np.zeros(cap, dtype=np.uint32)
            rc = self._L.gwaoi_export_relation(self._h, _u32p(rp), _u32p(cols), cap, ctypes.byref(nnz))
            if rc == _lib.GWAOI_OK:
                return rp, cols[: nnz.value]
            if rc == _lib.GWAOI_ERR_INVALID and nnz.value > cap:
                cap = int(nnz.value)
                continue
            check(rc)

    def relation_delta(self, cap: int = 0) -> np.ndarray:
        """Net relation changes of the last tick (gwaoi_export_relation_delta): (n, 2) uint32 rows
        {row, col | GWAOI_EV_ENTER (joined) or col (left)}."""
        n = ctypes.c_uint64(0)
        cap = max(cap, 1024)
        while True:
            out = np.empty((cap, 2), dtype=np.uint32)
            rc = self._L.gwaoi_export_relation_delta(self._h, out.ctypes.data, cap, ctypes.byref(n))
            if rc == _lib.GWAOI_OK:
                return out[: n.value]
            if rc == _lib.GWAOI_ERR_INVALID and n.value > cap:
                cap = int(n.value)
                continue
            check(rc)

    def relation_device(self):
        """Device-resident CSR view of the relation: (row_ptr device address, cols device address, nnz),
        manager-owned, valid until the next pass (gwaoi_relation_device)."""
        v = _lib.RelationView()
        check(self._L.gwaoi_relation_device(self._h, ctypes.byref(v)))
        return v.row_ptr, v.cols, int(v.nnz)

    # ---- timing ----
    def set_timing(self, on: bool = True):
        check(self._L.gwaoi_set_timing(self._h, 1 if on else 0))

    def stats(self) -> dict:
        st = _lib.Stats()
        check(self._L.gwaoi_get_stats(self._h, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in _lib.Stats._fields_}

    def reset_stats(self):
        check(self._L.gwaoi_reset_stats(self._h))

    # ---- test hooks ----
    def debug_set_next_seq(self, v: int):
        check(self._L.gwaoi_debug_set_next_seq(self._h, v))

    def debug_relation_mode(self, mode: int = -1):
        """Relation view path: 0 = incremental from the tick's events when possible, 1 = always rebuilt
        from the grid, -1 = unchanged. Returns (views built incrementally, views rebuilt, reason code of
        the last rebuild: include/gwaoi_tools.h)."""
        ni, nf, why = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_int(0)
        check(self._L.gwaoi_debug_set_relation_mode(self._h, mode, ctypes.byref(ni), ctypes.byref(nf),
                                                    ctypes.byref(why)))
        return ni.value, nf.value, why.value

    def debug_build_mode(self, mode: int = -1):
        """Grid build: 0 = one-pass tile build when the previous build's tile starts fit (re-run with the
        counting build on overflow), 1 = always counting, -1 = unchanged. Returns (one-pass builds,
        counting builds, re-runs)."""
        nf, nc, nr = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(self._L.gwaoi_debug_set_build_mode(self._h, mode, ctypes.byref(nf), ctypes.byref(nc), ctypes.byref(nr)))
        return nf.value, nc.value, nr.value

    def debug_set_sweep_lds(self, on: bool):
        check(self._L.gwaoi_debug_set_sweep_lds(self._h, 1 if on else 0))

    def debug_set_band(self, mode: int = -1) -> int:
        """gwaoi_debug_set_band: the band walk of the global-memory movers on (1, default: every mover with a
        band plan; 2 is the same) or off (0: their whole rings); returns the movers that took the band walk
        so far."""
        n = ctypes.c_uint64()
        check(self._L.gwaoi_debug_set_band(self._h, int(mode), ctypes.byref(n)))
        return int(n.value)

    def debug_sweep_sizes(self, enable: int = -1):
        """gwaoi_debug_sweep_sizes: tiles the LDS sweeps walked (small, mid, big) since counting was enabled
        (1: count; 0: read and stop; -1: read)."""
        t = (ctypes.c_uint64 * 3)()
        check(self._L.gwaoi_debug_sweep_sizes(self._h, int(enable), t))
        return tuple(int(v) for v in t)

    def debug_small_pass(self, mode: int = -1) -> int:
        """Small passes (gwaoi_debug_set_small_pass): mode 0 off, 1 auto, 2 whenever possible, -1 keep;
        returns the number of small passes run so far."""
        n = ctypes.c_uint64()
        check(self._L.gwaoi_debug_set_small_pass(self._h, int(mode), ctypes.byref(n)))
        return n.value

    def debug_set_cells_per_dist(self, v: float):
        check(self._L.gwaoi_debug_set_cells_per_dist(self._h, v))

    def debug_set_cell_side(self, v: float):
        check(self._L.gwaoi_debug_set_cell_side(self._h, v))

    def debug_set_index_limit(self, v: int):
        check(self._L.gwaoi_debug_set_index_limit(self._h, int(v)))


class DeviceBuffer:
    """Raw device allocation via libgwaoi (no torch dependency)."""

    def __init__(self, nbytes: int, device: int = 0):
        L = _lib.load()
        self._L = L
        self.device = device
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(L.gwaoi_dev_malloc(device, self.nbytes, ctypes.byref(p)))
        self.ptr = p.value

    def upload(self, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        check(self._L.gwaoi_dev_htod(self.device, ctypes.c_void_p(self.ptr), a.ctypes.data_as(ctypes.c_void_p),
                                     a.nbytes))

    def download(self, dtype, count: int, offset_bytes: int = 0) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        check(self._L.gwaoi_dev_dtoh(self.device, out.ctypes.data_as(ctypes.c_void_p),
                                     ctypes.c_void_p(self.ptr + offset_bytes), out.nbytes))
        return out

    def free(self):
        if self.ptr:
            self._L.gwaoi_dev_free(self.device, ctypes.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def wl_init(device: int, d_x: int, d_z: int, n: int, seed: int, L: float):
    check(_lib.load().gwaoi_wl_init(device, ctypes.c_void_p(d_x), ctypes.c_void_p(d_z), n, seed, L))


def wl_step(device: int, d_xp: int, d_zp: int, d_xo: int, d_zo: int, n: int, seed: int, tick: int, L: float,
            s: float = 1.0):
    check(_lib.load().gwaoi_wl_step(device, ctypes.c_void_p(d_xp), ctypes.c_void_p(d_zp), ctypes.c_void_p(d_xo),
                                    ctypes.c_void_p(d_zo), n, seed, tick, L, s))


def wl_iota(device: int, d: int, n: int):
    check(_lib.load().gwaoi_wl_iota(device, ctypes.c_void_p(d), n))


def wl_init_spaces(device: int, d_x: int, d_z: int, n_per: int, nspaces: int, seed0: int, L: float, nhot: int = 0,
                   sigma: float = 0.0, hot_every: int = 10):
    check(_lib.load().gwaoi_wl_init_spaces(device, ctypes.c_void_p(d_x), ctypes.c_void_p(d_z), n_per, nspaces, seed0,
                                           L, nhot, sigma, hot_every))


def wl_step_spaces(device: int, d_xp: int, d_zp: int, d_xo: int, d_zo: int, n_per: int, nspaces: int, seed0: int,
                   tick: int, L: float, s: float = 1.0):
    check(_lib.load().gwaoi_wl_step_spaces(device, ctypes.c_void_p(d_xp), ctypes.c_void_p(d_zp), ctypes.c_void_p(d_xo),
                                           ctypes.c_void_p(d_zo), n_per, nspaces, seed0, tick, L, s))
