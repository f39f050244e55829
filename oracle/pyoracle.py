"""TEST INFRASTRUCTURE ONLY — ctypes front end of the CPU oracles in oracle/_build/liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product (goworld_amd, libgwaoi) never does.

  XZListOracle  oracle (i): faithful restatement of go-aoi v0.2.0 XZListAOIManager (xzlist_aoi.c)
  GridOracle    oracle (ii): stateful §8a-R semantic model with grid candidate search (grid_aoi.c)
  workload_*    host copy of include/gwaoi_workload.h (the seeded random walk of SURVEY.md §8d)

PARITY UNPINNED: go-aoi is not vendored in /root/reference and no Go toolchain exists here; the
reference holds no AOI golden vectors. See DESIGN.md "Oracle".
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")

EV_ENTER = 0x80000000
EV_SLOT_MASK = 0x7FFFFFFF

_lib = None


def build() -> str:
    """Compile the oracle library (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        f32p = ctypes.POINTER(ctypes.c_float)
        vp = ctypes.c_void_p
        for pre in ("xz", "gr"):
            getattr(L, pre + "_destroy").argtypes = [vp]
            getattr(L, pre + "_enter").argtypes = [vp, ctypes.c_uint32, ctypes.c_float, ctypes.c_float]
            getattr(L, pre + "_leave").argtypes = [vp, ctypes.c_uint32]
            getattr(L, pre + "_moved").argtypes = [vp, ctypes.c_uint32, ctypes.c_float, ctypes.c_float]
            getattr(L, pre + "_moved_batch").argtypes = [vp, ctypes.c_uint32, u32p, f32p, f32p]
            getattr(L, pre + "_bulk_enter").argtypes = [vp, ctypes.c_uint32, u32p, f32p, f32p]
            getattr(L, pre + "_event_count").argtypes = [vp]
            getattr(L, pre + "_event_count").restype = ctypes.c_uint64
            getattr(L, pre + "_events").argtypes = [vp]
            getattr(L, pre + "_events").restype = ctypes.POINTER(ctypes.c_uint32)
            getattr(L, pre + "_clear_events").argtypes = [vp]
            getattr(L, pre + "_set_record").argtypes = [vp, ctypes.c_int]
            getattr(L, pre + "_export_relation").argtypes = [vp, u32p, u32p, ctypes.c_uint64]
            getattr(L, pre + "_export_relation").restype = ctypes.c_int64
        L.xz_create.argtypes = [ctypes.c_float, ctypes.c_uint32]
        L.xz_create.restype = vp
        L.xz_check_invariants.argtypes = [vp]
        L.gr_create.argtypes = [ctypes.c_float, ctypes.c_uint32] + [ctypes.c_float] * 4
        L.gr_create.restype = vp
        L.ow_init.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_float, f32p, f32p]
        L.ow_step.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_float,
                              ctypes.c_float, f32p, f32p]
        L.ow_skew_init.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_float, ctypes.c_uint32, ctypes.c_float,
                                   ctypes.c_uint32, f32p, f32p]
        L.ow_u01.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                             ctypes.c_uint32]
        L.ow_u01.restype = ctypes.c_float
        _lib = L
    return _lib


def _u32(a):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def _f32(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class _Base:
    _pre = ""

    def __init__(self, handle, cap):
        self._h = handle
        self.cap = cap
        self._L = lib()

    def _f(self, name):
        return getattr(self._L, self._pre + "_" + name)

    def close(self):
        if self._h:
            self._f("destroy")(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def enter(self, slot, x, z):
        r = self._f("enter")(self._h, slot, x, z)
        if r:
            raise ValueError(f"oracle enter({slot}) failed: {r}")

    def leave(self, slot):
        r = self._f("leave")(self._h, slot)
        if r:
            raise ValueError(f"oracle leave({slot}) failed: {r}")

    def moved(self, slot, x, z):
        r = self._f("moved")(self._h, slot, x, z)
        if r:
            raise ValueError(f"oracle moved({slot}) failed: {r}")

    def moved_batch(self, slots, x, z):
        s, sp = _u32(slots)
        xa, xp = _f32(x)
        za, zp = _f32(z)
        r = self._f("moved_batch")(self._h, len(s), sp, xp, zp)
        if r:
            raise ValueError(f"oracle moved_batch failed: {r}")

    def bulk_enter(self, slots, x, z):
        s, sp = _u32(slots)
        xa, xp = _f32(x)
        za, zp = _f32(z)
        r = self._f("bulk_enter")(self._h, len(s), sp, xp, zp)
        if r:
            raise ValueError(f"oracle bulk_enter failed: {r}")

    def set_record(self, on: bool):
        self._f("set_record")(self._h, 1 if on else 0)

    def take_events(self) -> np.ndarray:
        """Events recorded since the last call, as an (n, 2) uint32 array [mover, other|kind]."""
        n = self._f("event_count")(self._h)
        if n == 0:
            out = np.zeros((0, 2), dtype=np.uint32)
        else:
            p = self._f("events")(self._h)
            out = np.ctypeslib.as_array(p, shape=(int(n) * 2,)).reshape(-1, 2).copy()
        self._f("clear_events")(self._h)
        return out

    def relation(self):
        """CSR (row_ptr[cap+1], cols) of the neighbour relation, rows ascending."""
        rp = np.zeros(self.cap + 1, dtype=np.uint32)
        cap = 1 << 16
        while True:
            cols = np.zeros(cap, dtype=np.uint32)
            r = self._f("export_relation")(self._h, _u32(rp)[1], _u32(cols)[1], cap)
            if r >= 0:
                return rp, cols[:r]
            cap = int(-r)


class XZListOracle(_Base):
    """oracle (i): go-aoi XZListAOIManager restated (two sorted linked lists + mark counting)."""
    _pre = "xz"

    def __init__(self, dist: float, cap: int):
        super().__init__(lib().xz_create(dist, cap), cap)

    def check_invariants(self) -> int:
        return self._L.xz_check_invariants(self._h)


class GridOracle(_Base):
    """oracle (ii): stateful sequential semantic model with a uniform candidate grid."""
    _pre = "gr"

    def __init__(self, dist: float, cap: int, bounds=(-1000.0, -1000.0, 1000.0, 1000.0)):
        super().__init__(lib().gr_create(dist, cap, *[float(b) for b in bounds]), cap)


def workload_init(seed: int, n: int, L: float):
    x = np.zeros(n, dtype=np.float32)
    z = np.zeros(n, dtype=np.float32)
    lib().ow_init(seed, n, L, _f32(x)[1], _f32(z)[1])
    return x, z


def workload_skew_init(seed: int, n: int, L: float, nhot: int, sigma: float, hot_every: int = 10):
    """config 5's skewed initial placement (gww_skew_init_coord)."""
    x = np.zeros(n, dtype=np.float32)
    z = np.zeros(n, dtype=np.float32)
    lib().ow_skew_init(seed, n, L, nhot, sigma, hot_every, _f32(x)[1], _f32(z)[1])
    return x, z


def workload_step(seed: int, tick: int, x: np.ndarray, z: np.ndarray, L: float, s: float = 1.0):
    """Advance positions from tick-1 to `tick` in place (arrays must be float32 contiguous)."""
    assert x.dtype == np.float32 and z.dtype == np.float32 and x.flags.c_contiguous and z.flags.c_contiguous
    lib().ow_step(seed, tick, len(x), L, s, _f32(x)[1], _f32(z)[1])


def canonical(events: np.ndarray, op_rank: np.ndarray) -> np.ndarray:
    """Sort pair events into the canonical replay order of include/gwaoi.h: mover's op rank, LEAVE
    before ENTER, other slot ascending. op_rank[slot] = position of the slot's op in staging order."""
    if len(events) == 0:
        return events.reshape(0, 2).astype(np.uint32)
    ev = np.asarray(events, dtype=np.uint32)
    order = np.lexsort((ev[:, 1], op_rank[ev[:, 0]]))
    return ev[order]
