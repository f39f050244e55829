"""ctypes binding of libgwaoi.so (include/gwaoi.h, include/gwaoi_tools.h).

The product path is the HIP library only: if libgwaoi.so is missing or cannot be loaded this module
raises; there is no CPU fallback. Import torch (if at all) BEFORE this module so the process uses
one HIP runtime (torch's bundled libamdhip64.so.7 and /opt/rocm's share the soname).
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# GWAOI_LIB selects another build of the same library (A/B experiments: scripts/variants.py)
SO_PATH = os.environ.get("GWAOI_LIB") or os.path.join(HERE, "libgwaoi.so")

GWAOI_OK = 0
GWAOI_ERR_INVALID = -1
GWAOI_ERR_STATE = -2
GWAOI_ERR_HIP = -3
GWAOI_ERR_NOMEM = -4
GWAOI_ERR_DEVICE_CHECK = -5
GWAOI_EV_ENTER = 0x80000000
GWAOI_EV_SLOT_MASK = 0x7FFFFFFF
GWAOI_TICK_DEVICE_EVENTS = 1
GWAOI_OP_MOVE, GWAOI_OP_ENTER, GWAOI_OP_LEAVE, GWAOI_OP_SILENT = 0, 1, 2, 0x80

# every symbol declared by include/gwaoi.h and include/gwaoi_tools.h
ABI_SYMBOLS = (
    "gwaoi_create", "gwaoi_create_spaces", "gwaoi_destroy", "gwaoi_set_stream", "gwaoi_enter",
    "gwaoi_enter_space", "gwaoi_stage_enters", "gwaoi_leave", "gwaoi_moved", "gwaoi_stage_moves", "gwaoi_stage_moves_device",
    "gwaoi_stage_buffers", "gwaoi_stage_moves_pinned", "gwaoi_stage_moves_pinned_partial",
    "gwaoi_stage_moves_pinned_async", "gwaoi_stage_ops_device",
    "gwaoi_stage_ops_device_spaces",
    "gwaoi_stage_ops_device_n", "gwaoi_adopt_device_state", "gwaoi_set_population_hint",
    "gwaoi_tick", "gwaoi_tick_ex", "gwaoi_count", "gwaoi_export_relation", "gwaoi_export_relation_delta", "gwaoi_relation_device", "gwaoi_set_timing",
    "gwaoi_get_stats", "gwaoi_reset_stats", "gwaoi_version", "gwaoi_last_error", "gwaoi_abi_version",
    "gwaoi_abi_minor",
)
TOOL_SYMBOLS = (
    "gwaoi_device_count", "gwaoi_dev_malloc", "gwaoi_dev_free", "gwaoi_dev_htod", "gwaoi_dev_dtoh",
    "gwaoi_dev_sync", "gwaoi_wl_init", "gwaoi_wl_step", "gwaoi_wl_iota", "gwaoi_wl_init_spaces",
    "gwaoi_wl_step_spaces", "gwaoi_debug_set_next_seq",
    "gwaoi_debug_set_cells_per_dist", "gwaoi_debug_set_cell_side", "gwaoi_debug_set_sweep_lds",
    "gwaoi_debug_read_stamps",
    "gwaoi_debug_sweep_occupancy", "gwaoi_wl_pack_ingest", "gwaoi_debug_set_index_limit",
    "gwaoi_debug_set_relation_mode", "gwaoi_debug_set_build_mode", "gwaoi_debug_set_small_pass", "gwaoi_debug_set_fanout_mode",
    "gwaoi_debug_set_band", "gwaoi_debug_sweep_sizes",
)


# include/gwaoi_strips.h (X-strip partition over several GPUs)
STRIP_SYMBOLS = (
    "gwaoi_strip_init_walk", "gwaoi_strip_walk", "gwaoi_strip_ingest", "gwaoi_strip_select",
    "gwaoi_strip_absorb", "gwaoi_strip_emit", "gwaoi_strip_scratch_words", "gwaoi_strip_init_skew",
    "gwaoi_strip_absorb_n", "gwaoi_strip_comm_id", "gwaoi_strip_comm_init", "gwaoi_strip_comm_destroy",
    "gwaoi_strip_exchange", "gwaoi_strip_local_init", "gwaoi_strip_emit_local", "gwaoi_strip_translate_events",
    "gwaoi_strip_region_init", "gwaoi_strip_region_start", "gwaoi_strip_region_walk", "gwaoi_strip_region_ingest",
    "gwaoi_strip_region_select", "gwaoi_strip_region_absorb", "gwaoi_strip_region_emit", "gwaoi_strip_region_absorb2",
)


# include/gwaoi_sync.h (tick-end sync fan-out and position ingest)
SYNC_SYMBOLS = (
    "gwaoi_sync_enable", "gwaoi_sync_get_tables", "gwaoi_sync_set_entities", "gwaoi_sync_set_clients",
    "gwaoi_sync_set_syncing", "gwaoi_sync_mark", "gwaoi_collect_sync", "gwaoi_ingest_positions",
    "gwaoi_sync_get_stats", "gwaoi_sync_reset_stats",
)
GWAOI_SYNC_OWN_CLIENT = 0x01
GWAOI_SYNC_NEIGHBOR_CLIENTS = 0x02
GWAOI_SYNC_FROM_CLIENT = 0x80
GWAOI_SYNC_NO_CLIENT = 0xFFFF
GWAOI_SYNC_MAX_GATES = 256
GWAOI_COLLECT_HOST = 0x1
GWAOI_COLLECT_KEEP_FLAGS = 0x2
GWAOI_INGEST_HOST_PAYLOAD = 0x1


class SyncTables(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_void_p), ("gate", ctypes.c_void_p), ("client_id", ctypes.c_void_p),
                ("entity_id", ctypes.c_void_p), ("y", ctypes.c_void_p), ("yaw", ctypes.c_void_p),
                ("capacity", ctypes.c_uint32), ("n_gates", ctypes.c_uint32)]


class SyncOut(ctypes.Structure):
    _fields_ = [("n_records", ctypes.c_uint64), ("n_gates", ctypes.c_uint32),
                ("gate_off", ctypes.POINTER(ctypes.c_uint64)), ("d_records", ctypes.c_void_p),
                ("records", ctypes.c_void_p), ("n_entities", ctypes.c_uint32)]


class IngestResult(ctypes.Structure):
    _fields_ = [("n_records", ctypes.c_uint32), ("n_moved", ctypes.c_uint32), ("n_unknown", ctypes.c_uint32),
                ("n_rejected", ctypes.c_uint32), ("n_passes", ctypes.c_uint32), ("n_nonfinite", ctypes.c_uint32)]


class SyncStats(ctypes.Structure):
    """gwaoi_sync_stats (include/gwaoi_sync.h): per-stage device time of collect/ingest."""
    _fields_ = [("collects", ctypes.c_uint64), ("ms_client_grid", ctypes.c_double), ("ms_count", ctypes.c_double),
                ("ms_write", ctypes.c_double), ("ms_gate", ctypes.c_double), ("records", ctypes.c_uint64),
                ("entities", ctypes.c_uint64), ("ingests", ctypes.c_uint64), ("ms_ingest", ctypes.c_double),
                ("ingest_records", ctypes.c_uint64)]


class StripGeom(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32),
        ("xa", ctypes.c_float), ("xb", ctypes.c_float),
        ("ra", ctypes.c_float), ("rb", ctypes.c_float),
        ("left_hi", ctypes.c_float), ("right_lo", ctypes.c_float),
        ("max_step", ctypes.c_float),
        ("has_left", ctypes.c_int32), ("has_right", ctypes.c_int32),
    ]


class StripRegion(ctypes.Structure):
    """gwaoi_strip_region (include/gwaoi_strips.h, ABI 2.1): a strip's state in local-slot order."""
    _fields_ = [("flags", ctypes.c_void_p), ("sx", ctypes.c_void_p), ("sz", ctypes.c_void_p),
                ("ex", ctypes.c_void_p), ("ez", ctypes.c_void_p), ("g2l", ctypes.c_void_p), ("l2g", ctypes.c_void_p),
                ("fq", ctypes.c_void_p), ("pend", ctypes.c_void_p), ("lctr", ctypes.c_void_p),
                ("rl", ctypes.c_void_p * 2), ("rs", ctypes.c_void_p * 2), ("nw", ctypes.c_void_p),
                ("lv", ctypes.c_void_p), ("srt", ctypes.c_void_p), ("ctr", ctypes.c_void_p),
                ("scratch", ctypes.c_void_p), ("n", ctypes.c_uint32), ("cap_l", ctypes.c_uint32),
                ("cap_new", ctypes.c_uint32), ("chunk", ctypes.c_uint32), ("cur", ctypes.c_uint32)]


class GwaoiError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"gwaoi error {code}: {msg}")
        self.code = code


class Event(ctypes.Structure):
    _fields_ = [("mover", ctypes.c_uint32), ("other", ctypes.c_uint32)]


class RelationView(ctypes.Structure):
    """gwaoi_relation_view (include/gwaoi.h): device-resident CSR of the relation."""
    _fields_ = [("row_ptr", ctypes.c_void_p), ("cols", ctypes.c_void_p), ("nnz", ctypes.c_uint64)]


class Events(ctypes.Structure):
    _fields_ = [
        ("events", ctypes.POINTER(Event)),
        ("count", ctypes.c_uint64),
        ("n_enter", ctypes.c_uint64),
        ("n_leave", ctypes.c_uint64),
        ("n_subticks", ctypes.c_uint32),
        ("n_ops", ctypes.c_uint32),
    ]


class SpaceDesc(ctypes.Structure):
    _fields_ = [("dist", ctypes.c_float), ("min_x", ctypes.c_float), ("min_z", ctypes.c_float),
                ("max_x", ctypes.c_float), ("max_z", ctypes.c_float)]


class Stats(ctypes.Structure):
    _fields_ = [
        ("ticks", ctypes.c_uint64),
        ("ms_apply", ctypes.c_double),
        ("ms_grid", ctypes.c_double),
        ("ms_sweep", ctypes.c_double),
        ("ms_order", ctypes.c_double),
        ("ms_total", ctypes.c_double),
        ("sweep_movers", ctypes.c_uint64),
        ("events", ctypes.c_uint64),
        ("grid_records", ctypes.c_uint64),
        ("grid_cells", ctypes.c_uint64),
        ("dense_movers", ctypes.c_uint64),
        ("band_movers", ctypes.c_uint64),
    ]


_lib = None


# ABI 2.1 additions (include/gwaoi.h GWAOI_ABI_MINOR): optional when an older build is loaded for an A/B
ABI_MINOR_SYMBOLS = ("gwaoi_stage_moves_pinned_partial", "gwaoi_stage_moves_pinned_async", "gwaoi_abi_minor",
                     "gwaoi_strip_region_init", "gwaoi_strip_region_start", "gwaoi_strip_region_walk",
                     "gwaoi_strip_region_ingest", "gwaoi_strip_region_select", "gwaoi_strip_region_absorb",
                     "gwaoi_strip_region_emit", "gwaoi_strip_region_absorb2")
ABI_VERSION = 2  # GWAOI_ABI_VERSION of include/gwaoi.h that these ctypes structs and signatures follow


def load(path: str = SO_PATH):
    """Load libgwaoi.so (raises if it is missing: build it with `python -m goworld_amd.build`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"libgwaoi.so not found at {path}: run `python -m goworld_amd.build` "
                          "(the AOI engine has no CPU fallback)")
    L = ctypes.CDLL(path)
    u32 = ctypes.c_uint32
    u64 = ctypes.c_uint64
    f32 = ctypes.c_float
    vp = ctypes.c_void_p
    u32p = ctypes.POINTER(ctypes.c_uint32)
    f32p = ctypes.POINTER(ctypes.c_float)
    mgrp = ctypes.POINTER(vp)
    sig = {
        "gwaoi_create": ([f32, u32, ctypes.c_int, mgrp], ctypes.c_int),
        "gwaoi_create_spaces": ([ctypes.POINTER(SpaceDesc), u32, u32, ctypes.c_int, mgrp], ctypes.c_int),
        "gwaoi_destroy": ([vp], ctypes.c_int),
        "gwaoi_set_stream": ([vp, vp], ctypes.c_int),
        "gwaoi_enter": ([vp, u32, f32, f32], ctypes.c_int),
        "gwaoi_enter_space": ([vp, u32, u32, f32, f32], ctypes.c_int),
        "gwaoi_stage_enters": ([vp, u32, u32p, f32p, f32p, u32], ctypes.c_int),
        "gwaoi_leave": ([vp, u32], ctypes.c_int),
        "gwaoi_moved": ([vp, u32, f32, f32], ctypes.c_int),
        "gwaoi_stage_moves": ([vp, u32p, f32p, f32p, u32], ctypes.c_int),
        "gwaoi_stage_moves_device": ([vp, vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_stage_buffers": ([vp, ctypes.POINTER(u32p), ctypes.POINTER(f32p), ctypes.POINTER(f32p),
                                 ctypes.POINTER(u32)], ctypes.c_int),
        "gwaoi_stage_moves_pinned": ([vp, u32], ctypes.c_int),
        "gwaoi_stage_moves_pinned_partial": ([vp, u32], ctypes.c_int),
        "gwaoi_stage_moves_pinned_async": ([vp, u32], ctypes.c_int),
        "gwaoi_stage_ops_device": ([vp, vp, vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_stage_ops_device_spaces": ([vp, vp, vp, vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_stage_ops_device_n": ([vp, vp, vp, vp, vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_adopt_device_state": ([vp], ctypes.c_int),
        "gwaoi_set_population_hint": ([vp, u32, u32], ctypes.c_int),
        "gwaoi_tick": ([vp, ctypes.POINTER(Events)], ctypes.c_int),
        "gwaoi_tick_ex": ([vp, u32, ctypes.POINTER(Events)], ctypes.c_int),
        "gwaoi_count": ([vp, u32p, u32p], ctypes.c_int),
        "gwaoi_export_relation": ([vp, u32p, u32p, u64, ctypes.POINTER(u64)], ctypes.c_int),
        "gwaoi_relation_device": ([vp, ctypes.POINTER(RelationView)], ctypes.c_int),
        "gwaoi_set_timing": ([vp, ctypes.c_int], ctypes.c_int),
        "gwaoi_get_stats": ([vp, ctypes.POINTER(Stats)], ctypes.c_int),
        "gwaoi_reset_stats": ([vp], ctypes.c_int),
        "gwaoi_export_relation_delta": ([vp, vp, u64, ctypes.POINTER(u64)], ctypes.c_int),
        "gwaoi_version": ([], ctypes.c_char_p),
        "gwaoi_abi_version": ([], ctypes.c_int),
        "gwaoi_abi_minor": ([], ctypes.c_int),
        "gwaoi_last_error": ([], ctypes.c_char_p),
        "gwaoi_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "gwaoi_dev_malloc": ([ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(vp)], ctypes.c_int),
        "gwaoi_dev_free": ([ctypes.c_int, vp], ctypes.c_int),
        "gwaoi_dev_htod": ([ctypes.c_int, vp, vp, ctypes.c_size_t], ctypes.c_int),
        "gwaoi_dev_dtoh": ([ctypes.c_int, vp, vp, ctypes.c_size_t], ctypes.c_int),
        "gwaoi_dev_sync": ([ctypes.c_int], ctypes.c_int),
        "gwaoi_wl_init": ([ctypes.c_int, vp, vp, u32, u64, f32], ctypes.c_int),
        "gwaoi_wl_step": ([ctypes.c_int, vp, vp, vp, vp, u32, u64, u64, f32, f32], ctypes.c_int),
        "gwaoi_wl_iota": ([ctypes.c_int, vp, u32], ctypes.c_int),
        "gwaoi_wl_init_spaces": ([ctypes.c_int, vp, vp, u32, u32, u64, f32, u32, f32, u32], ctypes.c_int),
        "gwaoi_wl_step_spaces": ([ctypes.c_int, vp, vp, vp, vp, u32, u32, u64, u64, f32, f32], ctypes.c_int),
        "gwaoi_debug_set_next_seq": ([vp, u32], ctypes.c_int),
        "gwaoi_debug_set_cells_per_dist": ([vp, f32], ctypes.c_int),
        "gwaoi_debug_set_cell_side": ([vp, f32], ctypes.c_int),
        "gwaoi_debug_set_sweep_lds": ([vp, ctypes.c_int], ctypes.c_int),
        "gwaoi_debug_read_stamps": ([vp, ctypes.c_size_t], ctypes.c_int),
        "gwaoi_debug_set_index_limit": ([vp, u64], ctypes.c_int),
        "gwaoi_debug_set_relation_mode": ([vp, ctypes.c_int, ctypes.POINTER(u64), ctypes.POINTER(u64),
                                           ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "gwaoi_debug_set_build_mode": ([vp, ctypes.c_int, ctypes.POINTER(u64), ctypes.POINTER(u64),
                                        ctypes.POINTER(u64)], ctypes.c_int),
        "gwaoi_debug_set_small_pass": ([vp, ctypes.c_int, ctypes.POINTER(u64)], ctypes.c_int),
        "gwaoi_debug_set_fanout_mode": ([vp, ctypes.c_int, ctypes.POINTER(u64)], ctypes.c_int),
        "gwaoi_debug_set_band": ([vp, ctypes.c_int, ctypes.POINTER(u64)], ctypes.c_int),
        "gwaoi_debug_sweep_sizes": ([vp, ctypes.c_int, ctypes.POINTER(u64)], ctypes.c_int),
        "gwaoi_strip_init_walk": ([vp, vp, vp, vp, vp, u64, f32], ctypes.c_int),
        "gwaoi_strip_walk": ([vp, vp, vp, vp, vp, vp, vp, u64, u64, f32, f32, vp], ctypes.c_int),
        "gwaoi_strip_ingest": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp], ctypes.c_int),
        "gwaoi_strip_select": ([vp, vp, vp, vp, vp, vp, vp, vp, u32, vp, vp], ctypes.c_int),
        "gwaoi_strip_absorb": ([vp, vp, vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_strip_emit": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "gwaoi_strip_scratch_words": ([u32], ctypes.c_size_t),
        "gwaoi_strip_local_init": ([vp, u32, u32, vp, vp, vp], ctypes.c_int),
        "gwaoi_strip_emit_local": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp],
                                   ctypes.c_int),
        "gwaoi_strip_translate_events": ([vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_strip_region_init": ([vp, vp], ctypes.c_int),
        "gwaoi_strip_region_start": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "gwaoi_strip_region_walk": ([vp, vp, vp, u64, u64, f32, f32, vp], ctypes.c_int),
        "gwaoi_strip_region_ingest": ([vp, vp, vp, vp, vp, vp, u32, vp], ctypes.c_int),
        "gwaoi_strip_region_select": ([vp, vp, vp, vp, vp, u32, vp, vp], ctypes.c_int),
        "gwaoi_strip_region_absorb": ([vp, vp, vp, vp, u32, vp], ctypes.c_int),
        "gwaoi_strip_region_absorb2": ([vp, vp, vp, vp, u32, vp, vp, u32, vp], ctypes.c_int),
        "gwaoi_strip_region_emit": ([vp, vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "gwaoi_strip_init_skew": ([vp, vp, vp, vp, vp, u64, f32, u32, f32, u32], ctypes.c_int),
        "gwaoi_strip_absorb_n": ([vp, vp, vp, vp, vp, vp, u32, vp], ctypes.c_int),
        "gwaoi_strip_comm_id": ([vp], ctypes.c_int),
        "gwaoi_strip_comm_init": ([vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)], ctypes.c_int),
        "gwaoi_strip_comm_destroy": ([vp], ctypes.c_int),
        "gwaoi_strip_exchange": ([vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, u32, vp, vp, vp], ctypes.c_int),
        "gwaoi_wl_pack_ingest": ([ctypes.c_int, vp, vp, vp, u32, u32, vp], ctypes.c_int),
        "gwaoi_sync_enable": ([vp, u32], ctypes.c_int),
        "gwaoi_sync_get_tables": ([vp, ctypes.POINTER(SyncTables)], ctypes.c_int),
        "gwaoi_sync_get_stats": ([vp, ctypes.POINTER(SyncStats)], ctypes.c_int),
        "gwaoi_sync_reset_stats": ([vp], ctypes.c_int),
        "gwaoi_sync_set_entities": ([vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_sync_set_clients": ([vp, vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_sync_set_syncing": ([vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_sync_mark": ([vp, vp, vp, vp, vp, u32], ctypes.c_int),
        "gwaoi_collect_sync": ([vp, u32, ctypes.POINTER(SyncOut)], ctypes.c_int),
        "gwaoi_ingest_positions": ([vp, vp, u64, u32, ctypes.POINTER(IngestResult)], ctypes.c_int),
        "gwaoi_debug_sweep_occupancy": ([ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
                                        ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        if (name in TOOL_SYMBOLS or name in ABI_MINOR_SYMBOLS) and not hasattr(L, name):
            continue  # a debug tool or ABI 2.1 call newer than this build (A/B runs of older libraries)
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.gwaoi_abi_version() != ABI_VERSION:  # structs of another ABI would be read or written out of shape
        raise ImportError(f"libgwaoi.so has ABI {L.gwaoi_abi_version()}, this binding expects {ABI_VERSION}: rebuild it")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != GWAOI_OK:
        raise GwaoiError(rc, (load().gwaoi_last_error() or b"").decode(errors="replace"))


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = load().gwaoi_device_count(ctypes.byref(n))
    return n.value if rc == GWAOI_OK else 0
