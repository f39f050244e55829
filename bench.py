#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: AOI entity-updates/sec + p99 tick latency at 1M entities.

Default workload: one Space per GPU, N = 1,000,000 entities, L = 35,000,
D = 100, seeded random walk (include/gwaoi_workload.h), every entity moves once per tick in ascending
slot order. A "step" is one tick: stage the N moves (device arrays, inputs resident in HBM) and run
the AOI pipeline until the tick's events are complete in device memory and their count is on the host.

Multi-GPU (torchrun, one process per GPU): every rank runs its own independent 1M-entity Space
(seed + rank) — the path shards by Space with no data-path collective ("scaling": "weak"); the only
collectives are the timing barrier and the max-over-ranks of the elapsed time.

Other workloads (--workload; the JSON line names the one measured):
  config3  512 Spaces x 2,000 entities per GPU in one manager (4,096 Spaces over 8 GPUs), L = 1,600
  skew     config 5: 4 Spaces x 1M per GPU, D = 50/100/200/400, 10% of the entities in 64 hotspots
  gametick one GoWorld game tick per step at config-2 scale: client position records ingested on the GPU,
           the AOI tick, and the sync fan-out into per-gate packet bodies (include/gwaoi_sync.h)
  strips   config 4: ONE world of 2M entities per GPU (16M, L = 140,000 at 8 GPUs) cut into X-strips,
           halo records exchanged with the neighbour GPUs every tick by gwaoi_strip_exchange (RCCL
           p2p over xGMI inside libgwaoi, on the strip's stream)
  strips_skew  config 5 in strips: the same world, 10% of the entities in Gaussian hotspots, strip
           edges at the x-quantiles of the entities

Prints ONE JSON line on rank 0. Also reports: p50/p99 tick latency with events left in HBM and with
events delivered to host memory (PCIe-inclusive, never `value`), the sweep kernel's roofline, and
the CPU baseline (oracle (i), the go-aoi XZListAOIManager restatement, on a bounded sample).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "AOI entity-updates/sec (p99 tick latency reported alongside) at 1M entities per Space"
DATA = "synthetic: seeded random walk of SURVEY.md §8(d) (include/gwaoi_workload.h), generated on device"
DENSITY = 1_000_000 / 35000.0 ** 2  # entities per unit^2 of every config (config 4: 16M / 140,000^2)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def percentile(v, p):
    v = sorted(v)
    if not v:
        return None
    k = min(len(v) - 1, max(0, int(round(p / 100.0 * (len(v) - 1)))))
    return v[k]


def cpu_baseline(n, L, dist, seed, target_s):
    """oracle (i) (faithful go-aoi XZListAOIManager restatement, C, one thread) on a bounded sample:
    bulk-load tick 0, then time Moved for the first M slots of tick 1 in slot order."""
    import numpy as np
    from oracle import pyoracle
    pyoracle.build()
    x, z = pyoracle.workload_init(seed, n, L)
    orc = pyoracle.XZListOracle(dist, n)
    t = time.perf_counter()
    orc.bulk_enter(np.arange(n, dtype=np.uint32), x, z)
    t_load = time.perf_counter() - t
    orc.set_record(True)
    pyoracle.workload_step(seed, 1, x, z, L, 1.0)
    slots = np.arange(n, dtype=np.uint32)
    m0 = min(n, 2000)
    t = time.perf_counter()
    orc.moved_batch(slots[:m0], x[:m0], z[:m0])
    t0 = time.perf_counter() - t
    m1 = int(min(n - m0, max(0, m0 * (target_s - t0) / max(t0, 1e-9))))
    t = time.perf_counter()
    if m1:
        orc.moved_batch(slots[m0:m0 + m1], x[m0:m0 + m1], z[m0:m0 + m1])
    t1 = time.perf_counter() - t
    ev = orc.take_events()
    orc.close()
    m = m0 + m1
    rate = m / (t0 + t1)
    return {"value": rate, "unit": "entity-updates/s", "cores": 1, "kind": "port",
            "sample": f"oracle (i) go-aoi XZListAOIManager restatement (C, 1 thread): Moved() of slots 0..{m - 1} "
                      f"of tick 1 after a bulk load of N={n} (config 2 state, load {t_load:.1f}s untimed); "
                      f"{m} updates in {t0 + t1:.2f}s, {len(ev)} pair events",
            "cpu": _cpu_model(), "nproc": os.cpu_count()}


def cpu_baseline_spaces(n_per, L, dist, seed0, nspaces, target_s, threads=None):
    """Config 3 on the CPU (one worker per Space, across the cores): oracle (i), one
    XZListAOIManager restatement per Space (C; ctypes drops the GIL), bulk-loaded at tick 0, then `nt`
    all-moving ticks of Moved() in slot order, Spaces handed to `threads` workers (default: every core
    this process may use, host_cores()). `nt` is sized from one calibration tick so the pool runs about
    `target_s`. Rate = updates / wall time of the pool; `value_at_nproc` = the rate scaled linearly to the
    machine's nproc (the Spaces are independent: GOMAXPROCS = nproc, §8(d)), labelled as extrapolated
    when fewer cores were usable."""
    usable, nproc = host_cores()
    if threads is None:  # the process's CPU share (the GPU box sets OMP_NUM_THREADS to it) and usable cores
        threads = min(usable, int(os.environ.get("OMP_NUM_THREADS", usable) or usable))
    import threading

    import numpy as np
    from oracle import pyoracle
    pyoracle.build()

    def space_run(s, nt):
        x, z = pyoracle.workload_init(seed0 + s, n_per, L)
        orc = pyoracle.XZListOracle(dist, n_per)
        slots = np.arange(n_per, dtype=np.uint32)
        orc.bulk_enter(slots, x, z)
        orc.set_record(True)
        ne = 0
        t = time.perf_counter()
        for k in range(1, nt + 1):
            pyoracle.workload_step(seed0 + s, k, x, z, L, 1.0)
            orc.moved_batch(slots, x, z)
            ne += len(orc.take_events())
        dt = time.perf_counter() - t
        orc.close()
        return ne, dt

    _, t_one = space_run(0, 1)  # calibration (and library warm-up), untimed
    nt = int(min(1000, max(1, target_s * threads / max(1e-9, nspaces * t_one))))
    lock = threading.Lock()
    state = {"next": 0, "events": 0}

    def worker():
        while True:
            with lock:
                s = state["next"]
                if s >= nspaces:
                    return
                state["next"] = s + 1
            ne, _ = space_run(s, nt)
            with lock:
                state["events"] += ne

    ts = [threading.Thread(target=worker) for _ in range(threads)]
    t = time.perf_counter()
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    wall = time.perf_counter() - t
    m = nspaces * n_per * nt
    per_core = m / wall / min(threads, usable)
    return {"value": m / wall, "unit": "entity-updates/s", "cores": threads, "kind": "port",
            "usable_cores": usable, "nproc": nproc,
            "value_at_nproc": per_core * nproc,
            "value_at_nproc_note": "measured" if min(threads, usable) >= nproc else
            f"linear extrapolation of the {min(threads, usable)}-core rate to nproc={nproc} (independent Spaces, "
            "one worker per Space); an upper bound for the host",
            "sample": f"oracle (i) go-aoi XZListAOIManager restatement (C), one manager per Space, {threads} worker "
                      f"threads: {nspaces} Spaces x {n_per} (L={L:g}, D={dist:g}, seeds {seed0:#x}+s), each "
                      f"bulk-loaded then {nt} all-moving ticks of Moved(); {m} updates in {wall:.2f}s wall "
                      f"(bulk loads inside the wall time), {state['events']} pair events",
            "cpu": _cpu_model()}


def sink_workers():
    """Worker threads of the sharded host sinks: the process's CPU share (OMP_NUM_THREADS on the GPU box),
    at most the usable cores."""
    usable, _ = host_cores()
    return max(1, min(usable, int(os.environ.get("OMP_NUM_THREADS", usable) or usable), 16))


def host_cores():
    """(usable, nproc): the cores this process may run on (affinity, and the cgroup CPU quota when one is
    set) and the machine's logical CPU count."""
    nproc = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            usable = min(usable, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return usable, nproc


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def lib_stamp(L_):
    """The source stamp compiled into the loaded library (gwaoi_version() ends with "src <hash>")."""
    v = L_.gwaoi_version().decode()
    return v, (v.rsplit(" src ", 1)[1] if " src " in v else None)


def pmc_traffic(workload, n, stamp, kernels=None):
    """HBM bytes per launch of the workload's roofline kernel(s), from the PMC passes summarised in
    profiles/pmc_latest.json (scripts/make_pmc_latest.py), used only when those passes ran the SAME
    library build as this run (the source stamp) at the same size. Returns (bytes or None, note)."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            pmc = json.load(f)
    except Exception as e:
        return None, f"no PMC summary ({e.__class__.__name__})"
    w = pmc.get("workloads", {}).get(workload)
    if w is None:
        return None, f"no PMC pass for workload {workload} in profiles/pmc_latest.json"
    if stamp is None or w.get("lib_src") != stamp:
        return None, (f"stale: the PMC pass ran library src {w.get('lib_src')}, this run loaded src {stamp}; "
                      "traffic withheld")
    if w.get("n") != n:
        return None, f"PMC pass at n={w.get('n')}, this run n={n}; traffic withheld"
    if kernels is None:
        kernels, b = w.get("kernels_summed", []), w.get("bytes_per_launch")
    else:
        kt = w.get("kernels", {})
        b = sum(kt[k]["bytes"] for k in kernels) if all("bytes" in kt.get(k, {}) for k in kernels) else None
    if b is None:
        return None, f"no FETCH_SIZE/WRITE_SIZE for {kernels} in the PMC pass"
    return b, (f"{w.get('source')}: {' + '.join(kernels)}, FETCH_SIZE x 2 (gfx950 wide-read correction) + "
               "WRITE_SIZE, median per launch")


def tick_counter_bytes(workload, n, stamp):
    """HBM bytes per TICK from the same PMC passes (verdict r4): FETCH_SIZE x 2 + WRITE_SIZE summed over
    every kernel that ran once or more per tick there (at least as many dispatches as k_sweep), i.e. the
    whole pipeline's counter traffic, beside SURVEY's formula. None when the passes are stale."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            w = json.load(f).get("workloads", {}).get(workload)
    except Exception:
        return None, None
    if not w or stamp is None or w.get("lib_src") != stamp or w.get("n") != n:
        return None, None
    kt = w.get("kernels", {})
    per_tick = kt.get("k_sweep", {}).get("dispatches")
    if not per_tick:
        return None, None
    # (>= 3/4 of k_sweep's dispatches: the first pass of a run, the bulk Enter, launches no global walk)
    ks = sorted(k for k, e in kt.items() if "bytes" in e and e.get("dispatches", 0) >= 0.75 * per_tick)
    return sum(kt[k]["bytes"] * max(1, round(kt[k]["dispatches"] / per_tick)) for k in ks), ks


def spaces_workload(args, rank):
    """(name, n_per, nspaces, dists, L, seed0, nhot, sigma, hot_every) of a device-staged, all-moving
    workload."""
    if args.workload == "config2":
        return ("config 2: single Space of 1,000,000 entities per GPU, L=35,000, D=100, all moving each tick",
                args.n, 1, [args.dist], args.L, args.seed + rank, 0, 0.0, 10)
    if args.workload == "config3":
        k = args.spaces
        return (f"config 3: {k} independent dungeon Spaces x 2,000 entities per GPU in one manager "
                f"(4,096 Spaces over 8 GPUs), L=1,600 each, D=100",
                2000, k, [100.0] * k, 1600.0, 0x5EED0003 + rank * k, 0, 0.0, 10)
    if args.workload == "skew":
        # 10% of the entities in 64 Gaussian hotspots, sigma 55: peak density ~100x the mean
        # (1,562 per hotspot / (2 pi 55^2) = 0.082 per unit^2 = 100 x 8.2e-4)
        return ("config 5: skewed crowd, 4 Spaces x 1,000,000 per GPU (D = 50/100/200/400), L=35,000, 10% of the "
                "entities in 64 Gaussian hotspots (sigma 55: peak density ~100x the mean)",
                1_000_000, 4, [50.0, 100.0, 200.0, 400.0], 35000.0, 0x5EED0005 + rank * 4, 64, 55.0, 10)
    if args.workload == "skew50":
        # SURVEY.md 8(d) proportions: 50% of the entities in 64 hotspots per Space, sigma 123 for the same
        # ~100x peak (7,812 per hotspot / (2 pi 123^2) = 0.082 per unit^2)
        return ("config 5 (SURVEY proportions): skewed crowd, 4 Spaces x 1,000,000 per GPU (D = 50/100/200/400), "
                "L=35,000, 50% of the entities in 64 Gaussian hotspots per Space (sigma 123: peak density ~100x "
                "the mean)",
                1_000_000, 4, [50.0, 100.0, 200.0, 400.0], 35000.0, 0x5EED0005 + rank * 4, 64, 123.0, 2)
    raise ValueError(args.workload)


def small_pass_leg(eng, n, L, xs, zs, reps, seed):
    """Passes with few ops into the full manager: the Go wrapper flushes every Enter and
    Leave as its own pass (gwaoi.go SyncEnterLeave; Space.go:188-251 calls), and a server may flush a
    handful of Moved calls between ticks. Per repetition: a 1-op Leave of a random present slot, the
    1-op Enter bringing it back at its position, then a 1,000-op Moved pass (distinct random slots, each
    moved by <= 1 unit), host-staged through the wrapper's calls, events left in HBM. Run with small
    passes on (auto: the overlay restarts when ops x overlay grows past its budget, so some 1k passes are
    full) and off (every pass a full pass), for comparison. Device time = the pass's hipEvents
    (stats ms_total), host time = stage + gwaoi_tick_ex wall time."""
    import numpy as np
    rng = np.random.default_rng(seed ^ 0x5A11)
    xs, zs = xs.copy(), zs.copy()
    eng.adopt_device_state()
    eng.set_timing(True)
    out = {}
    for mode, tag in ((1, "small_on"), (0, "small_off")):
        eng.debug_small_pass(mode)
        rec = {"leave_1op": [], "enter_1op": [], "moved_1k": []}
        for _ in range(reps):
            s = int(rng.integers(n))
            mv = np.sort(rng.choice(n, 1000, replace=False)).astype(np.uint32)

            def moved():
                xs[mv] = np.clip(xs[mv] + rng.uniform(-1, 1, mv.size), 0, np.nextafter(np.float32(L), 0))
                zs[mv] = np.clip(zs[mv] + rng.uniform(-1, 1, mv.size), 0, np.nextafter(np.float32(L), 0))
                eng.stage_moves(mv, xs[mv], zs[mv])

            for kind, stage in (("leave_1op", lambda: eng.leave(s)),
                                ("enter_1op", lambda: eng.enter(s, float(xs[s]), float(zs[s]))),
                                ("moved_1k", moved)):
                n0 = eng.debug_small_pass()
                eng.reset_stats()
                t0 = time.perf_counter()
                stage()
                eng.tick_device()
                dt = time.perf_counter() - t0
                st = eng.stats()
                rec[kind].append((eng.debug_small_pass() > n0, st["ms_total"], dt * 1e3, int(eng.last.count),
                                  st["ms_sweep"]))
        res = {}
        for kind, v in rec.items():
            sm = [r for r in v if r[0]]
            fu = [r for r in v if not r[0]]
            res[kind] = {
                "passes": len(v), "small_passes": len(sm),
                "device_ms_p50_small": percentile([r[1] for r in sm], 50) if sm else None,
                "device_ms_p50_full": percentile([r[1] for r in fu], 50) if fu else None,
                "sweep_stage_ms_p50_small": percentile([r[4] for r in sm], 50) if sm else None,
                "host_ms_p50": percentile([r[2] for r in v], 50),
                "events_mean": float(np.mean([r[3] for r in v])),
            }
        if mode == 1:
            # the same 1-op passes with timing off (no hipEvent records between the kernels) and the events
            # delivered to the host, as the Go wrapper's flushed Enter / Leave (gwaoi_tick)
            eng.set_timing(False)
            hl, he = [], []
            for _ in range(reps):
                s = int(rng.integers(n))
                for lst, stage in ((hl, lambda: eng.leave(s)), (he, lambda: eng.enter(s, float(xs[s]), float(zs[s])))):
                    t0 = time.perf_counter()
                    stage()
                    eng.tick_raw()
                    lst.append((time.perf_counter() - t0) * 1e3)
            res["leave_1op"]["host_ms_p50_host_events_no_timing"] = percentile(hl, 50)
            res["enter_1op"]["host_ms_p50_host_events_no_timing"] = percentile(he, 50)
            res["leave_1op"]["host_ms_p99_host_events_no_timing"] = percentile(hl, 99)
            res["enter_1op"]["host_ms_p99_host_events_no_timing"] = percentile(he, 99)
            eng.set_timing(True)
        out[tag] = res
    eng.debug_small_pass(1)
    eng.set_timing(False)
    out["note"] = (
        f"{reps} repetitions per setting of a 1-op Leave, the 1-op Enter bringing the slot back, and a 1,000-op "
        "Moved pass (<= 1 unit each), host-staged, events in HBM, into the full manager; device = the pass's "
        "hipEvents (first to last: the event records between the kernels included), sweep_stage = the hipEvents "
        "around the sweep kernel (a single op: the whole pass, apply + sweep + order + publication, is that one "
        "kernel); host = stage + tick wall time; small_passes = passes that took the small path; "
        "host_ms_*_host_events_no_timing: the same 1-op passes with timing off and the events delivered to "
        "host memory (gwaoi_tick, the Go wrapper's flushed Enter / Leave)")
    return out


def run_spaces(args, rank, world, dev, sync_all, allmax):
    import ctypes

    import numpy as np
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine, wl_init_spaces, wl_iota, wl_step_spaces

    name, n_per, nsp, dists, L, seed0, nhot, sigma, hot_every = spaces_workload(args, rank)
    if args.dists:  # A/B: the same workload with other per-Space distances (one Space per entry)
        dists = [float(v) for v in args.dists.split(",")]
        nsp = len(dists)
        name += f" [dists overridden: {dists}]"
    n = n_per * nsp
    W, K, H = args.warmup, args.steps, args.latency_ticks
    HS = args.host_staged_ticks
    S = min(K, args.stage_ticks)  # instrumented ticks (per-stage hipEvents) after the timed region
    T = W + K + S + H + 1  # (the host-staged and p99 loops generate their positions as they go)
    L_ = _lib.load()

    # ---- untimed setup: positions for every tick generated on the device ----
    t_setup = time.perf_counter()
    snap = DeviceBuffer(2 * 4 * n * T, dev)  # [T][x|z][n] float32
    slots = DeviceBuffer(4 * n, dev)
    wl_iota(dev, slots.ptr, n)

    def px(t):
        return snap.ptr + (2 * t) * 4 * n

    def pz(t):
        return snap.ptr + (2 * t + 1) * 4 * n

    wl_init_spaces(dev, px(0), pz(0), n_per, nsp, seed0, L, nhot, sigma, hot_every)
    for t in range(1, T):
        wl_step_spaces(dev, px(t - 1), pz(t - 1), px(t), pz(t), n_per, nsp, seed0, t, L, 1.0)
    eng = Engine(capacity=n, device=dev, spaces=[(d, (0.0, 0.0, L, L)) for d in dists])
    if args.cells_per_dist:
        eng.debug_set_cells_per_dist(args.cells_per_dist)
    if args.cell_side:
        eng.debug_set_cell_side(args.cell_side)
    if args.sweep_lds != 1:
        eng._L.gwaoi_debug_set_sweep_lds(eng.handle, args.sweep_lds)
    if args.band != 1:  # A/B: the band walk of the global-memory movers off (their whole rings)
        eng.debug_set_band(args.band)
    if args.counting_build:
        eng.debug_build_mode(1)
    # bulk restore (untimed): one device-staged pass of SILENT Enters into their Spaces; the relation
    # is rebuilt without reporting its pairs (billions for config 5 in SURVEY proportions)
    kinds = DeviceBuffer(n, dev)
    kinds.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
    spc = DeviceBuffer(4 * n, dev)
    spc.upload(np.repeat(np.arange(nsp, dtype=np.uint32), n_per))
    log(f"[rank {rank}] {n} entities generated ({time.perf_counter() - t_setup:.1f}s); running the Enter pass")
    eng.stage_ops_device(slots.ptr, px(0), pz(0), kinds.ptr, n, spc.ptr)
    eng.tick_device()
    kinds.free()
    spc.free()
    log(f"[rank {rank}] setup {time.perf_counter() - t_setup:.1f}s: {eng.count()[0]} entities in {nsp} Spaces")

    def tick_dev(t):
        eng.stage_moves_device(slots.ptr, px(t), pz(t), n)
        return eng.tick_device()

    for t in range(1, W + 1):
        tick_dev(t)

    # ---- timed region: K ticks, events left in HBM (no per-stage hipEvents: recording and reading them
    # sits on the host's path between ticks) ----
    sync_all()
    lat = []
    t0 = time.perf_counter()
    for t in range(W + 1, W + K + 1):
        ts = time.perf_counter()
        tick_dev(t)
        lat.append(time.perf_counter() - ts)
    sync_all()
    elapsed = allmax(time.perf_counter() - t0)
    log(f"[rank {rank}] timed {K} ticks in {elapsed:.3f}s")
    # ---- the next S ticks of the same walk with per-stage hipEvents (stage_ms, the roofline's kernel time) ----
    eng.set_timing(True)
    eng.reset_stats()
    for t in range(W + K + 1, W + K + S + 1):
        tick_dev(t)
    st = eng.stats()
    eng.set_timing(False)

    if rank == 0:
        occ, ldsb = ctypes.c_int(0), ctypes.c_int(0)
        if L_.gwaoi_debug_sweep_occupancy(dev, ctypes.byref(occ), ctypes.byref(ldsb)) == 0:
            log(f"[rank 0] sweep: {occ.value} resident blocks per CU, {ldsb.value} B LDS per block")
    if args.stamps and rank == 0:
        buf = np.zeros(16 * 16384, dtype=np.uint64)
        _lib.check(L_.gwaoi_debug_read_stamps(buf.ctypes.data, buf.nbytes))
        np.save(args.stamps, buf.reshape(-1, 16))

    # ---- host-delivered latency (PCIe-inclusive; reported, never `value`) ----
    lat_host = []
    for t in range(W + K + S + 1, W + K + S + H + 1):
        ts = time.perf_counter()
        eng.stage_moves_device(slots.ptr, px(t), pz(t), n)
        eng.tick_raw()
        lat_host.append(time.perf_counter() - ts)

    # the walk continues after the staged ticks, each tick's positions generated on the device (and
    # synchronised) before its clock starts: two [x|z][n] tick slots, ping-pong
    walk = DeviceBuffer(2 * 2 * 4 * n, dev)
    wstate = {"prev": (px(T - 1), pz(T - 1)), "t": T, "k": 0}

    def walk_next():
        k = wstate["k"]
        bx, bz = walk.ptr + (2 * k) * 4 * n, walk.ptr + (2 * k + 1) * 4 * n
        wl_step_spaces(dev, *wstate["prev"], bx, bz, n_per, nsp, seed0, wstate["t"], L, 1.0)
        wstate.update(prev=(bx, bz), t=wstate["t"] + 1, k=k ^ 1)
        return bx, bz

    # ---- SURVEY 8(d) p99, the headline: from the positions in host memory through the cgo wrapper's one
    # staging call per tick to the events in the pinned host buffer, over HS >= 1,000 ticks; the first
    # --replay-ticks of them also replayed into per-entity hash sets (tools/replay_sets.c:
    # Entity.interest/uninterest, 4 set ops per pair event, Entity.go:227-246) ----
    lat_hs, stage_hs, replay_s, replay_bad = [], [], [], 0
    replay_sh_s, replay_sh_bad = [], 0
    rs = rss = None
    sink_threads = sink_workers()
    if HS and args.replay and nsp == 1:
        try:
            from tools.replay import ReplaySets, ShardedReplaySets
            rp_h, cols_h = eng.relation()
            rs = ReplaySets(2 * len(cols_h))
            t_ld = time.perf_counter()
            rs.load_relation(rp_h, cols_h)
            log(f"[rank {rank}] replay sets: {rs.size()} entries loaded in {time.perf_counter() - t_ld:.1f}s")
            rss = ShardedReplaySets(2 * len(cols_h), sink_threads)
            rss.load_relation(rp_h, cols_h)
            del rp_h, cols_h
        except Exception as e:  # the tool is a bench aid: report, never fail the GPU line
            log(f"[rank {rank}] replay sets unavailable: {e!r}")
            rs = rss = None
    if HS:
        eng.adopt_device_state()  # the restore was a device batch: host staging from here on
    # the cgo wrapper's path: Moved calls written into the manager's pinned staging arrays as the client
    # packets arrive (here: the tick's positions copied in, untimed), then ONE gwaoi_stage_moves_pinned
    # (one DMA copy, validation and repeat detection on the GPU). The last `copyin` ticks use the
    # copy-in gwaoi_stage_moves (host validation) from plain host arrays instead, for comparison.
    slots_h = np.arange(n, dtype=np.uint32)
    xh = np.empty(n, np.float32)
    zh = np.empty(n, np.float32)
    pin_s = pin_x = pin_z = None
    if HS:
        pin_s, pin_x, pin_z = eng.stage_buffers()
        pin_s[:n] = slots_h
    # The headline ticks stage with gwaoi_stage_moves_pinned_async (ABI 2.1: the DMA copy, the device checks
    # and the pipeline enqueued back to back, the checks' verdict read by the pass); then `syncpin` ticks
    # with the synchronous gwaoi_stage_moves_pinned (its verdict read back before the pipeline starts) and
    # `copyin` ticks with the copy-in gwaoi_stage_moves (host validation), for comparison.
    async_ok = hasattr(L_, "gwaoi_stage_moves_pinned_async") and args.pin_mode == "async"
    copyin = min(10, HS // 2)
    syncpin = min(100, HS // 2) if async_ok else 0
    stage_ci, lat_sp, stage_sp = [], [], []
    for i in range(HS + syncpin + copyin):
        use_pin = i < HS + syncpin
        dx, dz = (pin_x, pin_z) if use_pin else (xh, zh)
        bx, bz = walk_next()  # untimed: the tick's positions into the host arrays
        _lib.check(L_.gwaoi_dev_dtoh(dev, dx.ctypes.data, ctypes.c_void_p(bx), 4 * n))
        _lib.check(L_.gwaoi_dev_dtoh(dev, dz.ctypes.data, ctypes.c_void_p(bz), 4 * n))
        ts = time.perf_counter()
        if use_pin and async_ok and i < HS:
            eng.stage_moves_pinned_async(n)
        elif use_pin:
            eng.stage_moves_pinned(n)
        else:
            eng.stage_moves(slots_h, xh, zh)
        t1 = time.perf_counter()
        ev = eng.tick_raw()
        te = time.perf_counter()
        if i < HS:
            lat_hs.append(te - ts)
            stage_hs.append(t1 - ts)
        elif use_pin:
            lat_sp.append(te - ts)
            stage_sp.append(t1 - ts)
        else:
            stage_ci.append(t1 - ts)
        if rs is not None and ev.count:
            tr = time.perf_counter()
            replay_bad += rs.replay(ctypes.cast(ev.events, ctypes.c_void_p).value, int(ev.count))
            replay_s.append(time.perf_counter() - tr)
        if rss is not None and ev.count:
            tr = time.perf_counter()
            replay_sh_bad += rss.replay(ctypes.cast(ev.events, ctypes.c_void_p).value, int(ev.count))
            replay_sh_s.append(time.perf_counter() - tr)
        if (rs is not None or rss is not None) and i + 1 >= args.replay_ticks:  # the sets stop following here
            if rs is not None:
                rs.close()
            if rss is not None:
                rss.close()
            rs = rss = None
    if rs is not None:
        rs.close()
    if rss is not None:
        rss.close()

    # ---- positions arriving over the tick (GameService.go:398-410: one position packet at a time): the tick's
    # Moved calls written into the pinned arrays in `chunks` parts, each part pushed when it has arrived
    # (gwaoi_stage_moves_pinned_partial, asynchronous DMA) and the arrivals spread over more time than the
    # pushes take (the device synchronised, untimed); timed: the Flush, i.e. the async staging of the whole
    # batch (only the last part still to copy) + gwaoi_tick, to the events in pinned host memory ----
    lat_ck = []
    CK = args.chunked_ticks if (HS and async_ok and hasattr(L_, "gwaoi_stage_moves_pinned_partial")) else 0
    nchunks = max(1, args.chunks)
    for i in range(CK):
        bx, bz = walk_next()
        _lib.check(L_.gwaoi_dev_dtoh(dev, pin_x.ctypes.data, ctypes.c_void_p(bx), 4 * n))
        _lib.check(L_.gwaoi_dev_dtoh(dev, pin_z.ctypes.data, ctypes.c_void_p(bz), 4 * n))
        for c in range(1, nchunks):
            eng.stage_moves_pinned_partial(n * c // nchunks)
        _lib.check(L_.gwaoi_dev_sync(dev))
        ts = time.perf_counter()
        eng.stage_moves_pinned_async(n)
        eng.tick_raw()
        lat_ck.append(time.perf_counter() - ts)

    # ---- device-resident p50/p99 (p99_tick_ms_device): a fixed loop of P ticks (events left in HBM),
    # independent of --steps ----
    lat_p = []
    for _ in range(args.p99_ticks):
        bx, bz = walk_next()
        ts = time.perf_counter()
        eng.stage_moves_device(slots.ptr, bx, bz, n)
        eng.tick_device()
        lat_p.append(time.perf_counter() - ts)

    # relation size for the SURVEY §8(d) formula (directed entries |S|)
    nnz = None
    rel_ms = rel_upd_ms = rel_upd_n = rel_delta_ms = rel_delta_n = rel_export_ms = rel_apply_ms = None
    rel_apply_mt_ms = None
    dr_bad = None
    if args.workload in ("config2", "config3"):  # config 5's relation runs to billions of entries
        # the relation as a device-resident CSR (SURVEY 8(f)3 view), timed host-side incl. its syncs:
        # rebuilt from the grid (mode 1, every call), then kept up to date from each tick's events
        eng.debug_relation_mode(1)
        eng.relation_device()
        L_.gwaoi_dev_sync(dev)
        reps = []
        for _ in range(5):
            t0 = time.perf_counter()
            nnz = eng.relation_device()[2]
            L_.gwaoi_dev_sync(dev)
            reps.append(time.perf_counter() - t0)
        rel_ms = sorted(reps)[len(reps) // 2] * 1e3
        eng.debug_relation_mode(0)
        n_inc0 = eng.debug_relation_mode()[0]
        reps, dreps, dlen, areps, areps_mt = [], [], [], [], []
        dr = None
        try:  # the consumer by delta on the host: per-slot sorted neighbour arrays (tools/delta_rows.c)
            from tools.replay import DeltaRows
            dr = DeltaRows(*eng.relation())
        except Exception as e:  # a bench aid: report, never fail the GPU line
            log(f"[rank {rank}] delta rows unavailable: {e!r}")
        dr_bad = 0
        for j in range(10):  # more ticks of the walk
            bx, bz = walk_next()
            eng.stage_moves_device(slots.ptr, bx, bz, n)
            eng.tick_device()
            L_.gwaoi_dev_sync(dev)
            # the consumer by delta: the tick's net relation changes, computed from its events in HBM
            # and copied to the host (gwaoi_export_relation_delta)
            t0 = time.perf_counter()
            dl = eng.relation_delta(cap=4 * n)
            dreps.append(time.perf_counter() - t0)
            dlen.append(len(dl))
            if dr is not None:  # (alternate ticks: one thread, then the rows over sink_threads workers)
                t0 = time.perf_counter()
                dr_bad += dr.apply(dl, threads=1 if j % 2 == 0 else sink_threads)
                (areps if j % 2 == 0 else areps_mt).append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            eng.relation_device()
            L_.gwaoi_dev_sync(dev)
            reps.append(time.perf_counter() - t0)
        rel_upd_ms = sorted(reps)[len(reps) // 2] * 1e3
        rel_delta_ms = sorted(dreps)[len(dreps) // 2] * 1e3
        rel_delta_n = float(np.mean(dlen))
        rel_apply_ms = sorted(areps)[len(areps) // 2] * 1e3 if areps else None
        rel_apply_mt_ms = sorted(areps_mt)[len(areps_mt) // 2] * 1e3 if areps_mt else None
        if dr is not None:
            dr_bad += dr.diff(*eng.relation())  # the patched arrays must equal the relation now
            dr.close()
        rel_upd_n = eng.debug_relation_mode()[0] - n_inc0
        # the whole relation copied to the host (gwaoi_export_relation: row_ptr + cols, ~130 MB at 1M)
        reps = []
        for _ in range(3):
            t0 = time.perf_counter()
            eng.relation()
            reps.append(time.perf_counter() - t0)
        rel_export_ms = sorted(reps)[1] * 1e3
    small = None
    if (args.workload in ("config2", "config3") and args.small_reps > 0 and nsp == 1
            and hasattr(L_, "gwaoi_debug_set_small_pass")):
        kp = wstate["k"] ^ 1  # the walk's last positions
        xs = walk.download(np.float32, n, (2 * kp) * 4 * n)
        zs = walk.download(np.float32, n, (2 * kp + 1) * 4 * n)
        small = small_pass_leg(eng, n, L, xs, zs, args.small_reps, seed0)
    eng.close()
    walk.free()
    if rank != 0:
        return None

    ms_step = elapsed / K * 1e3
    ticks = max(1, st["ticks"])
    sweep_ms = st["ms_sweep"] / ticks
    ev_per_tick = st["events"] / ticks
    # algorithmic bytes of ONE sweep launch (DESIGN.md "Measurement"): every record of the pass's
    # cell-sorted grid read once (32 B: binned + start state), every cell start once (4 B), the
    # per-op event count written (4 B per mover), every event staged once (16 B).
    rec_per_tick = st["grid_records"] / ticks
    cells = st["grid_cells"] / ticks
    b_sweep = 32.0 * rec_per_tick + 4.0 * cells + 4.0 * n + 16.0 * ev_per_tick
    achieved = b_sweep / (sweep_ms * 1e-3) / 1e9
    lib_v, stamp = lib_stamp(L_)
    t_bytes, t_note = pmc_traffic(args.workload if not args.dists else None, n, stamp)
    traffic = t_bytes / (sweep_ms * 1e-3) / 1e9 if t_bytes else None  # GB/s, same unit as achieved
    tick_bytes, tick_kernels = tick_counter_bytes(args.workload if not args.dists else None, n, stamp)
    # SURVEY.md §8(d) whole-tick formula (assumes a CSR-state design; ours keeps no lists)
    b_survey = 24.0 * n + 4.0 * (2 * nnz) + 8.0 * ev_per_tick if nnz is not None else None
    return {
        "metric": METRIC,
        "value": n * K * world / elapsed,
        "unit": "entity-updates/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": DATA,
        "config": {
            "workload": name,
            "entities_per_gpu": n, "spaces_per_gpu": nsp, "world_L": L, "aoi_dist": dists if nsp > 1 else dists[0],
            "seed": hex(seed0 - rank * (nsp if nsp > 1 else 1)),
            "parallelism": "independent Spaces, one manager per GPU, no data-path collective" if world > 1 else "1 GPU",
        },
        "p50_tick_ms": percentile(lat_hs or lat_p or lat, 50) * 1e3,
        "p99_tick_ms": percentile(lat_hs or lat_p or lat, 99) * 1e3,
        "p99_samples": len(lat_hs or lat_p or lat),
        "p99_note": (f"SURVEY 8(d): host wall time from the positions in host memory to the events in host memory, "
                     f"{len(lat_hs)} ticks after the timed region (the tick's positions written into the manager's "
                     "pinned staging arrays, untimed; gwaoi_stage_moves_pinned + gwaoi_tick = one DMA copy in, the "
                     "pipeline, the events copied into pinned host memory by the GPU)" if lat_hs else
                     f"host wall time of {len(lat_p)} device-resident ticks" if lat_p else "over the timed ticks"),
        "p50_tick_ms_device": percentile(lat_p, 50) * 1e3 if lat_p else None,
        "p99_tick_ms_device": percentile(lat_p, 99) * 1e3 if lat_p else None,
        "p99_device_note": (f"host wall time of {len(lat_p)} device-resident ticks (stage_moves_device -> events "
                            "ordered in HBM, count on the host), each tick's positions generated before its clock "
                            "starts") if lat_p else None,
        "p50_tick_ms_timed": percentile(lat, 50) * 1e3,
        "p99_tick_ms_timed": percentile(lat, 99) * 1e3,
        "p50_tick_ms_host_events": percentile(lat_host, 50) * 1e3 if lat_host else None,
        "p99_tick_ms_host_events": percentile(lat_host, 99) * 1e3 if lat_host else None,
        "host_stage_ms": percentile(stage_hs, 50) * 1e3 if stage_hs else None,
        "host_staging_call": ("gwaoi_stage_moves_pinned_async" if async_ok else "gwaoi_stage_moves_pinned") if lat_hs else None,
        "p50_tick_ms_sync_staging": percentile(lat_sp, 50) * 1e3 if lat_sp else None,
        "p99_tick_ms_sync_staging": percentile(lat_sp, 99) * 1e3 if lat_sp else None,
        "host_stage_ms_sync_staging": percentile(stage_sp, 50) * 1e3 if stage_sp else None,
        "sync_staging_note": (f"{len(lat_sp)} host-staged ticks with the synchronous gwaoi_stage_moves_pinned (the "
                              "device check's verdict read back before the pipeline is launched), after the headline "
                              "ticks") if lat_sp else None,
        "p50_flush_ms_chunked": percentile(lat_ck, 50) * 1e3 if lat_ck else None,
        "p99_flush_ms_chunked": percentile(lat_ck, 99) * 1e3 if lat_ck else None,
        "chunked_note": (f"positions arriving over the tick: {len(lat_ck)} ticks, each batch written into the pinned "
                         f"arrays in {nchunks} parts pushed as they arrive (gwaoi_stage_moves_pinned_partial, "
                         "asynchronous DMA; arrivals slower than the pushes: the device synchronised, untimed); "
                         "timed from the Flush (gwaoi_stage_moves_pinned_async of the whole batch, only the last "
                         "part left to copy, + gwaoi_tick) to the events in pinned host memory") if lat_ck else None,
        "host_stage_copyin_ms": percentile(stage_ci, 50) * 1e3 if stage_ci else None,
        "replay_ms": percentile(replay_s, 50) * 1e3 if replay_s else None,
        "replay_ms_sharded": percentile(replay_sh_s, 50) * 1e3 if replay_sh_s else None,
        "replay_sharded_note": (f"the same set operations split by owning entity over {sink_threads} worker threads "
                                f"(tools/replay_sets.c rs_sharded_*); {replay_sh_bad} inconsistent set ops")
        if replay_sh_s else None,
        "replay_note": ("events replayed into per-entity InterestedIn/InterestedBy hash sets in C, 4 set ops per "
                        "pair event (tools/replay_sets.c); host_staged = gwaoi_stage_moves_pinned (the positions "
                        "written into the manager's pinned staging arrays; one DMA copy, validated on the GPU) -> "
                        f"events in pinned host memory, {len(lat_hs)} ticks; host_stage_copyin_ms = the copy-in "
                        f"gwaoi_stage_moves (host validation), {len(stage_ci)} ticks" + (f"; {replay_bad} inconsistent set ops"
                                                                          if replay_s else "")) if lat_hs else None,
        "events_per_tick": ev_per_tick,
        "relation_directed_entries": nnz,
        "relation_view_ms": rel_ms,
        "relation_update_ms": rel_upd_ms,
        "relation_delta_ms": rel_delta_ms,
        "relation_delta_entries": rel_delta_n,
        "relation_export_ms": rel_export_ms,
        "relation_delta_apply_ms": rel_apply_ms,
        "relation_delta_apply_ms_threads": rel_apply_mt_ms,
        "sink_threads": sink_threads,
        "relation_delta_inconsistent": dr_bad,
        "relation_consumer_note": None if rel_delta_ms is None else
        "relation_delta_ms = gwaoi_export_relation_delta (net changes of the tick from its events in HBM, "
        "O(events), into host memory); relation_delta_apply_ms = those entries patched into per-slot sorted "
        "neighbour arrays on the host (tools/delta_rows.c, the Go Sets consumer; relation_delta_inconsistent = "
        "bad entries + rows differing from the relation afterwards, 0 expected); relation_export_ms = "
        "gwaoi_export_relation (the whole CSR to the host)",
        "relation_update_note": None if rel_upd_ms is None else
        f"view updated from each tick's events (k_rd_*), {rel_upd_n}/10 ticks incremental; "
        "relation_view_ms = rebuilt from the grid",
        "stage_ms": {k: st[k] / ticks for k in ("ms_apply", "ms_grid", "ms_sweep", "ms_order", "ms_total")},
        "stage_ms_note": f"per-stage hipEvents over {ticks} ticks of the same walk run after the timed region "
                         "(the timed ticks run without them)",
        "small_pass": small,
        "roofline": {
            "bound": "hbm",
            "kernel": "k_sweep",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_bytes_per_launch": t_bytes if traffic else None,
            "traffic_note": t_note,
            "algorithmic_bytes_per_launch": b_sweep,
            "grid_records_per_tick": rec_per_tick,
            "grid_cells": cells,
            "dense_movers_per_tick": st["dense_movers"] / ticks,
            "band_movers_per_tick": st["band_movers"] / ticks,
            "avg_launch_ms": sweep_ms,
            "kernels_timed": "k_sweep" +
                             (" + k_sweep<SwMid> + k_sweep<SwBig>" if args.workload in ("skew", "skew50") else "") +
                             (" + k_band_sort + k_sweep_band" if st["band_movers"] else "") +
                             (" + k_sweep_dense" if st["dense_movers"] else "") +
                             " (the pass's sweep stage, hipEvents on the manager's stream)",
            "tick_counter_bytes": tick_bytes,
            "tick_counter_GBps": tick_bytes / (ms_step * 1e-3) / 1e9 if tick_bytes else None,
            "tick_counter_note": (f"PMC bytes per tick of every per-tick kernel ({len(tick_kernels)}: "
                                  f"{', '.join(tick_kernels)}) over ms_per_step") if tick_bytes else None,
            "survey_formula": None if b_survey is None else {
                "bytes_per_tick": b_survey,
                "achieved_GBps_over_tick": b_survey / (ms_step * 1e-3) / 1e9,
                "frac": b_survey / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "note": "B_alg = 24N + 4(|S0|+|SB|) + 8|E| of SURVEY.md §8(d); counts CSR list traffic this "
                        "design does not have (relation is recomputed from positions + op order)",
            },
        },
        "lib": lib_v,
        "cpu_baseline": None,
    }


def run_gametick(args, rank, world, dev, sync_all, allmax):
    """One GoWorld game tick per step at config-2 scale (SURVEY.md 8(f) rows 1-2 around the AOI path):
    the tick's client position records (32 B each, [EntityID | x y z yaw], resident in HBM) are ingested
    (HandleSyncPositionYawFromClient, GameService.go:398-410), the AOI tick runs, and the sync fan-out
    (CollectEntitySyncInfos, Entity.go:1221-1267) writes every gate's packet body into HBM."""
    import numpy as np
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine, wl_init_spaces, wl_iota, wl_step_spaces
    from goworld_amd.sync import EntitySync

    n, L, D = args.n, args.L, args.dist
    seed = args.seed + rank
    W, K = args.warmup, args.steps
    S = min(K, args.stage_ticks)  # instrumented steps (per-stage hipEvents) after the timed region
    T = W + K + S + 1
    L_ = _lib.load()
    t_setup = time.perf_counter()
    snap = DeviceBuffer(2 * 4 * n * T, dev)
    slots = DeviceBuffer(4 * n, dev)
    wl_iota(dev, slots.ptr, n)

    def px(t):
        return snap.ptr + (2 * t) * 4 * n

    def pz(t):
        return snap.ptr + (2 * t + 1) * 4 * n

    wl_init_spaces(dev, px(0), pz(0), n, 1, seed, L, 0, 0.0, 10)
    for t in range(1, T):
        wl_step_spaces(dev, px(t - 1), pz(t - 1), px(t), pz(t), n, 1, seed, t, L, 1.0)
    # entity ids: slot number in the first 4 bytes, a fixed tag after; clients: a fraction of the slots
    ids = np.zeros((n, 16), np.uint8)
    ids[:, :4] = np.arange(n, dtype=np.uint32).view(np.uint8).reshape(n, 4)
    ids[:, 4:] = np.frombuffer(b"GWAOI-ENTITY", np.uint8)
    d_ids = DeviceBuffer(16 * n, dev)
    d_ids.upload(ids)
    payload = DeviceBuffer(32 * n * T, dev)
    for t in range(1, T):
        _lib.check(L_.gwaoi_wl_pack_ingest(dev, d_ids.ptr, px(t), pz(t), n, t, payload.ptr + 32 * n * t))
    eng = Engine(capacity=n, device=dev, spaces=[(D, (0.0, 0.0, L, L))])
    kinds = DeviceBuffer(n, dev)
    kinds.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
    eng.stage_ops_device(slots.ptr, px(0), pz(0), kinds.ptr, n)
    eng.tick_device()
    kinds.free()
    sy = EntitySync(eng, args.gates)
    if hasattr(L_, "gwaoi_debug_set_fanout_mode"):
        sy.debug_fanout_mode(args.fanout)
    direct = args.fanout == 0 and args.gates <= 8 and hasattr(L_, "gwaoi_debug_set_fanout_mode")
    all_slots = np.arange(n, dtype=np.uint32)
    sy.set_entities(all_slots, ids)
    has_client = (all_slots.astype(np.uint64) * 2654435761 % 1000) < int(args.client_frac * 1000)
    gates = np.where(has_client, all_slots % args.gates, _lib.GWAOI_SYNC_NO_CLIENT).astype(np.uint16)
    sy.set_clients(all_slots, gates, ids[:, ::-1].copy())
    sy.set_client_syncing(all_slots, np.ones(n, np.uint8))
    log(f"[rank {rank}] gametick setup {time.perf_counter() - t_setup:.1f}s: {n} entities, "
        f"{int(has_client.sum())} with clients on {args.gates} gates")

    def step(t, lat):
        t0 = time.perf_counter()
        r = sy.ingest_device(payload.ptr + 32 * n * t, 32 * n)
        t1 = time.perf_counter()
        eng.tick_device()
        t2 = time.perf_counter()
        o = sy.collect_raw(0)
        t3 = time.perf_counter()
        if lat is not None:
            lat.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0, int(o.n_records), int(r.n_moved)))

    for t in range(1, W + 1):
        step(t, None)
    sync_all()
    lat = []
    t0 = time.perf_counter()
    for t in range(W + 1, W + K + 1):
        step(t, lat)
    sync_all()
    elapsed = allmax(time.perf_counter() - t0)
    # per-stage device times: the next S steps with hipEvents on (they cost host time between kernels)
    eng.set_timing(True)
    eng.reset_stats()
    sy.reset_stats()
    for t in range(W + K + 1, W + K + S + 1):
        step(t, None)
    st = eng.stats()
    ss = sy.stats()
    eng.set_timing(False)
    eng.close()
    if rank != 0:
        return None
    a = np.asarray(lat, dtype=np.float64)
    ms = a[:, :4].mean(axis=0) * 1e3
    recs = float(a[:, 4].mean())
    moved = float(a[:, 5].mean())
    ticks = max(1, st["ticks"])
    rec_grid = st["grid_records"] / ticks
    # Device time per stage (hipEvents on the manager's stream, gwaoi_sync_get_stats) and algorithmic
    # bytes per launch (DESIGN.md "Sync fan-out"):
    #  write walk (k_fan_tile<true>): grid record read (x z slot 16 B + seq 4 B + scanned count 4 B) per
    #    record walked + per collected entity flag/gate 3 B, EntityID/Y/yaw 24 B read, info 32 B written
    #    + 8 B per pair written + the client sub-grid records (16 B) staged once;
    #  gate partition (k_gate_hist + k_gate_scatter): per record the pair (8 B) and its gate (1 B), the
    #    receiver's ClientID (16 B) and the entity's info (32 B) gathered, the 48-B record written;
    #  ingest: payload read (32 B) + hash probe (16 B key + 4 B slot) + staged Moved (12 B) + flag/y/yaw (9 B).
    #  direct write pass (k_fan_dwrite, n_gates <= 8): per record walked its 16-B binned record, collected
    #    bits (1 B) and per-gate counts (4 B x gates rounded up to 4); per collected entity gate 2 B +
    #    EntityID/Y/yaw 24 B; per wire record 48 B written + the receiver's ClientID (16 B) gathered; the
    #    client sub-grid records (16 B + gate 1 B) staged once.
    nc = max(1, ss["collects"])
    ents = ss["entities"] / nc
    n_client = float(has_client.sum())
    d_write = ss["ms_write"] / nc
    d_gate = ss["ms_gate"] / nc
    d_cg = ss["ms_client_grid"] / nc
    d_count = ss["ms_count"] / nc
    d_ing = ss["ms_ingest"] / max(1, ss["ingests"])
    b_write = 24.0 * rec_grid + 59.0 * ents + 8.0 * recs + 16.0 * n_client
    b_gate = (8.0 + 1.0 + 16.0 + 32.0 + 48.0) * recs
    b_ing = (32.0 + 20.0 + 12.0 + 9.0) * n
    gbs = lambda b, d: b / (d * 1e-3) / 1e9 if d > 0 else 0.0
    if direct:
        gstride = (args.gates + 3) // 4 * 4
        b_dwrite = (17.0 + 4.0 * gstride) * rec_grid + 26.0 * ents + 64.0 * recs + 17.0 * n_client
        stages = {"write_walk": (d_write, b_dwrite, "k_fan_dwrite")}
    else:
        stages = {"write_walk": (d_write, b_write, "k_fan_tile<true>"),
                  "gate_partition": (d_gate, b_gate, "k_gate_hist + k_gate_scatter")}
    dom = max(stages, key=lambda k: stages[k][0])
    dd, db, dk = stages[dom]
    ach = gbs(db, dd)
    lib_v, stamp = lib_stamp(L_)
    t_bytes, t_note = pmc_traffic("gametick", n, stamp, [dk] if dom == "write_walk" else ["k_gate_hist", "k_gate_scatter"])
    return {
        "metric": "GoWorld game tick (client position ingest + AOI tick + sync fan-out) entity-updates/s at 1M "
                  "entities per Space",
        "value": n * K * world / elapsed,
        "unit": "entity-updates/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": DATA + "; ingest payload packed on device (32-B records, slot order)",
        "config": {
            "workload": f"game tick at config 2 scale: {n} entities, L={L:.0f}, D={D}, every entity's client sends "
                        f"its position each tick; {args.client_frac:.0%} of the entities have a client, "
                        f"{args.gates} gates",
            "entities_per_gpu": n, "world_L": L, "aoi_dist": D, "seed": hex(seed - rank),
            "client_frac": args.client_frac, "gates": args.gates,
            "parallelism": "independent Spaces, one manager per GPU" if world > 1 else "1 GPU",
        },
        "p50_step_ms": percentile(list(a[:, 3] * 1e3), 50),
        "p99_step_ms": percentile(list(a[:, 3] * 1e3), 99),
        "stage_ms": {"ingest": ms[0], "aoi_tick": ms[1], "collect_sync": ms[2]},
        "aoi_stage_ms": {k: st[k] / ticks for k in ("ms_apply", "ms_grid", "ms_sweep", "ms_order", "ms_total")},
        "moved_per_tick": moved,
        "sync_records_per_tick": recs,
        "sync_bytes_per_tick": 48.0 * recs,
        "events_per_tick": st["events"] / ticks,
        "device_stage_ms": {"ingest": d_ing, "client_grid": d_cg, "count_walk": d_count, "write_walk": d_write,
                            "gate_partition": d_gate},
        "fanout": "direct (records written into the gate packets: k_fan_dcount, scan, k_fan_dwrite)" if direct else
                  "pair list + gate partition (k_fan_tile, k_gate_hist, k_gate_scatter)",
        "roofline": {
            "bound": "hbm", "kernel": dk, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "traffic": gbs(t_bytes, dd) if t_bytes else None,
            "traffic_bytes_per_launch": t_bytes, "traffic_note": t_note, "algorithmic_bytes_per_launch": db,
            "avg_launch_ms": dd, "timing": "hipEvents on the manager's stream (gwaoi_sync_get_stats)",
            "stages": {k: {"kernel": v[2], "ms": v[0], "algorithmic_bytes": v[1], "achieved": gbs(v[1], v[0]),
                           "frac": gbs(v[1], v[0]) / HBM_PEAK_GBS} for k, v in stages.items()}
                      | {"ingest": {"ms": d_ing, "algorithmic_bytes": b_ing, "achieved": gbs(b_ing, d_ing),
                                    "frac": gbs(b_ing, d_ing) / HBM_PEAK_GBS}},
        },
        "lib": lib_v,
        "cpu_baseline": None,
    }


def run_strips(args, rank, world, dev, sync_all, allmax, via_cpu):
    """config 4: one world of per_gpu * world entities (density of config 2) in X-strips, one per rank.
    strips_skew (config 5 in strips): the same world with 10% of the entities in Gaussian hotspots
    (sigma 55, ~1,560 entities each: peak ~100x the mean density) and the strip edges at the
    x-quantiles of the entities. On GPUs the halo exchange is gwaoi_strip_exchange (RCCL p2p inside
    libgwaoi, enqueued on the strip's stream: StripNode.tick_rccl); via_cpu (several ranks on one GPU,
    gloo) keeps the host-driven exchange."""
    import numpy as np
    import torch
    from goworld_amd.strips import StripComm, StripLayout, StripNode, exchange_dist

    n = args.per_gpu * world
    L = float(math.sqrt(n / DENSITY))
    W, K = args.warmup, args.steps
    skew = None
    seed = args.seed_strips
    t_setup = time.perf_counter()
    if args.workload == "strips_skew":
        from goworld_amd.engine import DeviceBuffer, wl_init_spaces
        seed = args.seed_strips + 0x50
        skew = (max(1, round(n / 15625)), 55.0, 10)
        bx, bz = DeviceBuffer(4 * n, dev), DeviceBuffer(4 * n, dev)
        wl_init_spaces(dev, bx.ptr, bz.ptr, n, 1, seed, L, *skew)
        lay = StripLayout.from_quantiles(world, bx.download(np.float32, n), L, args.dist, 1.0)
        bx.free()
        bz.free()
    else:
        lay = StripLayout(world, L, args.dist, 1.0)
    nd = StripNode(lay, rank, n, device=dev, seed=seed, skew=skew)
    if args.counting_build:
        nd.eng.debug_build_mode(1)
    comm = None
    if not via_cpu:
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        comm = StripComm.from_dist(rank, world, dev) if world > 1 else StripComm(StripComm.make_id(), 1, 0, dev)
    ev0 = nd.start()
    log(f"[rank {rank}] strips setup {time.perf_counter() - t_setup:.1f}s: world {n} entities, L={L:.0f}, "
        f"{nd.last_ops} in this region, {int(ev0.count)} owned enter pairs")

    def tick(t, time_exchange=False):
        if comm is not None:
            ev = nd.tick_rccl(t, comm, time_exchange=time_exchange)
            return ev, 0  # halo counts are read from the device after the run
        lo, ro = nd.prepare(t)
        if world > 1:
            li, ri = exchange_dist(lo, ro, rank, world, via_cpu=via_cpu)
        else:
            li = ri = None
        return nd.finish(li, ri), int(lo.shape[0] + ro.shape[0])

    for t in range(1, W + 1):
        tick(t)
    sync_all()
    lat, sent, ops, evs = [], 0, 0, 0
    t0 = time.perf_counter()
    for t in range(W + 1, W + K + 1):
        ts = time.perf_counter()
        ev, k = tick(t)
        lat.append(time.perf_counter() - ts)
        sent += k
        ops += nd.last_ops
        evs += int(ev.count)
    sync_all()
    elapsed = allmax(time.perf_counter() - t0)
    # per-stage hipEvents over the next ticks of the walk (every rank runs them: the exchange is collective)
    S = min(K, args.stage_ticks)
    nd.eng.set_timing(True)
    nd.eng.reset_stats()
    for t in range(W + K + 1, W + K + S + 1):
        tick(t, time_exchange=True)
    st = nd.eng.stats()
    nd.eng.set_timing(False)
    xms = nd.exchange_ms() if comm is not None else None
    if comm is not None:  # the last tick's halo sizes (the RCCL path keeps them on the device)
        sent = int(nd.counts[:2].sum().item()) * K
    nd.close()
    if comm is not None:
        comm.close()
    if world > 1:
        import torch.distributed as dist
        tot = torch.tensor([evs, sent], dtype=torch.float64, device="cpu" if via_cpu else torch.device("cuda", dev))
        dist.all_reduce(tot)
        evs, sent = float(tot[0]), float(tot[1])
    xms_max = allmax(xms) if xms is not None else None
    if rank != 0:
        return None
    ticks = max(1, st["ticks"])
    sweep_ms = st["ms_sweep"] / ticks
    ops_t = ops / K
    ev0_t = st["events"] / ticks
    rec_t = st["grid_records"] / ticks
    b_sweep = 32.0 * rec_t + 4.0 * st["grid_cells"] / ticks + 4.0 * ops_t + 16.0 * ev0_t
    ach = b_sweep / (sweep_ms * 1e-3) / 1e9 if sweep_ms > 0 else 0.0
    from goworld_amd import _lib
    lib_v, stamp = lib_stamp(_lib.load())
    t_bytes, t_note = pmc_traffic(args.workload, n, stamp) if world == 1 else (None, "PMC passes run at one rank")
    return {
        "metric": METRIC,
        "value": n * K / elapsed,
        "unit": "entity-updates/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": DATA,
        "config": {
            "workload": (f"config 4: one open world of {n} entities ({args.per_gpu} per GPU), L={L:.0f}, D={args.dist}, "
                         f"X-strips over {world} GPU(s), halo {lay.halo:.1f} exchanged with the neighbours each tick"
                         if skew is None else
                         f"config 5 in strips: one open world of {n} entities ({args.per_gpu} per GPU), L={L:.0f}, "
                         f"D={args.dist}, 10% in {skew[0]} Gaussian hotspots (sigma {skew[1]:.0f}), X-strips at the "
                         f"x-quantiles over {world} GPU(s), halo {lay.halo:.1f}"),
            "entities_total": n, "world_L": L, "aoi_dist": args.dist, "seed": hex(seed),
            "strip_edges": lay.edges,
            "parallelism": (f"{world} X-strips, halo exchange " +
                            ("over torch.distributed (gloo via host)" if via_cpu else
                             "by gwaoi_strip_exchange (RCCL p2p over xGMI, on the strip's stream)"))
                           if world > 1 else "1 GPU (one strip)",
        },
        "p50_tick_ms": percentile(lat, 50) * 1e3,
        "p99_tick_ms": percentile(lat, 99) * 1e3,
        "events_per_tick": evs / K,
        "halo_records_per_tick": sent / K,
        "exchange_ms": xms_max,
        "exchange_note": None if xms_max is None else
        f"gwaoi_strip_exchange device time per tick (hipEvents on the strip's stream around the RCCL group, the "
        f"wait for the neighbours included), mean over {S} instrumented ticks, max over ranks",
        "rank0_ops_per_tick": ops / K,
        "stage_ms_rank0": {k: st[k] / ticks for k in ("ms_apply", "ms_grid", "ms_sweep", "ms_order", "ms_total")},
        "roofline": {
            "bound": "hbm", "kernel": "k_sweep (rank 0's strip)", "achieved": ach, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "traffic": t_bytes / (sweep_ms * 1e-3) / 1e9 if t_bytes and sweep_ms > 0 else None,
            "traffic_bytes_per_launch": t_bytes, "traffic_note": t_note, "algorithmic_bytes_per_launch": b_sweep,
            "avg_launch_ms": sweep_ms, "grid_records_per_tick": rec_t, "movers_per_tick": ops_t,
            "timing": "hipEvents around the sweep launch (gwaoi_get_stats)",
            "halo_bytes_per_tick": 16.0 * sent / K,
        },
        "lib": lib_v,
        "cpu_baseline": None,
    }


def strips_submeasurement(args, rank, world, dev, sync_all, allmax, backend):
    """The config-4 strips line of this world size, condensed (run by every rank: the exchange is
    collective). Under --dry-run (CPU rehearsal of the plumbing) only the rendezvous and its shape."""
    import copy
    sa = copy.copy(args)
    sa.workload, sa.steps, sa.warmup = "strips", args.strips_steps, min(args.warmup, 5)
    sa.stage_ticks = min(args.stage_ticks, 20)
    if args.dry_run:
        sync_all()
        return {"dry_run": True, "workload": "strips", "n_gpus": world, "steps": sa.steps,
                "elapsed": allmax(0.001 * (rank + 1))} if rank == 0 else (allmax(0.001 * (rank + 1)) and None)
    r = run_strips(sa, rank, world, dev, sync_all, allmax, via_cpu=(backend == "gloo"))
    if rank != 0:
        return None
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "scaling", "p50_tick_ms",
            "p99_tick_ms", "events_per_tick", "halo_records_per_tick", "exchange_ms", "exchange_note",
            "stage_ms_rank0", "config", "roofline")
    return {k: r.get(k) for k in keep}


def arm_deadline(seconds, rank, result):
    """Timer for a sub-measurement: when it fires, rank 0 prints `result` (the measured line) with the
    sub-measurement marked as timed out, and every rank exits with status 0."""
    import threading

    def fire():
        log(f"[rank {rank}] strips sub-measurement still running after {seconds:.0f}s: abandoned")
        if rank == 0:
            result["strips"] = {"error": f"did not finish within {seconds:.0f}s (abandoned; the headline line "
                                         "above it was measured before it started)"}
            print(json.dumps(result), file=_stdout_for_json(), flush=True)
        os._exit(0)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def arm_watchdog(seconds, rank):
    """A daemon timer that ends this rank with status 3 after `seconds` (a hung collective or kernel then
    fails the launcher instead of holding the GPUs). os._exit from the timer thread: no exec, no
    cleanup that could itself block on the device."""
    import threading

    def fire():
        log(f"[rank {rank}] watchdog: still running after {seconds:.0f}s, exiting with status 3")
        os._exit(3)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def self_launch_command(argv, env, gpus, port):
    """The child command that starts `gpus` ranks of this script, or None when no launch is needed.

    `bench.py --gpus N` (N > 1) started WITHOUT a launcher (no WORLD_SIZE in the environment) starts
    `python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>` as a CHILD process and
    relays rank 0's JSON line. The decision is taken before anything touches the GPU: the parent never
    initialises HIP (no torch.cuda call, no libgwaoi load), so it never has to exec over a live device."""
    if gpus <= 1 or "WORLD_SIZE" in env:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(cmd):
    """Run the launcher as a child; relay the JSON line(s) rank 0 prints; exit with the child's status."""
    import subprocess
    log("launching " + " ".join(cmd[1:5]) + " ... (one rank per GPU)")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    for line in p.stdout:  # rank 0 prints exactly one JSON line; anything else is relayed to stderr
        if line.lstrip().startswith("{"):
            print(line.rstrip("\n"), file=_stdout_for_json(), flush=True)
        else:
            log(line.rstrip("\n"))
    rc = p.wait()
    if rc != 0:
        log(f"launcher exited with status {rc}")
    return rc


_JSON_OUT = None


def _stdout_for_json():
    """The bench's stdout carries exactly one JSON line. Native libraries print to file descriptor 1
    (RCCL's version banner on communicator init, for one), so fd 1 is pointed at stderr and the JSON line
    goes to a duplicate of the original stdout."""
    global _JSON_OUT
    if _JSON_OUT is None:
        sys.stdout.flush()
        fd = os.dup(1)
        os.dup2(2, 1)
        _JSON_OUT = os.fdopen(fd, "w")
    return _JSON_OUT


def main():
    _stdout_for_json()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=["config2", "config3", "skew", "skew50", "strips", "strips_skew", "gametick"], default="config2")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--L", type=float, default=35000.0)
    ap.add_argument("--dist", type=float, default=100.0)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0002)
    ap.add_argument("--spaces", type=int, default=512, help="config3: Spaces per GPU")
    ap.add_argument("--per-gpu", type=int, default=2_000_000, help="strips: entities per GPU")
    ap.add_argument("--seed-strips", type=lambda s: int(s, 0), default=0x5EED0004)
    ap.add_argument("--gates", type=int, default=8, help="gametick: gates (dense indices)")
    ap.add_argument("--client-frac", type=float, default=0.25, help="gametick: fraction of entities with a client")
    ap.add_argument("--latency-ticks", type=int, default=200, help="extra ticks with events delivered to host")
    ap.add_argument("--p99-ticks", type=int, default=1000,
                    help="device-resident ticks after the timed region for p50/p99 (SURVEY 8(d): >= 1,000)")
    ap.add_argument("--small-reps", type=int, default=20,
                    help="config 2/3: repetitions of the small-pass leg (1-op Leave, 1-op Enter, 1k-op Moved "
                         "passes into the full manager, small passes on and off); 0 skips it")
    ap.add_argument("--replay-ticks", type=int, default=20,
                    help="host-staged ticks whose events are also replayed into the hash-set sink (replay_ms)")
    ap.add_argument("--host-staged-ticks", type=int, default=1000,
                    help="extra ticks staged from host arrays (gwaoi_stage_moves), events to host, replayed")
    ap.add_argument("--no-replay", dest="replay", action="store_false",
                    help="skip the C replay of events into per-entity hash sets")
    ap.add_argument("--pin-mode", choices=["async", "sync"], default="async",
                    help="host-staged headline ticks: gwaoi_stage_moves_pinned_async (ABI 2.1) or the sync call")
    ap.add_argument("--chunked-ticks", type=int, default=300,
                    help="ticks of the chunked-arrival leg (p99_flush_ms_chunked); 0 = off")
    ap.add_argument("--chunks", type=int, default=16, help="parts of the chunked-arrival leg's batch")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cells-per-dist", type=float, default=None)
    ap.add_argument("--dists", default=None, help="skew workloads: comma list of per-Space D (A/B)")
    ap.add_argument("--cell-side", type=float, default=None, help="absolute cell side for every Space (A/B)")
    ap.add_argument("--sweep-lds", type=int, default=1, help="0: global-memory sweep path (A/B)")
    ap.add_argument("--fanout", type=int, default=0,
                    help="gametick: 0 = direct fan-out when gates <= 8 (default), 1 = pair list + gate partition (A/B)")
    ap.add_argument("--band", type=int, default=1,
                    help="A/B: the band walk of the global-memory movers (1 on, 0 off: their whole rings)")
    ap.add_argument("--stage-ticks", type=int, default=200,
                    help="ticks run with per-stage hipEvents after the timed region (stage_ms, roofline)")
    ap.add_argument("--counting-build", action="store_true",
                    help="grid built by the counting tile build every pass, not the one-pass build (A/B)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch + rendezvous + barrier only, no GPU work (CPU test of the multi-rank plumbing)")
    ap.add_argument("--stamps", default=None, help="diagnostic GW_STAMPS build: dump the last sweep's per-block "
                                                   "phase timestamps to this .npy file")
    ap.add_argument("--strips-steps", type=int, default=100,
                    help="N > 1 (config 2): ticks of the config-4 X-strip sub-measurement (RCCL halo exchange over "
                         "xGMI) appended to the line as \"strips\" (0: none)")
    ap.add_argument("--watchdog", type=float, default=None,
                    help="seconds after which a rank still running exits with status 3 (a hung collective ends the "
                         "job instead of holding the GPUs; default 900 + 2 ms per step)")
    args = ap.parse_args()

    # N > 1 without an external launcher: start the ranks as a child before any GPU call
    cmd = self_launch_command(sys.argv[1:], os.environ, args.gpus, _free_port() if args.gpus > 1 else 0)
    if cmd is not None:
        sys.exit(_self_launch(cmd))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    arm_watchdog(args.watchdog if args.watchdog is not None else 900.0 + 0.002 * (args.steps + args.strips_steps),
                 rank)
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")

    import torch  # first: one HIP runtime per process (see goworld_amd/_lib.py)
    import torch.distributed as dist
    have_cuda = torch.cuda.is_available()
    # one rank per GPU; more ranks than GPUs only for functional runs with gloo (ranks share a GPU)
    ndev = torch.cuda.device_count() if have_cuda else 0
    dev = local % ndev if ndev else local
    backend = None
    if world > 1:
        backend = os.environ.get("GWAOI_DIST_BACKEND", "nccl" if have_cuda else "gloo")
        if have_cuda:
            torch.cuda.set_device(dev)
        dist.init_process_group(backend=backend)
    elif have_cuda:
        torch.cuda.set_device(dev)

    from goworld_amd import _lib
    L_ = None if args.dry_run else _lib.load()

    def sync_all():
        if not args.dry_run:
            _lib.check(L_.gwaoi_dev_sync(dev))
        if have_cuda:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def allmax(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    if args.dry_run:
        sync_all()
        result = {"dry_run": True, "n_gpus": world, "devices": ndev, "backend": backend,
                  "elapsed": allmax(0.001 * (rank + 1)), "workload": args.workload}
    elif args.workload in ("strips", "strips_skew"):
        result = run_strips(args, rank, world, dev, sync_all, allmax, via_cpu=(backend == "gloo"))
    elif args.workload == "gametick":
        result = run_gametick(args, rank, world, dev, sync_all, allmax)
    else:
        result = run_spaces(args, rank, world, dev, sync_all, allmax)
    # N > 1: the config-4 X-strip world (2M per GPU, halo exchange by RCCL p2p over xGMI inside libgwaoi)
    # measured after the headline line and appended to it; `value` stays the headline workload's
    if world > 1 and args.workload == "config2" and args.strips_steps > 0:
        # its own deadline: the headline line is already measured, so a strips run that does not finish
        # (a hung RCCL peer) is reported in it, and every rank ends cleanly, instead of losing the line
        guard = arm_deadline(120.0 + 0.05 * args.strips_steps, rank, result)
        try:
            sub = strips_submeasurement(args, rank, world, dev, sync_all, allmax, backend)
        except Exception as e:  # a failed strips run is reported in the already-measured line, never loses it
            log(f"[rank {rank}] strips sub-measurement failed: {e!r}")
            if rank == 0:
                result["strips"] = {"error": f"failed on rank 0: {e!r} (the headline line above it was measured "
                                             "before it started)"}
                print(json.dumps(result), file=_stdout_for_json(), flush=True)
            # (the other ranks may wait in a collective of the strips run: their deadline ends them, status 0)
            os._exit(0)
        guard.cancel()
        if rank == 0:
            result["strips"] = sub

    # ---- CPU baseline (rank 0, N=1: config 2, and config 3 per Space) ----
    if rank == 0 and world == 1 and args.workload == "config2" and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(args.n, args.L, args.dist, args.seed, args.cpu_baseline_seconds)
        except Exception as e:  # reported, never fatal to the GPU line
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0 and world == 1 and args.workload == "config3" and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline_spaces(2000, 1600.0, 100.0, 0x5EED0003, args.spaces,
                                                         args.cpu_baseline_seconds)
        except Exception as e:  # reported, never fatal to the GPU line
            result["cpu_baseline"] = {"error": repr(e)}
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        if have_cuda and 0 < ndev < world:  # functional runs only: several ranks time-share one GPU
            result["ranks_share_devices"] = f"{world} ranks on {ndev} device(s)"
        print(json.dumps(result), file=_stdout_for_json(), flush=True)


if __name__ == "__main__":
    main()
