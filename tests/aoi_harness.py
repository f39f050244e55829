"""Shared test harness: op scripts, the oracle driver and the GPU driver.

An op script is a list of ticks; a tick is a list of ops (kind, slot, x, z) with kind
MOVE=0 (go-aoi Moved), ENTER=1 (Enter), LEAVE=2 (Leave) — the three AOIManager calls of
/root/reference/engine/entity/Space.go:211/221, 243, 259.

Canonical event order (include/gwaoi.h): ops in staging order; inside one op LEAVE before ENTER and
other slot ascending. Sub-passes forced by re-staging a slot keep that order, so the oracle side is
simply "apply op by op, sort each op's events by other|kind".
"""
from __future__ import annotations

import numpy as np

MOVE, ENTER, LEAVE = 0, 1, 2
EV_ENTER = 0x80000000


def f32(v) -> float:
    return float(np.float32(v))


def nextafter32(v, direction) -> float:
    return float(np.nextafter(np.float32(v), np.float32(direction)))


# ------------------------------------------------------------------------------------------------
# drivers

def oracle_tick(orc, ops) -> np.ndarray:
    """Apply one tick's ops to an oracle op by op; canonical (n,2) uint32 events."""
    slots = [o[1] for o in ops]
    if ops and all(o[0] == MOVE for o in ops) and len(set(slots)) == len(slots):
        s = np.asarray(slots, np.uint32)
        orc.moved_batch(s, np.asarray([o[2] for o in ops], np.float32), np.asarray([o[3] for o in ops], np.float32))
        ev = orc.take_events()
        if len(ev) == 0:
            return ev
        rank = np.zeros(orc.cap, np.int64)
        rank[s] = np.arange(len(s))
        return ev[np.lexsort((ev[:, 1], rank[ev[:, 0]]))]
    out = []
    for kind, slot, x, z in ops:
        if kind == ENTER:
            orc.enter(slot, x, z)
        elif kind == LEAVE:
            orc.leave(slot)
        else:
            orc.moved(slot, x, z)
        ev = orc.take_events()
        if len(ev):
            out.append(ev[np.argsort(ev[:, 1], kind="stable")])
    if not out:
        return np.zeros((0, 2), np.uint32)
    return np.concatenate(out).astype(np.uint32)


def semantic_tick(model, ops) -> np.ndarray:
    out = []
    for kind, slot, x, z in ops:
        if kind == ENTER:
            ev = model.enter(slot, x, z)
        elif kind == LEAVE:
            ev = model.leave(slot)
        else:
            ev = model.moved(slot, x, z)
        if ev:
            a = np.asarray(ev, np.uint32)
            out.append(a[np.argsort(a[:, 1], kind="stable")])
    return np.concatenate(out) if out else np.zeros((0, 2), np.uint32)


def gpu_tick(eng, ops) -> np.ndarray:
    """Stage one tick's ops on an Engine and tick it."""
    slots = [o[1] for o in ops]
    if ops and all(o[0] == ENTER for o in ops) and len(set(slots)) == len(slots):
        eng.stage_enters(np.asarray(slots, np.uint32), np.asarray([o[2] for o in ops], np.float32),
                         np.asarray([o[3] for o in ops], np.float32))
    elif ops and all(o[0] == MOVE for o in ops) and len(set(slots)) == len(slots):
        eng.stage_moves(np.asarray(slots, np.uint32), np.asarray([o[2] for o in ops], np.float32),
                        np.asarray([o[3] for o in ops], np.float32))
    else:
        for kind, slot, x, z in ops:
            if kind == ENTER:
                eng.enter(slot, x, z)
            elif kind == LEAVE:
                eng.leave(slot)
            else:
                eng.moved(slot, x, z)
    return eng.tick()


def gpu_tick_pinned(eng, ops, mode="sync", chunk=0) -> np.ndarray:
    """The cgo wrapper's batching: Moved calls are written into the manager's pinned
    staging arrays and pushed with ONE gwaoi_stage_moves_pinned before the next Enter/Leave and at the
    flush; a slot moved twice stays in the batch (the device splits it into sub-passes). mode "async":
    gwaoi_stage_moves_pinned_async (the verdict read by the pass); chunk > 0: every `chunk` Moved calls
    are pushed early with gwaoi_stage_moves_pinned_partial (ABI 2.1)."""
    ps, px, pz = eng.stage_buffers()
    k = 0

    def push():
        nonlocal k
        if k:
            (eng.stage_moves_pinned_async if mode == "async" else eng.stage_moves_pinned)(k)
            k = 0

    for kind, slot, x, z in ops:
        if kind == MOVE:
            ps[k], px[k], pz[k] = slot, x, z
            k += 1
            if k == len(ps):
                push()
            elif chunk and k % chunk == 0:
                eng.stage_moves_pinned_partial(k)
            continue
        push()
        if kind == ENTER:
            eng.enter(slot, x, z)
        else:
            eng.leave(slot)
    push()
    return eng.tick()


def fmt_diff(a: np.ndarray, b: np.ndarray, limit=10) -> str:
    sa = set(map(tuple, a.tolist()))
    sb = set(map(tuple, b.tolist()))
    only_a = sorted(sa - sb)[:limit]
    only_b = sorted(sb - sa)[:limit]
    return f"|a|={len(a)} |b|={len(b)} only_a={only_a} only_b={only_b}"


# ------------------------------------------------------------------------------------------------
# op scripts

def case_origin_monsters():
    """MySpace.OnSpaceCreated (examples/test_game/MySpace.go:27-34): EnableAOI(100), 10 Monsters at
    Vector3{}; then an Avatar enters, and DoTestAOI (Avatar.go:267-280) enters an AOITester at the
    avatar's position and destroys it one tick later."""
    ticks = [[(ENTER, i, 0.0, 0.0) for i in range(10)],
             [(ENTER, 10, 37.5, -12.25)],
             [(ENTER, 11, 37.5, -12.25)],
             [(LEAVE, 11, 0.0, 0.0)],
             [(MOVE, 10, 250.0, 0.0)],
             [(MOVE, 10, 100.0, 0.0), (MOVE, 3, 0.0, 0.0)]]
    return dict(name="origin_monsters", dist=100.0, cap=16, ticks=ticks)


def case_boundaries(dist=100.0):
    """Entities placed exactly on and one ulp around the float32 box bounds fl(c±D), at several
    magnitudes (including where ulp(c) >> 0 and the bounds round), negative coordinates, ties; then
    moves that step the anchors by one ulp so membership flips, from both perspectives."""
    D = np.float32(dist)
    anchors = [0.0, 0.3, -0.3, 1e-3, 12345.678, -65536.5, 1048576.0 + 0.0625, 3.0e7, -2.5e6]
    ticks = []
    slot = 0
    enters = []
    groups = []
    for c in anchors:
        c = np.float32(c)
        hi = np.float32(c + D)
        lo = np.float32(c - D)
        xs = [c, hi, lo, np.nextafter(hi, np.float32(np.inf)), np.nextafter(hi, np.float32(-np.inf)),
              np.nextafter(lo, np.float32(-np.inf)), np.nextafter(lo, np.float32(np.inf))]
        g = []
        for i, x in enumerate(xs):
            zs = [c, xs[(i + 3) % len(xs)]]
            for zz in zs:
                enters.append((ENTER, slot, float(x), float(zz)))
                g.append(slot)
                slot += 1
        groups.append((c, g))
    ticks.append(enters)
    # tick 2: every anchor entity steps one ulp up, in ascending slot order
    rng = np.random.default_rng(7)
    pos = {op[1]: (np.float32(op[2]), np.float32(op[3])) for op in enters}
    for t in range(4):
        ops = []
        order = rng.permutation(slot)
        for s in order[: slot // 2]:
            x, z = pos[int(s)]
            d = rng.integers(0, 4)
            if d == 0:
                x = np.nextafter(x, np.float32(np.inf))
            elif d == 1:
                x = np.nextafter(x, np.float32(-np.inf))
            elif d == 2:
                z = np.nextafter(z, np.float32(np.inf))
            else:
                z = np.nextafter(z, np.float32(-np.inf))
            pos[int(s)] = (x, z)
            ops.append((MOVE, int(s), float(x), float(z)))
        ticks.append(ops)
    return dict(name="boundaries", dist=float(D), cap=slot, ticks=ticks)


def case_random_ops(seed=1, n=200, nticks=12, ops_per_tick=150, world=400.0, dist=50.0, snap=True,
                    dup=True):
    """Random Enter/Leave/Moved mixes, partial movers, teleports, repeated staging of one slot in a
    tick (forces sub-passes), positions snapped to a coarse lattice (ties and exact-D offsets)."""
    rng = np.random.default_rng(seed)
    present = np.zeros(n, bool)
    pos = np.zeros((n, 2), np.float32)
    ticks = []
    for t in range(nticks):
        ops = []
        for _ in range(ops_per_tick):
            s = int(rng.integers(n))
            if not dup and any(o[1] == s for o in ops):
                continue
            r = rng.random()
            if snap and r < 0.3:
                x, z = (rng.integers(-8, 9, 2) * dist / 2).astype(np.float32)
            elif r < 0.5 and present[s]:
                x, z = pos[s] + rng.uniform(-3, 3, 2).astype(np.float32)
            else:
                x, z = rng.uniform(-world, world, 2).astype(np.float32)
            if not present[s]:
                ops.append((ENTER, s, float(x), float(z)))
                present[s] = True
                pos[s] = (x, z)
            elif rng.random() < 0.1:
                ops.append((LEAVE, s, 0.0, 0.0))
                present[s] = False
            else:
                ops.append((MOVE, s, float(x), float(z)))
                pos[s] = (x, z)
        ticks.append(ops)
    return dict(name=f"random_ops_{seed}", dist=dist, cap=n, ticks=ticks)


def case_walk(seed, n, L, nticks, dist=100.0, step=1.0, workload=None):
    """The seeded random walk of SURVEY.md §8(d): tick 0 = n Enters (uniform in [0,L)^2, slot
    order), ticks 1.. = every slot moves once, in ascending slot order. `workload` is
    oracle.pyoracle (its host copy of include/gwaoi_workload.h)."""
    x, z = workload.workload_init(seed, n, L)
    ticks = [[(ENTER, i, float(x[i]), float(z[i])) for i in range(n)]]
    for t in range(1, nticks):
        workload.workload_step(seed, t, x, z, L, step)
        ticks.append([(MOVE, i, float(x[i]), float(z[i])) for i in range(n)])
    return dict(name=f"walk_{n}_{seed:x}", dist=dist, cap=n, ticks=ticks, bounds=(0.0, 0.0, L, L))


def case_denormal():
    """Tiny AOI distance with denormal coordinates: bounds fl(c±D) land in the subnormal range.
    Go keeps subnormals; the GPU build must not flush them."""
    D = 2.0e-38
    vals = [0.0, 1e-45, -1e-45, 3e-39, -3e-39, 2e-38, -2e-38, 2.5e-38, 1.9e-38]
    ticks = [[(ENTER, i, float(np.float32(v)), float(np.float32(vals[(i * 5) % len(vals)])))
              for i, v in enumerate(vals)]]
    ticks.append([(MOVE, i, float(np.float32(vals[(i + 1) % len(vals)])), 0.0) for i in range(len(vals))])
    return dict(name="denormal", dist=D, cap=len(vals), ticks=ticks, bounds=(-1e-37, -1e-37, 1e-37, 1e-37))
