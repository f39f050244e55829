"""TEST INFRASTRUCTURE ONLY — oracle (iv): the events of SAMPLED movers of one all-moving tick, at any size.

Only tests/ may import this module; the product (goworld_amd, libgwaoi) never does.

The full-size checks of configs 4 and 5 (16M entities; 4 x 1M with hotspots, billions of relation
pairs) cannot run a stateful oracle over the whole world. Their ticks have a shape that makes the
events of one mover a closed-form function of two position snapshots: every earlier tick entered or
moved EVERY entity of the Space exactly once, in slot order, and so does this one. Then, restating
SURVEY.md §8a-R (the relation is N(a, b) = in(L, F), L the member whose last op is later; go-aoi's
XZListAOIManager evaluates in() with float32 bounds rounded from L's coordinate, inclusive, the
manager-wide D: oracle/xzlist_aoi.c, Space.go:105,259):

  before the tick, the later actor of a and b is max(a, b) (both last acted in the previous tick, in
  slot order), so N(a, b) = in(p0[max(a, b)], p0[min(a, b)]);
  when m moves (op rank m), every o < m has already moved: N(m, o) = in(p1[o], p0[m]), and every
  o > m has not: N(m, o) = in(p0[o], p0[m]);
  after m's move, N(m, o) = in(p1[m], q) with q = p1[o] for o < m, p0[o] for o > m;
  m raises (m, o) when the two differ, ENTER when the pair is in afterwards.

Candidates come from a uniform point grid over both snapshots (numpy), then the predicate is
evaluated exactly in float32 (numpy float32 arithmetic: one IEEE binary32 add/sub per bound, as Go).
It shares no code with the C oracles or the product; tests/test_oracle.py checks it against oracle
(ii) event for event on small worlds. PARITY UNPINNED against go-aoi itself.
"""
from __future__ import annotations

import numpy as np

EV_ENTER = 0x80000000


class PointGrid:
    """Indices of points by a uniform grid of side c (for candidate search only)."""

    def __init__(self, x: np.ndarray, z: np.ndarray, c: float):
        self.c = float(c)
        self.x0 = float(min(x.min(), z.min())) - 1.0
        cx = np.floor((x.astype(np.float64) - self.x0) / self.c).astype(np.int64)
        cz = np.floor((z.astype(np.float64) - self.x0) / self.c).astype(np.int64)
        self.w = int(max(cx.max(), cz.max())) + 2
        key = cz * self.w + cx
        self.order = np.argsort(key, kind="stable")
        self.sk = key[self.order]

    def box(self, xlo: float, xhi: float, zlo: float, zhi: float) -> np.ndarray:
        c0 = int(np.floor((xlo - self.x0) / self.c)) - 1
        c1 = int(np.floor((xhi - self.x0) / self.c)) + 1
        r0 = int(np.floor((zlo - self.x0) / self.c)) - 1
        r1 = int(np.floor((zhi - self.x0) / self.c)) + 1
        out = []
        for r in range(max(r0, 0), r1 + 1):
            a = np.searchsorted(self.sk, r * self.w + max(c0, 0), "left")
            b = np.searchsorted(self.sk, r * self.w + c1, "right")
            if b > a:
                out.append(self.order[a:b])
        return np.concatenate(out) if out else np.zeros(0, np.int64)


def _in(cx, cz, px, pz, D):
    """in(c, p): p inside the box of an entity at c, bounds rounded to float32 from c (inclusive)."""
    lx, hx = cx - D, cx + D
    lz, hz = cz - D, cz + D
    return (px >= lx) & (px <= hx) & (pz >= lz) & (pz <= hz)


class AllMovingTick:
    """One Space's all-moving tick: positions before (x0, z0) and after (x1, z1), slots base..base+n-1."""

    def __init__(self, x0, z0, x1, z1, dist: float, base: int = 0):
        self.x0 = np.asarray(x0, np.float32)
        self.z0 = np.asarray(z0, np.float32)
        self.x1 = np.asarray(x1, np.float32)
        self.z1 = np.asarray(z1, np.float32)
        self.D = np.float32(dist)
        self.base = int(base)
        step = float(max(np.abs(self.x1 - self.x0).max(), np.abs(self.z1 - self.z0).max()))
        # any pair whose state can change has |o - m| <= D + step (+ rounding) in some snapshot pair
        self.reach = float(dist) + step + 1e-3 * (1.0 + float(dist))
        c = max(float(dist) / 2.0, 1.0)
        self.g0 = PointGrid(self.x0, self.z0, c)
        self.g1 = PointGrid(self.x1, self.z1, c)

    def events(self, m: int) -> np.ndarray:
        """Events of local mover m as (global mover, global other | ENTER), sorted by the other column."""
        D, r = self.D, self.reach
        xs = (float(self.x0[m]), float(self.x1[m]))
        zs = (float(self.z0[m]), float(self.z1[m]))
        lo_x, hi_x, lo_z, hi_z = min(xs) - r, max(xs) + r, min(zs) - r, max(zs) + r
        cand = np.unique(np.concatenate([self.g0.box(lo_x, hi_x, lo_z, hi_z), self.g1.box(lo_x, hi_x, lo_z, hi_z)]))
        o = cand[cand != m]
        early = o < m
        px = np.where(early, self.x1[o], self.x0[o])  # o at m's op: moved already, or not yet
        pz = np.where(early, self.z1[o], self.z0[o])
        before = _in(px, pz, self.x0[m], self.z0[m], D)  # box of the later actor (o), test m's start
        after = _in(self.x1[m], self.z1[m], px, pz, D)   # m's new box, test o at m's op
        hit = before != after
        oth = (o[hit] + self.base).astype(np.uint32) | np.where(after[hit], np.uint32(EV_ENTER), np.uint32(0))
        ev = np.stack([np.full(len(oth), m + self.base, np.uint32), oth], axis=1)
        return ev[np.argsort(ev[:, 1], kind="stable")]

    def sample(self, movers) -> np.ndarray:
        evs = [self.events(int(m)) for m in movers]
        return np.concatenate(evs) if evs else np.zeros((0, 2), np.uint32)


def pick(events: np.ndarray, movers_global) -> np.ndarray:
    """The rows of an event array whose mover is in movers_global, sorted by (mover, other)."""
    sel = events[np.isin(events[:, 0], np.asarray(movers_global, np.uint32))]
    return sel[np.lexsort((sel[:, 1], sel[:, 0]))] if len(sel) else sel.reshape(0, 2)
