"""TEST INFRASTRUCTURE ONLY — oracle (iii): brute-force numpy restatement of SURVEY.md §8a-R.

O(N) per op with a dense boolean relation matrix; for small cases only (N <= a few thousand). It
shares nothing with the C oracles or the product. Float semantics: numpy float32 scalar/array ops
are single IEEE binary32 operations, as Go's float32 arithmetic in go-aoi's Mark walks
(go-aoi v0.2.0 XZListAOIManager, Gopkg.lock:155-159 [UPSTREAM-RECALLED]).
PARITY UNPINNED (see oracle/xzlist_aoi.c header).
"""
from __future__ import annotations

import numpy as np

EV_ENTER = 0x80000000


class SemanticModel:
    def __init__(self, dist: float, cap: int):
        self.D = np.float32(dist)
        self.cap = cap
        self.x = np.zeros(cap, np.float32)
        self.z = np.zeros(cap, np.float32)
        self.present = np.zeros(cap, bool)
        self.rel = np.zeros((cap, cap), bool)

    def _inside(self, m: int) -> np.ndarray:
        """in(m, o) for every o: o inside m's box, bounds rounded to float32 from m's coordinate."""
        lx = self.x[m] - self.D
        hx = self.x[m] + self.D
        lz = self.z[m] - self.D
        hz = self.z[m] + self.D
        r = (self.x >= lx) & (self.x <= hx) & (self.z >= lz) & (self.z <= hz) & self.present
        r[m] = False
        return r

    def _events(self, m, before, after):
        out = []
        for o in np.nonzero(before & ~after)[0]:
            out.append((m, int(o)))
        for o in np.nonzero(after & ~before)[0]:
            out.append((m, int(o) | EV_ENTER))
        return out

    def enter(self, m, x, z):
        assert not self.present[m]
        self.x[m], self.z[m] = np.float32(x), np.float32(z)
        self.present[m] = True
        after = self._inside(m)
        ev = self._events(m, np.zeros(self.cap, bool), after)
        self.rel[m, :] = after
        self.rel[:, m] = after
        return ev

    def leave(self, m):
        assert self.present[m]
        before = self.rel[m].copy()
        ev = self._events(m, before, np.zeros(self.cap, bool))
        self.rel[m, :] = False
        self.rel[:, m] = False
        self.present[m] = False
        return ev

    def moved(self, m, x, z):
        assert self.present[m]
        before = self.rel[m].copy()
        self.x[m], self.z[m] = np.float32(x), np.float32(z)
        after = self._inside(m)
        ev = self._events(m, before, after)
        self.rel[m, :] = after
        self.rel[:, m] = after
        return ev

    def relation(self):
        rp = np.zeros(self.cap + 1, np.uint32)
        cols = []
        for s in range(self.cap):
            rp[s] = len(cols)
            if self.present[s]:
                cols.extend(np.nonzero(self.rel[s])[0].tolist())
        rp[self.cap] = len(cols)
        return rp, np.asarray(cols, np.uint32)
