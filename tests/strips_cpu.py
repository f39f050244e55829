"""TEST INFRASTRUCTURE: a CPU restatement of one strip of goworld_amd/strips.py (include/gwaoi_strips.h)
with oracle (i) as the region's manager. It lets the multi-process protocol (the product's
exchange_dist over gloo, world_size > 1) run on CPU, and it is the checker the GPU kernels of each
step are compared against.
"""
from __future__ import annotations

import numpy as np
import torch

P, O, E = 1, 2, 4
MOVE, ENTER, LEAVE, SILENT = 0, 1, 2, 0x80
f32 = np.float32


class CPUStripNode:
    def __init__(self, layout, rank, n, po, seed=0x5EED0004):
        self.layout, self.rank, self.n, self.seed, self.po = layout, rank, n, seed, po
        self.g = layout.geom(rank, n)
        self.flags = np.zeros(n, np.uint8)
        self.sx, self.sz, self.ex, self.ez = (np.zeros(n, f32) for _ in range(4))
        self.orc = po.XZListOracle(layout.dist, n)
        # the whole world's seeded walk (only the owned entries are ever read)
        self.wx, self.wz = po.workload_init(seed, n, layout.L)

    def _in(self, x, lo, hi):
        return (x >= f32(lo)) & (x < f32(hi))

    def start(self):
        g = self.g
        x, z = self.wx, self.wz
        reg = self._in(x, g.ra, g.rb)
        self.flags[reg] |= E
        self.ex[reg], self.ez[reg] = x[reg], z[reg]
        self.flags[self._in(x, g.xa, g.xb)] |= O
        return self.emit()

    def prepare(self, t, step=1.0):
        g = self.g
        self.po.workload_step(self.seed, t, self.wx, self.wz, self.layout.L, step)
        own = (self.flags & O) != 0
        assert np.all(np.abs(self.wx[own] - self.sx[own]) <= f32(g.max_step))
        self.ex[own], self.ez[own] = self.wx[own], self.wz[own]
        self.flags[own] |= E
        sel = own
        lt = sel & ((self.sx < f32(g.left_hi)) | (self.ex < f32(g.left_hi))) if g.has_left else np.zeros(self.n, bool)
        rt = sel & ((self.sx >= f32(g.right_lo)) | (self.ex >= f32(g.right_lo))) if g.has_right else np.zeros(self.n, bool)
        return self._recs(np.nonzero(lt)[0]), self._recs(np.nonzero(rt)[0])

    def _recs(self, ids):
        r = np.zeros((len(ids), 4), np.uint32)
        r[:, 0] = ids
        r[:, 1] = self.ex[ids].view(np.uint32)
        r[:, 2] = self.ez[ids].view(np.uint32)
        return torch.from_numpy(r.view(np.int32))

    def absorb(self, left_in, right_in):
        for recs in (left_in, right_in):
            if recs is not None and recs.numel():
                r = recs.cpu().numpy().view(np.uint32)
                ids = r[:, 0]
                self.ex[ids] = r[:, 1].view(f32)
                self.ez[ids] = r[:, 2].view(f32)
                self.flags[ids] |= E

    def finish(self, left_in, right_in):
        self.absorb(left_in, right_in)
        return self.emit()

    def ops(self):
        """The id-ordered op list of this tick (ids, kinds) — what gwaoi_strip_emit produces."""
        f = self.flags
        ids = np.nonzero((f & (P | E)) != 0)[0]
        p, e = (f[ids] & P) != 0, (f[ids] & E) != 0
        kinds = np.where(p & e, MOVE, np.where(p, LEAVE, ENTER)).astype(np.uint8)
        kinds |= np.where((f[ids] & O) != 0, 0, SILENT).astype(np.uint8)
        return ids, kinds

    def emit(self):
        g = self.g
        ids, kinds = self.ops()
        loud = []
        for i, k in zip(ids.tolist(), kinds.tolist()):
            kk = k & 3
            if kk == MOVE:
                self.orc.moved(i, float(self.ex[i]), float(self.ez[i]))
            elif kk == ENTER:
                self.orc.enter(i, float(self.ex[i]), float(self.ez[i]))
            else:
                self.orc.leave(i)
            if not k & SILENT:
                loud.append(i)
        ev = self.orc.take_events()
        ev = ev[np.isin(ev[:, 0], np.asarray(loud, np.uint32))] if len(ev) else ev
        # state advance
        e = (self.flags & E) != 0
        self.sx[e], self.sz[e] = self.ex[e], self.ez[e]
        nf = np.zeros(self.n, np.uint8)
        nf[e] = P
        nf[e & (self.ex >= f32(g.xa)) & (self.ex < f32(g.xb))] |= O
        self.flags = nf
        return ev[np.lexsort((ev[:, 1], ev[:, 0]))] if len(ev) else ev.reshape(0, 2)


def global_events(po, n, L, dist, seed, nticks, step=1.0):
    """One oracle-(i) manager over the whole world: tick 0 = Enter in id order, then every id moves
    once per tick in id order. Events per tick sorted by (mover, other|kind)."""
    x, z = po.workload_init(seed, n, L)
    orc = po.XZListOracle(dist, n)
    out = []
    for i in range(n):
        orc.enter(i, float(x[i]), float(z[i]))
    ev = orc.take_events()
    out.append(ev[np.lexsort((ev[:, 1], ev[:, 0]))])
    ids = np.arange(n, dtype=np.uint32)
    for t in range(1, nticks):
        po.workload_step(seed, t, x, z, L, step)
        orc.moved_batch(ids, x, z)
        ev = orc.take_events()
        out.append(ev[np.lexsort((ev[:, 1], ev[:, 0]))] if len(ev) else ev.reshape(0, 2))
    return out


def merge_sorted(evs):
    evs = [e for e in evs if len(e)]
    if not evs:
        return np.zeros((0, 2), np.uint32)
    a = np.concatenate(evs)
    return a[np.lexsort((a[:, 1], a[:, 0]))]
