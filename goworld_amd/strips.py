"""One Space partitioned into X-strips over several GPUs — host side of include/gwaoi_strips.h.

SURVEY.md §8(e), config 4: a huge open world split into vertical strips, one per GPU (one process
per GPU), halo copies of the entities near each strip edge exchanged every tick with the two
neighbouring GPUs (torch.distributed point-to-point: RCCL over xGMI with the "nccl" backend, gloo in
the CPU tests). The protocol and why it reproduces one manager's events exactly are in
include/gwaoi_strips.h; in short, GPU r applies the op of every entity of its region in global id
order, its owned entities loud and halo copies GWAOI_OP_SILENT, and reports the events of its owned
movers only.

torch is plumbing here (device buffers, the stream, the collectives); every per-entity step runs in
libgwaoi's HIP kernels. A node is driven in two halves per tick so that several nodes can share one
process (LoopbackExchange, the single-GPU tests) or run one per process (exchange_dist):
    left, right = node.prepare(t)        # owned end positions + the records the neighbours need
    left_in, right_in = <exchange>       # what the neighbours sent
    events = node.finish(left_in, right_in)
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import check
from .engine import Engine

f32 = np.float32
STRIP_ERR_SLOTS = 8  # GWAOI_STRIP_ERR_SLOTS (include/gwaoi_strips.h)
STRIP_ERR_NEWLIST = 16  # GWAOI_STRIP_ERR_NEWLIST (region state)


class StripLayout:
    """Strips over [0, L) in x: equal widths (config 4's uniform world), or explicit inner edges (e.g.
    x-quantiles of a skewed crowd, config 5: from_quantiles). The halo covers D + the largest per-tick
    step."""

    def __init__(self, world: int, L: float, dist: float, max_step: float, margin: Optional[float] = None,
                 edges: Optional[Sequence[float]] = None):
        self.world, self.L, self.dist, self.max_step = int(world), float(L), float(dist), float(max_step)
        # query boxes are widened by (|c| + D) * 2^-20 before they become cell ranges; the halo keeps a
        # margin far above that and above float rounding of the bounds
        if margin is None:
            margin = max(1.0, (self.L + self.dist) * 2.0 ** -16)
        self.halo = float(f32(self.dist + self.max_step + margin))
        self.uniform = edges is None  # equal widths (else: explicit edges, e.g. x-quantiles)
        if edges is None:
            edges = [rank * self.L / self.world for rank in range(1, self.world)]
        if len(edges) != self.world - 1:
            raise ValueError(f"{self.world} strips need {self.world - 1} inner edges, got {len(edges)}")
        self.edges = [float(f32(e)) for e in edges]
        lo = [0.0] + self.edges
        hi = self.edges + [self.L]
        for r in range(self.world):
            if self.world > 1 and hi[r] - lo[r] <= 2 * self.halo + self.max_step:
                raise ValueError(f"strip {r} of width {hi[r] - lo[r]} is too narrow for a halo of {self.halo}")

    @classmethod
    def from_quantiles(cls, world: int, x: np.ndarray, L: float, dist: float, max_step: float,
                       margin: Optional[float] = None) -> "StripLayout":
        """Inner edges at the x-quantiles of the entities (equal entity counts per strip, SURVEY.md §8(e)
        config 5), each strip kept wider than 2 halo + step (narrow quantile strips are merged into
        their neighbours' width by pushing the edge out)."""
        probe = cls(1, L, dist, max_step, margin)
        min_w = 2 * probe.halo + max_step + 1.0
        q = np.quantile(np.asarray(x, dtype=np.float64), [r / world for r in range(1, world)]) if world > 1 else []
        edges, prev = [], 0.0
        for r, e in enumerate(q):
            left = world - 1 - r  # strips still to place right of this edge
            e = min(max(float(e), prev + min_w), L - left * min_w)
            edges.append(e)
            prev = e
        return cls(world, L, dist, max_step, margin, edges=edges)

    def bounds(self, rank: int) -> Tuple[float, float]:
        xa = -math.inf if rank == 0 else self.edges[rank - 1]
        xb = math.inf if rank == self.world - 1 else self.edges[rank]
        return xa, xb

    def owner_of(self, x: np.ndarray) -> np.ndarray:
        """Strip index of each x (the same float32 comparisons as the kernels)."""
        edges = np.asarray([self.bounds(r)[0] for r in range(1, self.world)], dtype=f32)
        return np.searchsorted(edges, np.asarray(x, dtype=f32), side="right")

    def geom(self, rank: int, n: int) -> _lib.StripGeom:
        xa, xb = self.bounds(rank)
        H = f32(self.halo)
        g = _lib.StripGeom()
        g.n = n
        g.xa, g.xb = xa, xb
        g.ra, g.rb = float(f32(f32(xa) - H)), float(f32(f32(xb) + H))
        g.left_hi = float(f32(f32(xa) + H))   # the left neighbour's region ends at its xb + H = xa + H
        g.right_lo = float(f32(f32(xb) - H))  # the right neighbour's region starts at xb - H
        g.max_step = float(f32(self.max_step))
        g.has_left = 1 if rank > 0 else 0
        g.has_right = 1 if rank < self.world - 1 else 0
        return g


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


class StripNode:
    """The strip of GPU `rank`: per-id state, the region's gwaoi manager, the per-tick kernels."""

    def __init__(self, layout: StripLayout, rank: int, n: int, device: int = 0, seed: int = 0x5EED0004,
                 halo_cap: Optional[int] = None, skew: Optional[Tuple[int, float, int]] = None,
                 local_slots: bool = True, cap_l: Optional[int] = None, region_state: Optional[bool] = None,
                 cap_new: int = 65536, sort_chunk: int = 0, stream: Optional[torch.cuda.Stream] = None):
        """skew = (nhot, sigma, hot_every): the skewed-crowd placement of config 5 instead of uniform.
        local_slots: the manager sees local slots (gwaoi_strip_emit_local); False: slot = global id.
        region_state (local slots only, ABI 2.1, default on; GWAOI_STRIP_REGION=0 / 1 forces it): the strip's
        state in local-slot order and the per-tick kernels over the region (gwaoi_strip_region_*), not over the
        world's id range; cap_new: ids that may come into (and Leaves that may leave) the region per tick;
        sort_chunk: the LDS sort's chunk of those (0: 16384; tests use small chunks to cover the merge).
        stream: a (non-null) stream to run on, e.g. one shared by several strips of a single-GPU loopback run so
        that their kernels do not overlap and each strip's hipEvents time its own work; default: its own."""
        self.layout, self.rank, self.n, self.seed = layout, int(rank), int(n), int(seed)
        self.skew = skew
        self.g = layout.geom(rank, n)
        self.device = torch.device("cuda", device)
        self._L = _lib.load()
        dev = self.device
        u8, i32, fl = torch.uint8, torch.int32, torch.float32
        # the halo of one side holds ~ 2 H L density entities; keep room for several times that (a skewed
        # crowd can put a hotspot on an edge: more)
        cap = halo_cap or max(4096, int((32 if skew else 8) * layout.halo * layout.L * n / (layout.L * layout.L)) + 4096)
        self.cap = min(cap, n) if n else 1
        self.left = torch.zeros((self.cap, 4), dtype=i32, device=dev)
        self.right = torch.zeros((self.cap, 4), dtype=i32, device=dev)
        # the node's counters in one device block, read back by ONE copy per tick into one pinned block:
        # [0, 4) counts [left, right, n_ops, err], [4, 8) local-slot counters, [8, 16) region-state counters
        self.ctrs = torch.zeros(16, dtype=i32, device=dev)
        self.h_ctrs = torch.zeros(16, dtype=i32).pin_memory()
        self.counts, self.h_counts = self.ctrs[0:4], self.h_ctrs[0:4]  # h_counts: read after each tick, no extra sync
        self.left_in, self.right_in, self.counts_in = None, None, None  # RCCL receive buffers (tick_rccl)
        self.scratch = torch.zeros(int(self._L.gwaoi_strip_scratch_words(n)), dtype=i32, device=dev)
        # a stream of the node's own (never the null stream: the manager would take that as "its
        # own stream" and the strip kernels and the pipeline would no longer be ordered)
        self.stream = stream if stream is not None else torch.cuda.Stream(dev)
        torch.cuda.synchronize(dev)  # the buffers above were zeroed on the current stream
        lo = max(self.g.ra, 0.0)
        hi = min(self.g.rb, layout.L)
        # the region holds about its share of the world's entities (equal widths: by area; quantile
        # strips: an equal count)
        own_w = max(1e-9, min(self.g.xb, layout.L) - max(self.g.xa, 0.0))  # owned strip width
        share = n * (hi - lo) / layout.L if layout.uniform else n / layout.world * (hi - lo) / own_w
        # Local slots (include/gwaoi_strips.h): the manager indexes the region's entities by a slot of
        # its own, so its per-pass work follows the region's population, not the world's id range.
        # cap_l: room for crowds drifting in (1.25x the share + 8k), at most n; the manager's capacity, so
        # every pass's per-slot work (grid build) follows it (ABI 2.1: any count, the free ring rounded up to
        # a power of two; 2.0 rounded cap_l itself: a 2M region took 4M slots)
        want = min(n, int(share * 1.25) + 8192) if local_slots else n
        if cap_l is not None:  # explicit (tests: a region that overflows its slots)
            want = int(cap_l)
        self.cap_l = max(1, want)
        self.local = bool(local_slots)
        if region_state is None:
            env = os.environ.get("GWAOI_STRIP_REGION")
            region_state = env != "0" if env is not None else True
        self.R = None
        # state: per local slot (region state) or per global id; the op list: at most cap_l ops (region state)
        m = self.cap_l if (self.local and region_state) else n
        self.flags = torch.zeros(m, dtype=u8, device=dev)
        self.sx, self.sz, self.ex, self.ez = (torch.zeros(m, dtype=fl, device=dev) for _ in range(4))
        self.ids = torch.zeros(m, dtype=i32, device=dev)
        self.ox, self.oz = torch.zeros(m, dtype=fl, device=dev), torch.zeros(m, dtype=fl, device=dev)
        self.kinds = torch.zeros(m, dtype=u8, device=dev)
        if self.local:
            ring = 1 << max(0, (self.cap_l - 1).bit_length())
            self.g2l = torch.empty(n, dtype=i32, device=dev)
            self.l2g = torch.zeros(self.cap_l, dtype=i32, device=dev)
            self.fq = torch.empty(ring, dtype=i32, device=dev)
            self.pend = torch.empty(self.cap_l, dtype=i32, device=dev)
            self.lctr, self.h_lctr = self.ctrs[4:8], self.h_ctrs[4:8]
            torch.cuda.synchronize(dev)
            if region_state:
                cn = max(1, min(int(cap_new), 8 * (int(sort_chunk) or 16384)))
                self.rl = [torch.zeros(self.cap_l, dtype=i32, device=dev) for _ in range(2)]
                self.rs = [torch.zeros(self.cap_l, dtype=i32, device=dev) for _ in range(2)]
                self.nw = torch.zeros(2 * cn, dtype=i32, device=dev)
                self.lv = torch.zeros(cn, dtype=i32, device=dev)
                self.srt = torch.zeros(3 * cn, dtype=i32, device=dev)
                self.rctr, self.h_rctr = self.ctrs[8:16], self.h_ctrs[8:16]
                R = _lib.StripRegion()
                for f in ("flags", "sx", "sz", "ex", "ez", "g2l", "l2g", "fq", "pend", "lctr", "nw", "lv", "srt",
                          "scratch"):
                    setattr(R, f, getattr(self, f).data_ptr())
                R.rl[0], R.rl[1] = self.rl[0].data_ptr(), self.rl[1].data_ptr()
                R.rs[0], R.rs[1] = self.rs[0].data_ptr(), self.rs[1].data_ptr()
                R.ctr = self.rctr.data_ptr()
                R.n, R.cap_l, R.cap_new, R.chunk = n, self.cap_l, cn, int(sort_chunk)
                self.R = R
                torch.cuda.synchronize(dev)
                check(self._L.gwaoi_strip_region_init(ctypes.c_void_p(0), ctypes.byref(R)))
            else:
                check(self._L.gwaoi_strip_local_init(ctypes.c_void_p(0), n, self.cap_l, _ptr(self.g2l),
                                                     _ptr(self.fq), _ptr(self.lctr)))
            torch.cuda.synchronize(dev)
        self.eng = Engine(layout.dist, capacity=self.cap_l if self.local else n, device=device,
                          bounds=(lo, 0.0, hi, layout.L))
        self.eng.set_stream(self.stream.cuda_stream)
        self.eng.set_population_hint(0, max(1, min(n, int(share * 1.05))))
        self.tick_no = 0
        self.max_new = 0  # region state: the most new ids or Leaves of one tick so far
        self.xev = []  # (start, end) hipEvents of timed exchanges (tick_rccl(time_exchange=True))
        # per-tick device time of the strip's own kernels (walk + select, absorb + emit), when timing
        # (scripts/strips_loopback_bench.py): hipEvents on the node's stream, read by strip_kernel_ms()
        self.timing = False
        self.sev = []
        # the ctypes arguments that never change, built once (the per-tick calls' host time is the gap
        # between the strip kernels on the stream)
        self._c_s = ctypes.c_void_p(self.stream.cuda_stream)
        self._c_g = ctypes.byref(self.g)
        self._c_err = ctypes.c_void_p(self.counts.data_ptr() + 12)
        self._c_R = ctypes.byref(self.R) if self.R is not None else None
        self._c_sel = (_ptr(self.left), _ptr(self.right), self.cap, ctypes.c_void_p(self.counts.data_ptr()))
        self._c_ops = (_ptr(self.ids), _ptr(self.ox), _ptr(self.oz), _ptr(self.kinds),
                       ctypes.c_void_p(self.counts.data_ptr() + 8))

    # ---- raw kernel calls ----
    def _s(self):
        return self._c_s

    def _g(self):
        return self._c_g

    def _err(self):
        return self._c_err

    def _emit_and_tick(self, host_events: bool, n_bound: int, start=None):
        """The op list goes to the manager with its count in device memory (no host round trip);
        n_bound bounds it: entities present at the start + records received this tick. start: tick 0's
        global-id arrays (flags, ex, ez) with a region state."""
        L = self._L
        common = (self._s(), self._g(), _ptr(self.flags), _ptr(self.sx), _ptr(self.sz), _ptr(self.ex), _ptr(self.ez),
                  _ptr(self.ids), _ptr(self.ox), _ptr(self.oz), _ptr(self.kinds), _ptr(self.scratch),
                  ctypes.c_void_p(self.counts.data_ptr() + 8))
        ops = self._c_ops
        if self.R is not None:
            if start is not None:
                check(L.gwaoi_strip_region_start(self._s(), self._g(), self._c_R, *(_ptr(a) for a in start), *ops))
            else:
                check(L.gwaoi_strip_region_emit(self._s(), self._g(), self._c_R, *ops))
        elif self.local:
            check(L.gwaoi_strip_emit_local(*common, _ptr(self.g2l), _ptr(self.l2g), _ptr(self.fq), _ptr(self.pend),
                                           self.cap_l, _ptr(self.lctr)))
        else:
            check(L.gwaoi_strip_emit(*common))
        self.h_ctrs.copy_(self.ctrs, non_blocking=True)  # every counter, stream-ordered before the tick's kernels
        f1 = self._mark()
        if f1 is not None and getattr(self, "_f0", None) is not None and getattr(self, "_ev_prep", (None, None))[1]:
            self.sev.append((self._ev_prep[0], self._ev_prep[1], self._f0, f1))
        self._f0 = None
        n_bound = max(1, min(self.cap_l if self.local else self.n, int(n_bound)))
        self.eng.stage_ops_device(self.ids.data_ptr(), self.ox.data_ptr(), self.oz.data_ptr(),
                                  self.kinds.data_ptr(), n_bound, d_count=self.counts.data_ptr() + 8)
        if host_events and self.local:
            dev_ev = self.eng.tick_device()
            ev = self._events_to_host(dev_ev)
        else:
            ev = self.eng.tick() if host_events else self.eng.tick_device()
        c = self.h_counts  # complete: the tick waited for every kernel after the copy
        flags = int(c[3]) | (int(self.h_lctr[3]) if self.local else 0) | (int(self.h_rctr[6]) if self.R is not None else 0)
        if flags:
            why = ""
            if flags & STRIP_ERR_SLOTS:
                why = " (the region holds more entities than its local slots, cap_l = %d: nothing of this tick was " \
                      "applied)" % self.cap_l
            elif flags & STRIP_ERR_NEWLIST:
                why = " (more than cap_new = %d entities came into or left the region in one tick: nothing of this " \
                      "tick was applied, the region state is not usable any more)" % self.R.cap_new
            raise _lib.GwaoiError(_lib.GWAOI_ERR_STATE, f"strip {self.rank}: protocol check failed (flags "
                                  f"{flags}){why}")
        self.last_ops = int(c[2])
        if self.R is not None:  # (the emit flipped cur: the tick's new ids were counted on the other side)
            cur = int(self.R.cur)
            self.max_new = max(self.max_new, int(self.h_rctr[2 + (cur ^ 1)]), int(self.h_rctr[4 + cur]))
        return ev

    def _events_to_host(self, ev) -> np.ndarray:
        """Device events of a local-slot tick -> (n, 2) global ids in the canonical order of one manager
        over the world: op (= global id) order, Leave before Enter, other id ascending."""
        n = int(ev.count)
        if n == 0:
            return np.zeros((0, 2), dtype=np.uint32)
        evp = ctypes.cast(ev.events, ctypes.c_void_p)  # device pointer (GWAOI_TICK_DEVICE_EVENTS)
        check(self._L.gwaoi_strip_translate_events(self._s(), _ptr(self.l2g), evp, n))
        self.stream.synchronize()
        host = np.empty(2 * n, dtype=np.uint32)
        check(self._L.gwaoi_dev_dtoh(self.eng.device, host.ctypes.data_as(ctypes.c_void_p), evp,
                                     8 * n))
        a = host.reshape(n, 2)
        return a[np.lexsort((a[:, 1] & 0x7FFFFFFF, a[:, 1] >> 31, a[:, 0]))]

    def last_op_ids(self) -> np.ndarray:
        """Global ids of the last tick's op list (the manager saw local slots when local_slots)."""
        ids = self.ids[: self.last_ops].cpu().numpy().view(np.uint32)
        if self.local:  # a Leave's slot is only recycled at the next emit: l2g still names it
            return self.l2g.cpu().numpy().view(np.uint32)[ids]
        return ids

    # ---- protocol ----
    def start(self, host_events: bool = False):
        """Tick 0: every entity of the region enters (the seeded workload's initial placement)."""
        with torch.cuda.stream(self.stream):
            if self.R is not None:  # the workload's tick 0 by global id, only for the start
                gf = torch.zeros(self.n, dtype=torch.uint8, device=self.device)
                gx, gz = (torch.zeros(self.n, dtype=torch.float32, device=self.device) for _ in range(2))
            else:
                gf, gx, gz = self.flags, self.ex, self.ez
            if self.skew:
                nhot, sigma, every = self.skew
                check(self._L.gwaoi_strip_init_skew(self._s(), self._g(), _ptr(gf), _ptr(gx), _ptr(gz),
                                                    ctypes.c_uint64(self.seed), ctypes.c_float(self.layout.L),
                                                    int(nhot), ctypes.c_float(sigma), int(every)))
            else:
                check(self._L.gwaoi_strip_init_walk(self._s(), self._g(), _ptr(gf), _ptr(gx), _ptr(gz),
                                                    ctypes.c_uint64(self.seed), ctypes.c_float(self.layout.L)))
            self.tick_no = 0
            return self._emit_and_tick(host_events, self.n, start=(gf, gx, gz) if self.R is not None else None)

    def prepare(self, t: int, step: float = 1.0, moves: Optional[Tuple[torch.Tensor, ...]] = None):
        """End positions of the owned entities (the seeded walk's tick t, or `moves` = (ids, x, z)
        device tensors) and the records each neighbour needs; returns (left, right) device tensors."""
        if moves is not None:  # produced on the caller's stream
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            return self._prepare(t, step, moves)

    def _mark(self):
        if not self.timing:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record(self.stream)
        return e

    def strip_kernel_ms(self) -> Optional[dict]:
        """Mean device time per timed tick of the strip kernels: prepare (walk or ingest + select) and finish
        (absorb + emit), from the hipEvents recorded while `timing` was on."""
        if not self.sev:
            return None
        self.stream.synchronize()
        k = len(self.sev)
        prep = sum(a.elapsed_time(b) for a, b, _, _ in self.sev) / k
        fin = sum(c.elapsed_time(d) for _, _, c, d in self.sev) / k
        return {"ms_strip_prepare": round(prep, 4), "ms_strip_finish": round(fin, 4), "ticks": k}

    def _walk(self, t, step):
        L = self._L
        if self.R is not None:
            check(L.gwaoi_strip_region_walk(self._s(), self._g(), self._c_R, ctypes.c_uint64(self.seed),
                                            ctypes.c_uint64(t), ctypes.c_float(self.layout.L), ctypes.c_float(step),
                                            self._err()))
        else:
            check(L.gwaoi_strip_walk(self._s(), self._g(), _ptr(self.flags), _ptr(self.sx), _ptr(self.sz),
                                     _ptr(self.ex), _ptr(self.ez), ctypes.c_uint64(self.seed), ctypes.c_uint64(t),
                                     ctypes.c_float(self.layout.L), ctypes.c_float(step), self._err()))

    def _ingest(self, moves):
        ids, x, z = moves
        if self.R is not None:
            check(self._L.gwaoi_strip_region_ingest(self._s(), self._g(), ctypes.byref(self.R), _ptr(ids), _ptr(x),
                                                    _ptr(z), int(ids.numel()), self._err()))
        else:
            check(self._L.gwaoi_strip_ingest(self._s(), self._g(), _ptr(self.flags), _ptr(self.sx), _ptr(self.ex),
                                             _ptr(self.ez), _ptr(ids), _ptr(x), _ptr(z), int(ids.numel()),
                                             self._err()))

    def _select(self):
        L = self._L
        if not (self.g.has_left or self.g.has_right):  # a one-strip world: nothing to send (counts stay 0)
            return
        if self.R is not None:
            check(L.gwaoi_strip_region_select(self._s(), self._g(), self._c_R, *self._c_sel, self._err()))
        else:
            check(L.gwaoi_strip_select(self._s(), self._g(), _ptr(self.flags), _ptr(self.sx), _ptr(self.ex),
                                       _ptr(self.ez), _ptr(self.left), _ptr(self.right), self.cap,
                                       ctypes.c_void_p(self.counts.data_ptr()), self._err()))

    def _absorb(self, recs, n_max: int, d_n=None):
        L = self._L
        if self.R is not None:
            check(L.gwaoi_strip_region_absorb(self._s(), ctypes.byref(self.R), _ptr(recs), d_n, int(n_max),
                                              self._err() if d_n is not None else None))
        elif d_n is not None:
            check(L.gwaoi_strip_absorb_n(self._s(), _ptr(self.flags), _ptr(self.ex), _ptr(self.ez), _ptr(recs), d_n,
                                         int(n_max), self._err()))
        else:
            check(L.gwaoi_strip_absorb(self._s(), _ptr(self.flags), _ptr(self.ex), _ptr(self.ez), _ptr(recs),
                                       int(n_max)))

    def _prepare(self, t, step, moves):
        self._ev_prep = (self._mark(),)
        if moves is None:
            self._walk(t, step)
        else:
            self._ingest(moves)
        self._select()
        self._ev_prep = (self._ev_prep[0], self._mark())
        self.tick_no = t
        if not (self.g.has_left or self.g.has_right):  # nothing to send: no round trip (errors: finish)
            return self.left[:0], self.right[:0]
        c = self.counts.cpu()
        if int(c[3]):
            raise _lib.GwaoiError(_lib.GWAOI_ERR_STATE, f"strip {self.rank}: protocol check failed (flags {int(c[3])})")
        return self.left[: int(c[0])], self.right[: int(c[1])]

    def finish(self, left_in: torch.Tensor, right_in: torch.Tensor, host_events: bool = False):
        """Absorb the neighbours' records, run the tick; returns the manager's Events (device) or the
        (n, 2) host array of the owned movers' events in canonical order."""
        self.stream.wait_stream(torch.cuda.current_stream(self.device))  # received on the caller's stream
        with torch.cuda.stream(self.stream):
            nin = 0
            got = []
            for recs in (left_in, right_in):
                if recs is not None and recs.numel():
                    recs = recs.to(self.device).contiguous()
                    recs.record_stream(self.stream)
                    nin += int(recs.shape[0])
                    got.append(recs)
                else:
                    got.append(None)
            f0 = self._mark()  # (from the first strip kernel's launch)
            if self.R is not None and any(g is not None for g in got):  # both messages, one launch
                (a, b) = got
                check(self._L.gwaoi_strip_region_absorb2(
                    self._s(), self._c_R, _ptr(a) if a is not None else None, None,
                    int(a.shape[0]) if a is not None else 0, _ptr(b) if b is not None else None, None,
                    int(b.shape[0]) if b is not None else 0, None))
            elif self.R is None:
                for recs in got:
                    if recs is not None:
                        self._absorb(recs, int(recs.shape[0]))
            self._f0 = f0
            return self._emit_and_tick(host_events, self.eng.count()[0] + nin)

    def tick_rccl(self, t: int, comm: "StripComm", host_events: bool = False, step: float = 1.0,
                  moves: Optional[Tuple[torch.Tensor, ...]] = None, peers: Optional[Tuple[int, int]] = None,
                  time_exchange: bool = False):
        """One whole tick with the halo exchange over RCCL inside libgwaoi (gwaoi_strip_exchange): walk /
        ingest, select, exchange, absorb, emit and the AOI pipeline all enqueued on the node's stream,
        no host round trip before the pipeline's own end-of-pass read. peers = (left, right) rank or -1
        (default: the neighbouring ranks). time_exchange: hipEvents around the exchange on the node's
        stream, kept in self.xev (read after a synchronisation: exchange_ms)."""
        if self.left_in is None:
            dev = self.device
            self.left_in = torch.zeros((self.cap, 4), dtype=torch.int32, device=dev)
            self.right_in = torch.zeros((self.cap, 4), dtype=torch.int32, device=dev)
            self.counts_in = torch.zeros(2, dtype=torch.int32, device=dev)
            torch.cuda.synchronize(dev)
        if peers is None:
            peers = (self.rank - 1 if self.g.has_left else -1, self.rank + 1 if self.g.has_right else -1)
        if moves is not None:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            if moves is None:
                self._walk(t, step)
            else:
                self._ingest(moves)
            self._select()
            if peers[0] >= 0 or peers[1] >= 0:  # (no neighbour: no RCCL call at all)
                if time_exchange:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                check(self._L.gwaoi_strip_exchange(comm.handle, self._s(), int(peers[0]), int(peers[1]),
                                                   _ptr(self.left), _ptr(self.right), _ptr(self.counts), self.cap,
                                                   _ptr(self.left_in), _ptr(self.right_in), _ptr(self.counts_in)))
                if time_exchange:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record()
                    self.xev.append((e0, e1))
            if self.R is not None:  # both messages, one launch (an absent peer: an empty message)
                cin = self.counts_in.data_ptr()
                on = (peers[0] >= 0, peers[1] >= 0)
                check(self._L.gwaoi_strip_region_absorb2(
                    self._s(), ctypes.byref(self.R), _ptr(self.left_in), ctypes.c_void_p(cin) if on[0] else None,
                    self.cap if on[0] else 0, _ptr(self.right_in), ctypes.c_void_p(cin + 4) if on[1] else None,
                    self.cap if on[1] else 0, self._err()))
            else:
                for k, recs in enumerate((self.left_in, self.right_in)):
                    if peers[k] >= 0:
                        self._absorb(recs, self.cap, ctypes.c_void_p(self.counts_in.data_ptr() + 4 * k))
            self.tick_no = t
            return self._emit_and_tick(host_events, self.eng.count()[0] + 2 * self.cap)

    def exchange_ms(self) -> Optional[float]:
        """Mean device time of the timed exchanges (tick_rccl(time_exchange=True)) since the last call:
        the RCCL group on the node's stream, including the wait for the neighbours' matching calls."""
        if not self.xev:
            return None
        self.stream.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in self.xev) / len(self.xev)
        self.xev = []
        return ms

    def close(self):
        self.eng.close()


class StripComm:
    """The RCCL communicator of a strip world inside libgwaoi (gwaoi_strip_comm_*): one rank per GPU.
    The 128-byte id is made on rank 0 and handed to the ranks by the caller (from_dist: over
    torch.distributed; a Go deployment uses its own transport)."""

    def __init__(self, comm_id: bytes, world: int, rank: int, device: int):
        L = _lib.load()
        self._L = L
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(comm_id)
        check(L.gwaoi_strip_comm_init(buf, int(world), int(rank), int(device), ctypes.byref(h)))
        self.handle = h
        self.world, self.rank = int(world), int(rank)

    @staticmethod
    def make_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        check(_lib.load().gwaoi_strip_comm_id(buf))
        return bytes(buf)

    @classmethod
    def from_dist(cls, rank: int, world: int, device: int) -> "StripComm":
        import torch.distributed as dist
        t = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            t[:] = torch.frombuffer(bytearray(cls.make_id()), dtype=torch.uint8)
        obj = [bytes(t.numpy())]
        dist.broadcast_object_list(obj, src=0)
        return cls(obj[0], world, rank, device)

    def close(self):
        if self.handle and self.handle.value:
            self._L.gwaoi_strip_comm_destroy(self.handle)
            self.handle = ctypes.c_void_p()


class LoopbackExchange:
    """Several strips in one process (tests, single-GPU runs): neighbour records handed over directly."""

    @staticmethod
    def exchange(outs: Sequence[Tuple[torch.Tensor, torch.Tensor]]) -> List[Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]]:
        w = len(outs)
        return [(outs[r - 1][1] if r > 0 else None, outs[r + 1][0] if r < w - 1 else None) for r in range(w)]


def exchange_dist(left_out: torch.Tensor, right_out: torch.Tensor, rank: int, world: int,
                  via_cpu: bool = False) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Halo exchange with the two neighbouring ranks over torch.distributed (RCCL with "nccl").
    Sizes first, then the records; every message carries at least one row so no transfer is empty.
    via_cpu: stage through host memory (gloo, e.g. several ranks sharing one GPU in a test)."""
    import torch.distributed as dist
    dev = left_out.device
    tdev = torch.device("cpu") if via_cpu else dev
    peers = [p for p in (rank - 1, rank + 1) if 0 <= p < world]
    out = {rank - 1: left_out, rank + 1: right_out}
    sizes_out = {p: torch.tensor([out[p].shape[0]], dtype=torch.int64, device=tdev) for p in peers}
    sizes_in = {p: torch.zeros(1, dtype=torch.int64, device=tdev) for p in peers}
    ops = []
    for p in peers:
        ops.append(dist.P2POp(dist.isend, sizes_out[p], p))
        ops.append(dist.P2POp(dist.irecv, sizes_in[p], p))
    for r in dist.batch_isend_irecv(ops):
        r.wait()
    ops = []
    recv = {}
    for p in peers:
        k = int(sizes_in[p].item())
        recv[p] = torch.zeros((max(1, k), 4), dtype=torch.int32, device=tdev)
        send = out[p].to(tdev)
        if send.shape[0] == 0:
            send = torch.zeros((1, 4), dtype=torch.int32, device=tdev)
        ops.append(dist.P2POp(dist.isend, send.contiguous(), p))
        ops.append(dist.P2POp(dist.irecv, recv[p], p))
    for r in dist.batch_isend_irecv(ops):
        r.wait()
    res = []
    for p in (rank - 1, rank + 1):
        if p in recv:
            k = int(sizes_in[p].item())
            res.append(recv[p][:k].to(dev))
        else:
            res.append(None)
    return res[0], res[1]
