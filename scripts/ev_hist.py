#!/usr/bin/env python3
"""Per-mover event counts of one moving tick of a bench workload (default skew50): how the order stage's
slices are distributed (k_slice_sort sorts slices of <= 8 events per thread, <= 64 per wave, longer
ones per block). usage: ev_hist.py [workload=skew50] [ticks=3]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
from goworld_amd import _lib  # noqa: E402
from goworld_amd.engine import DeviceBuffer, Engine, wl_init_spaces, wl_iota, wl_step_spaces  # noqa: E402


class A:
    workload = sys.argv[1] if len(sys.argv) > 1 else "skew50"
    n, dist, L, seed, spaces = 1_000_000, 100.0, 35000.0, 0x5EED0002, 512


ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 3
name, n_per, nsp, dists, L, seed0, nhot, sigma, hot_every = bench.spaces_workload(A, 0)
n = n_per * nsp
snap = DeviceBuffer(2 * 4 * n * (ticks + 1), 0)
slots = DeviceBuffer(4 * n, 0)
wl_iota(0, slots.ptr, n)
px = lambda t: snap.ptr + (2 * t) * 4 * n  # noqa: E731
pz = lambda t: snap.ptr + (2 * t + 1) * 4 * n  # noqa: E731
wl_init_spaces(0, px(0), pz(0), n_per, nsp, seed0, L, nhot, sigma, hot_every)
for t in range(1, ticks + 1):
    wl_step_spaces(0, px(t - 1), pz(t - 1), px(t), pz(t), n_per, nsp, seed0, t, L, 1.0)
eng = Engine(capacity=n, device=0, spaces=[(d, (0.0, 0.0, L, L)) for d in dists])
kinds = DeviceBuffer(n, 0)
kinds.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
spc = DeviceBuffer(4 * n, 0)
spc.upload(np.repeat(np.arange(nsp, dtype=np.uint32), n_per))
eng.stage_ops_device(slots.ptr, px(0), pz(0), kinds.ptr, n, spc.ptr)
eng.tick_device()
for t in range(1, ticks):
    eng.stage_moves_device(slots.ptr, px(t), pz(t), n)
    eng.tick_device()
eng.stage_moves_device(slots.ptr, px(ticks), pz(ticks), n)
ev = eng.tick()
cnt = np.bincount(ev[:, 0], minlength=n)
edges = [0, 1, 2, 9, 65, 257, 1025, 4097, 1 << 30]
out = {"workload": A.workload, "events": int(ev.shape[0]), "movers": n, "buckets": []}
for lo, hi in zip(edges[:-1], edges[1:]):
    m = (cnt >= lo) & (cnt < hi)
    out["buckets"].append({"len": f"[{lo},{hi})", "ops": int(m.sum()), "events": int(cnt[m].sum())})
sp = np.repeat(np.arange(nsp), n_per)
out["per_space"] = [{"D": dists[s], "events": int(cnt[sp == s].sum()), "max": int(cnt[sp == s].max()),
                     "ops_gt64": int((cnt[sp == s] > 64).sum())} for s in range(nsp)]
print(json.dumps(out))
