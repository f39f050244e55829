#!/usr/bin/env python3
"""Per-mover event counts (the order stage's slice lengths) of one tick of a spaces workload (bench.py's
skew50 by default): how many slices, and how many events, fall in each length class of k_slice_sort
(registers <= 8, wave window <= GW_MED_MAX, block bitonic above). usage: slice_hist.py [workload] [ticks]"""
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
    pass


args = A()
args.workload = sys.argv[1] if len(sys.argv) > 1 else "skew50"
args.spaces = 4
args.n, args.dist, args.L, args.seed = 1_000_000, 100.0, 35000.0, 0x5EED0002
ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 3
name, n_per, nsp, dists, L, seed0, nhot, sigma, every = bench.spaces_workload(args, 0)
n = n_per * nsp
dev = 0
px, pz, qx, qz = (DeviceBuffer(4 * n, dev) for _ in range(4))
slots = DeviceBuffer(4 * n, dev)
wl_iota(dev, slots.ptr, n)
wl_init_spaces(dev, px.ptr, pz.ptr, n_per, nsp, seed0, L, nhot, sigma, every)
eng = Engine(capacity=n, device=dev, spaces=[(d, (0.0, 0.0, L, L)) for d in dists])
kinds = DeviceBuffer(n, dev)
kinds.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
spc = DeviceBuffer(4 * n, dev)
spc.upload(np.repeat(np.arange(nsp, dtype=np.uint32), n_per))
eng.stage_ops_device(slots.ptr, px.ptr, pz.ptr, kinds.ptr, n, spc.ptr)
eng.tick_device()
edges = [0, 1, 2, 9, 65, 257, 513, 2049, 8193, 1 << 31]
out = {"workload": name, "ticks": []}
for t in range(1, ticks + 1):
    wl_step_spaces(dev, px.ptr, pz.ptr, qx.ptr, qz.ptr, n_per, nsp, seed0, t, L, 1.0)
    px, qx, pz, qz = qx, px, qz, pz
    eng.stage_moves_device(slots.ptr, px.ptr, pz.ptr, n)
    ev = eng.tick()
    mv = ev[:, 0]
    cnt = np.bincount(mv, minlength=n)
    rows = []
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = (cnt >= lo) & (cnt < hi)
        rows.append({"len": f"[{lo},{hi})", "slices": int(sel.sum()), "events": int(cnt[sel].sum())})
    sp = np.arange(n) // n_per
    per_space = [int(cnt[sp == k].sum()) for k in range(nsp)]
    out["ticks"].append({"events": int(len(ev)), "max_slice": int(cnt.max()), "classes": rows,
                         "events_per_space": per_space})
    print(f"tick {t}: {len(ev)} events, max slice {cnt.max()}", file=sys.stderr, flush=True)
print(json.dumps(out))
eng.close()
