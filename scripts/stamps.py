#!/usr/bin/env python3
"""Analyse per-block sweep phase stamps (bench.py --stamps, GW_STAMPS=1 build).
Columns: 0 start, 1 before staging, 2 after staging, 3 after walk barrier, 4 end (s_memrealtime, 100 MHz),
5 staged records, 6 HW_ID | XCC_ID << 32, 7 thread 0 walk done; 8-13 staging / ordering sub-phases."""
import sys
import numpy as np

a = np.load(sys.argv[1]).astype(np.int64)
# optional item range [lo, hi) (tile indices: e.g. the big sweep's Spaces), else the first n items
if len(sys.argv) > 3:
    a = a[int(sys.argv[2]):int(sys.argv[3])]
    a = a[a[:, 0] > 0]
    n = a.shape[0]
else:
    n = int(sys.argv[2]) if len(sys.argv) > 2 else int((a[:, 0] > 0).sum())
    a = a[:n]
t0 = a[:, 0].min()
us = lambda v: v / 100.0  # 100 MHz -> us
print(f"blocks {n}; kernel span {us(a[:, 4].max() - t0):.1f} us")
phases = {"pre": (0, 1), "stage": (1, 2), "walk": (2, 3), "flush": (3, 4), "total": (0, 4)}
if a.shape[1] >= 14 and a[:, 13].any():  # sub-phases (16-word stamps)
    phases.update({" cells+scan": (1, 8), " srcmap": (8, 9), " colmajor": (9, 10), " gather": (10, 11),
                   " stage end": (11, 2), " count": (2, 12), " sort": (12, 13), " walk only": (13, 3)})
for name, (i, j) in phases.items():
    d = us(a[:, j] - a[:, i])
    print(f"  {name:6s} mean {d.mean():7.2f}  p50 {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f}")
st = us(a[:, 0] - t0)
print("  start times: p10 %.1f p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(st, [10, 50, 90, 100])))
xcc = a[:, 6] >> 32
hw = a[:, 6] & 0xffffffff
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
key = xcc * 1000 + se * 100 + sh * 16 + cu
u, c = np.unique(key, return_counts=True)
print(f"  distinct CUs {len(u)}; blocks per CU min {c.min()} max {c.max()}")
# concurrency: blocks alive over time
ev = sorted([(x, 1) for x in a[:, 0]] + [(x, -1) for x in a[:, 4]])
cur = mx = 0
for _, d in ev:
    cur += d
    mx = max(mx, cur)
print(f"  max concurrent blocks {mx} (of {len(u)} CUs)")
