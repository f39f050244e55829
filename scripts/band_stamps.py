#!/usr/bin/env python3
"""Phase shares and work counts of the flat band walk from a GW_STAMPS dump (bench.py --stamps;
k_sweep_band sums per-wave s_memtime deltas and counts into words 16*16381 + k; the ring walk's are at
16*16383). usage: band_stamps.py <dump.npy>"""
import sys

import numpy as np

a = np.load(sys.argv[1]).reshape(-1)
for base, title in ((16381, "band walk"), (16383, "ring walk (k_sweep_dense)")):
    d = a[16 * base:16 * base + 16].astype(np.float64)
    print(f"== {title}")
    if base == 16381:
        names = ["batch setup", "item decode", "cell starts", "key search", "candidate rounds"]
        tot = d[:5].sum()
        mv = max(d[15], 1)
        for k, nm in enumerate(names):
            print(f"{nm:18s} {d[k] / max(tot, 1):6.1%}  {d[k] / mv:10.0f} cycles per band mover")
        print(f"band movers {d[15]:.0f}  items/mover {d[11] / mv:.1f}  searched/mover {d[12] / mv:.1f}  "
              f"whole/mover {d[13] / mv:.1f}  candidates/mover {d[14] / mv:.1f}  cand rounds {d[10]:.0f}")
    else:
        names = ["batch loads", "mover setup", "part enumeration", "range loads + scan", "candidate rounds"]
        tot = d[:5].sum()
        mv = max(d[8], 1)
        for k, nm in enumerate(names):
            print(f"{nm:18s} {d[k] / max(tot, 1):6.1%}  {d[k] / mv:10.0f} cycles per mover")
        print(f"movers {d[8]:.0f}  flushes/mover {d[9] / mv:.2f}  rounds/mover {d[10] / mv:.2f}")
