#!/usr/bin/env python3
"""Phase shares of the dense walk from a GW_STAMPS dump (bench.py --stamps; k_sweep_dense sums its
per-wave s_memtime deltas into words 16*16383 + k). usage: dense_stamps.py <dump.npy>"""
import sys

import numpy as np

d = np.load(sys.argv[1]).reshape(-1)[16 * 16383:16 * 16384].astype(np.float64)
names = ["batch loads", "mover setup", "part enumeration", "range loads + scan", "candidate rounds"]
tot = d[:5].sum()
for k, nm in enumerate(names):
    print(f"{nm:22s} {d[k] / tot:6.1%}   {d[k] / max(d[8], 1):10.0f} cycles per mover")
print(f"movers {d[8]:.0f}  flushes per mover {d[9] / max(d[8], 1):.2f}  rounds per mover {d[10] / max(d[8], 1):.2f}  "
      f"cycles per mover {tot / max(d[8], 1):.0f}")
