#!/usr/bin/env python3
"""Ring-walk phase shares of k_sweep from a GW_STAMPS dump (bench.py --stamps; sweep_lds sums per
wave the s_memtime deltas of its phases into words 16*16382 + k). usage: sweep_stamps.py <dump.npy>"""
import sys

import numpy as np

d = np.load(sys.argv[1]).reshape(-1)[16 * 16382:16 * 16383].astype(np.float64)
names = ["judge setup + ring plan", "row stream", "column stream", "emission"]
tot = d[:4].sum()
n = max(d[4], 1.0)
for k, nm in enumerate(names):
    print(f"{nm:24s} {d[k] / tot:6.1%}   {d[k] / n:8.0f} cycles per wave-walk")
print(f"wave-walks {d[4]:.0f}   cycles per wave-walk {tot / n:.0f}")
