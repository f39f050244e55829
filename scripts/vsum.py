#!/usr/bin/env python3
"""Summarise variant bench lines: python scripts/vsum.py gpurun_out/TAG_*.json"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads([ln for ln in open(f) if ln.startswith("{")][-1])
    except Exception as e:  # noqa: BLE001
        print(f"{f}: unreadable ({e})")
        continue
    s = d.get("stage_ms") or d.get("stage_ms_rank0") or {}
    print(f"{f:40s} ms/step {d['ms_per_step']:.4f} p50 {d.get('p50_tick_ms', 0):.4f} "
          + " ".join(f"{k[3:]} {v * 1e3:.1f}" for k, v in s.items()) + f"  ev {d.get('events_per_tick', 0):.0f}")
