#!/usr/bin/env python3
"""One line per bench JSON: ms/step, stage ms, dense / band movers, events (A/B summaries)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.load(open(f))
    except Exception as e:  # empty or partial line
        print(f, "unreadable:", e)
        continue
    r = d.get("roofline", {})
    st = d.get("stage_ms", {})
    print(f"{f.split('/')[-1]:34s} {d['ms_per_step']:7.3f} ms  " +
          " ".join(f"{k[3:]}={v:.3f}" for k, v in st.items()) +
          f"  dense={r.get('dense_movers_per_tick', 0):.0f} band={r.get('band_movers_per_tick', 0):.0f}"
          f" ev={d.get('events_per_tick', 0):.0f}")
