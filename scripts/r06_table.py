#!/usr/bin/env python3
"""Round-6 DESIGN.md §8 table rows from the evidence calls' JSON (bench lines, loopback).
usage: r06_table.py <default bench json> <workload json dir> <tag> <loopback json>"""
import json
import os
import sys


def load(p):
    try:
        with open(p) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def stages(d):
    s = d.get("stage_ms") or {}
    if not s:
        return ""
    return " / ".join(f"{s.get(k, 0):.3f}" for k in ("ms_apply", "ms_grid", "ms_sweep", "ms_order"))


base, wdir, tag, loop = sys.argv[1:5]
d = load(base)
rows = []
if d:
    rf = d.get("roofline") or {}
    rows.append(
        f"| config 2 (1M, D 100), the BASELINE line | **{d['ms_per_step']:.4f}** | **{d['value']:.3g}** | {stages(d)} | "
        f"host-staged p50 / p99 **{d['p50_tick_ms']:.3f} / {d['p99_tick_ms']:.3f}** (async push; synchronous "
        f"{d.get('p99_tick_ms_sync_staging') or 0:.3f}), device p99 {d.get('p99_tick_ms_device') or 0:.3f}; chunked Flush p99 "
        f"{d.get('p99_flush_ms_chunked') or 0:.3f}; `k_sweep` {rf.get('achieved', 0):.0f} GB/s algorithmic "
        f"({100 * (rf.get('frac') or 0):.1f}% of 8 TB/s), PMC {(rf.get('traffic_bytes_per_launch') or 0) / 1e6:.1f} MB per launch "
        f"for {(rf.get('algorithmic_bytes_per_launch') or 0) / 1e6:.1f} MB algorithmic; relation view "
        f"{d.get('relation_view_ms') or 0:.3f} ms, update {d.get('relation_update_ms') or 0:.3f}, delta "
        f"{d.get('relation_delta_ms') or 0:.3f}; CPU baseline {(d.get('cpu_baseline') or {}).get('value', 0):,.0f} updates/s "
        f"(oracle (i), 1 thread) |")
names = {"config3": "config 3 (512 × 2k per GPU)", "strips": "config 4, one strip of 2M (RCCL exchange path, one rank)",
         "strips_skew": "config 5 in strips: 2M skewed, quantile strips", "skew": "config 5 light (skew)",
         "skew50": "config 5 SURVEY proportions (skew50)", "gametick": "gametick (1M: ingest + AOI tick + fan-out, 8 gates)"}
for w in ("config3", "strips", "strips_skew", "skew", "skew50", "gametick"):
    x = load(os.path.join(wdir, f"{tag}_{w}.json"))
    if not x:
        continue
    note = ""
    if w == "config3":
        note = f"p99 {x.get('p99_tick_ms') or 0:.3f} host-staged"
    if w in ("skew", "skew50"):
        note = f"{(x.get('events_per_tick') or 0) / 1e6:.1f} M events per tick"
    st = stages(x)
    if w == "gametick":
        g = x.get("stage_ms") or {}
        st = ""
        note = f"ingest {g.get('ingest', 0):.3f}, AOI tick {g.get('aoi_tick', 0):.3f}, sync fan-out {g.get('collect_sync', 0):.3f} ms"
    if w == "strips":
        xm = x.get("exchange_ms")
        note = f"p99 {x.get('p99_tick_ms') or 0:.3f}; " + (f"RCCL exchange {1e3 * xm:.1f} µs per tick" if xm is not None
                                                          else "one strip: no halo, no select, no RCCL call")
    rows.append(f"| {names[w]} | **{x['ms_per_step']:.4f}** | {x['value']:.3g} | {st} | {note} |")
lp = load(loop)
if lp:
    ps = lp["per_strip"]
    rows.append(
        f"| config 4, 8 strips of 2M on one GPU (loopback halo, one shared stream) | {min(p['ms_total'] for p in ps):.3f}–"
        f"{max(p['ms_total'] for p in ps):.3f} per strip (pipeline) | | | strip kernels + pipeline "
        f"{min(p['ms_device_total'] for p in ps):.3f}–{max(p['ms_device_total'] for p in ps):.3f} ms per strip "
        f"({min(p['device_total_over_pipeline'] for p in ps):.2f}–{max(p['device_total_over_pipeline'] for p in ps):.2f}× "
        f"the pipeline); {lp['halo_records_per_tick']:,.0f} halo records per tick; all 8 strips {lp['wall_ms_per_tick_all_strips']:.2f} ms "
        f"wall on the one GPU |")
print("| workload | ms/tick | updates/s | stages (apply / grid / sweep / order, ms) | notes |")
print("|---|---|---|---|---|")
print("\n".join(rows))
