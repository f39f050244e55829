#!/usr/bin/env python3
"""Per-strip pipeline cost of a W-strip world on ONE GPU (loopback exchange): what each rank of a
W-GPU strips run would pay per tick, stage by stage (hipEvents). Used to see how the per-rank tick
grows with the world size (the manager's slot space is the whole world's id range).
usage: strips_loopback_bench.py [world=8] [per_gpu=2000000] [ticks=20] [streams=shared|own]
shared (default): every strip on one stream, so no strip's kernels overlap another's and its hipEvents time
what its own GPU would run; own: a stream per strip (kernels of different strips overlap, so each strip's
stage times include the others' contention)."""
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (one HIP runtime per process)

from goworld_amd.strips import LoopbackExchange, StripLayout, StripNode  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
per = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
ticks = int(sys.argv[3]) if len(sys.argv) > 3 else 20
shared = (sys.argv[4] if len(sys.argv) > 4 else "shared") == "shared"
n = per * world
L = math.sqrt(n / (1_000_000 / 35000.0 ** 2))
lay = StripLayout(world, L, 100.0, 1.0)
t0 = time.perf_counter()
st = torch.cuda.Stream(0) if shared else None
nodes = [StripNode(lay, r, n, device=0, seed=0x5EED0004, stream=st) for r in range(world)]
for nd in nodes:
    nd.start(host_events=False)
print(f"setup {time.perf_counter() - t0:.1f}s, world {n}, L {L:.0f}", file=sys.stderr, flush=True)
for t in range(1, 4):
    ins = LoopbackExchange.exchange([nd.prepare(t) for nd in nodes])
    for nd, i in zip(nodes, ins):
        nd.finish(*i)
for nd in nodes:
    nd.eng.set_timing(True)
    nd.eng.reset_stats()
    nd.timing = True  # the strip kernels' own device time (walk + select, absorb + emit)
torch.cuda.synchronize()
halo = [0] * world
t0 = time.perf_counter()
for t in range(4, 4 + ticks):
    outs = [nd.prepare(t) for nd in nodes]
    for r, (lo, ro) in enumerate(outs):  # records this strip sends its neighbours (its halo on their side)
        halo[r] += int(lo.shape[0]) + int(ro.shape[0])
    ins = LoopbackExchange.exchange(outs)
    for nd, i in zip(nodes, ins):
        nd.finish(*i)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / ticks * 1e3
rows = []
for nd in nodes:
    st = nd.eng.stats()
    k = max(1, st["ticks"])
    rows.append({key: round(st[key] / k, 4) for key in ("ms_apply", "ms_grid", "ms_sweep", "ms_order", "ms_total")})
    rows[-1].update(nd.strip_kernel_ms() or {})
    rows[-1]["ms_device_total"] = round(rows[-1]["ms_total"] + rows[-1].get("ms_strip_prepare", 0.0)
                                        + rows[-1].get("ms_strip_finish", 0.0), 4)
    rows[-1]["device_total_over_pipeline"] = round(rows[-1]["ms_device_total"] / max(1e-9, rows[-1]["ms_total"]), 4)
    rows[-1]["ops"] = nd.last_ops
    rows[-1]["region_state"] = nd.R is not None  # the strip's state in local-slot order (ABI 2.1)
    rows[-1]["halo_records_sent_per_tick"] = halo[nd.rank] / ticks
    nd.close()
print(json.dumps({"world": world, "per_gpu": per, "ticks": ticks, "streams": "shared" if shared else "own",
                  "halo_records_per_tick": sum(halo) / ticks,
                  "wall_ms_per_tick_all_strips": wall,
                  "note": "W strips of one world on ONE GPU, halo records handed over in-process (LoopbackExchange); "
                          "per strip: its pipeline stages (hipEvents), its strip kernels (prepare = walk + select, finish = "
                          "absorb + emit, hipEvents on its stream), their sum (ms_device_total) and the records it sends "
                          "its neighbours",
                  "per_strip": rows}))
