#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from rocprofv3 --pmc passes (scripts/pmc.sh), medians over
the dispatches of a short config-2 bench, written to profiles/pmc_latest.json for bench.py.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch. MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
reports half the bytes of a wide streaming read (16 B per lane); the sweep's record loads are 16-B
per-lane loads, so fetch bytes are doubled ("corrected"); the raw value is kept beside it.
usage: make_pmc_latest.py <pmc dir prefix> <n entities> [out.json]"""
import collections
import csv
import glob
import json
import sys

prefix, n = sys.argv[1], int(sys.argv[2])
out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_latest.json"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(prefix + "*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
med = lambda v: sorted(v)[len(v) // 2]
kern = {}
for k, cs in vals.items():
    d = {c: med(v) for c, v in cs.items()}
    e = {}
    if "FETCH_SIZE" in d:
        e["fetch_bytes_raw"] = d["FETCH_SIZE"] * 1024.0
        e["fetch_bytes_corrected"] = 2.0 * d["FETCH_SIZE"] * 1024.0
    if "WRITE_SIZE" in d:
        e["write_bytes"] = d["WRITE_SIZE"] * 1024.0
    for c in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_WAVES"):
        if c in d:
            e[c] = d[c]
    if "SQ_LDS_BANK_CONFLICT" in d and d.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_bank_conflict_cycles_frac"] = d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"]
    kern[k.replace("gw::", "")] = e
sw = kern.get("k_sweep", {})
res = {"n": n, "source": prefix, "kernels": kern}
if "fetch_bytes_corrected" in sw and "write_bytes" in sw:
    res["sweep_bytes_per_launch"] = sw["fetch_bytes_corrected"] + sw["write_bytes"]
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
for k, e in sorted(kern.items()):
    print(k, {a: round(b) if isinstance(b, float) and b > 10 else b for a, b in e.items()})
