#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from rocprofv3 --pmc passes (scripts/pmc.sh) over a short bench
run of one workload, medians over the dispatches, merged into profiles/pmc_latest.json under
workloads[<workload>] for bench.py's roofline `traffic`.

Each entry carries the source stamp of the library the passes ran (`lib_src`, from the bench JSON lines
the passes wrote: gwaoi_version() ends with "src <hash>", goworld_amd/build.py source_hash). bench.py
uses an entry only when its stamp equals the stamp of the library it loaded, so a kernel change makes
the traffic figure null until the PMC passes are run again.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch. MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
reports half the bytes of a wide streaming read (16 B per lane); the sweep's record loads are 16-B
per-lane loads, so fetch bytes are doubled ("corrected"); the raw value is kept beside it.
usage: make_pmc_latest.py <pmc dir prefix> <workload> [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

prefix, workload = sys.argv[1], sys.argv[2]
out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_latest.json"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(prefix + "*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        name = name.replace("void ", "").replace("gw::", "").strip()
        # the LDS sweep's two sizes and the ring walk's two lists under stable names
        if name.startswith("k_sweep<SwCfg<"):
            # SwCfg<threads, record cap, ...>: the small sweep (512, cap <= 1600), the mid one (512, more) and the
            # big one (1024)
            args = [x.strip() for x in name[len("k_sweep<SwCfg<"):].split(",")]
            blk, cap = int(args[0]), int(args[1])
            name = "k_sweep_big" if blk > 512 else ("k_sweep_mid" if cap > 1600 else "k_sweep")
        elif name.startswith("k_sweep_dense<"):
            name = "k_sweep_dense"
        elif name.startswith("k_sweep_band<"):
            name = "k_sweep_band"
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
lib, n = set(), set()
for f in sorted(glob.glob(prefix + "*.json")):
    try:
        line = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    if "lib" in line:
        lib.add(line["lib"].rsplit(" src ", 1)[-1])
    c = line.get("config", {})
    n.add(c.get("entities_per_gpu") or c.get("entities_total"))
if len(lib) != 1 or len(n) != 1:
    sys.exit(f"make_pmc_latest: need exactly one library stamp and size across {prefix}*.json, got {lib} {n}")
med = lambda v: sorted(v)[len(v) // 2]
kern = {}
for k, cs in vals.items():
    d = {c: med(v) for c, v in cs.items()}
    e = {"dispatches": max(len(v) for v in cs.values())}
    if "FETCH_SIZE" in d:
        e["fetch_bytes_raw"] = d["FETCH_SIZE"] * 1024.0
        e["fetch_bytes_corrected"] = 2.0 * d["FETCH_SIZE"] * 1024.0
    if "WRITE_SIZE" in d:
        e["write_bytes"] = d["WRITE_SIZE"] * 1024.0
    if "fetch_bytes_corrected" in e and "write_bytes" in e:
        e["bytes"] = e["fetch_bytes_corrected"] + e["write_bytes"]
    for c in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_WAVES",
              "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"):
        if c in d:
            e[c] = d[c]
    if "SQ_LDS_BANK_CONFLICT" in d and d.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_bank_conflict_cycles_frac"] = d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"]
    if "SQ_WAIT_ANY" in d and d.get("SQ_WAVE_CYCLES"):
        e["wait_any_frac"] = d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]
    kern[k] = e
# the workload's roofline kernel(s), as bench.py times them (the pass's sweep stage)
dominant = {"gametick": ["k_fan_dwrite", "k_fan_tile<true>"]}.get(workload, ["k_sweep", "k_sweep_mid", "k_sweep_big", "k_band_sort", "k_sweep_band", "k_sweep_dense"])
# (only kernels that ran (nearly) every tick of the passes, >= 3/4 of k_sweep's dispatches: a band walk launched once
# in a config-2 run, for the bulk Enter pass, is not the tick's)
per_tick = kern.get("k_sweep", {}).get("dispatches", 0)
summed = [k for k in dominant if "bytes" in kern.get(k, {}) and kern[k].get("dispatches", 0) >= 0.75 * per_tick]
entry = {"lib_src": lib.pop(), "n": n.pop(), "source": prefix, "kernels": kern, "kernels_summed": summed,
         "bytes_per_launch": sum(kern[k]["bytes"] for k in summed) if summed else None}
res = {}
if os.path.exists(out):
    try:
        res = json.load(open(out))
    except ValueError:
        res = {}
if "workloads" not in res:
    res = {"workloads": {}}
res["workloads"][workload] = entry
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps({k: v for k, v in entry.items() if k != "kernels"}, indent=1))
for k, e in sorted(kern.items()):
    print(k, {a: round(b) if isinstance(b, float) and b > 10 else b for a, b in e.items()})
