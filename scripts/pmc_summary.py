#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs (scripts/pmc.sh) per kernel: mean counter value per
dispatch over the dispatches of the timed bench ticks.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 derived counters). Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE on gfx950 reports half the bytes of wide coalesced
streaming reads: `fetch_bytes_corrected` doubles it; other access widths are uncalibrated.

usage: pmc_summary.py <dir-prefix> [--json out.json]
"""
import collections
import csv
import glob
import json
import sys


def load(prefix):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(prefix + "*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    prefix = sys.argv[1]
    per = load(prefix)
    out = {}
    for k, cs in sorted(per.items()):
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in d:
            d["fetch_bytes"] = d["FETCH_SIZE"] * 1024.0
            d["fetch_bytes_corrected"] = 2.0 * d["FETCH_SIZE"] * 1024.0
        if "WRITE_SIZE" in d:
            d["write_bytes"] = d["WRITE_SIZE"] * 1024.0
        if d.get("SQ_WAVE_CYCLES"):
            w = d["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    d[c + "_frac"] = d[c] / w
        if d.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in d and d.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_frac"] = d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"]
        if "TCC_HIT_sum" in d and (d["TCC_HIT_sum"] + d.get("TCC_MISS_sum", 0)) > 0:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        out[k] = d
    for k, d in out.items():
        if d["dispatches"] < 5:
            continue
        print(k)
        for c, v in sorted(d.items()):
            print(f"    {c:28s} {v:16.4f}" if isinstance(v, float) else f"    {c:28s} {v}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
