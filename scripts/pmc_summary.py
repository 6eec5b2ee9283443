#!/usr/bin/env python3
"""Fold rocprofv3 outputs (scripts/profile.sh) into profiles/<tag>_*.{csv,json}.

HBM bytes per dispatch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import collections
import csv
import json
import shutil
import sys


def main(src, tag):
    per = collections.defaultdict(lambda: {"fetch_kb": [], "write_kb": []})
    for name, key in (("fetch", "fetch_kb"), ("write", "write_kb")):
        for r in csv.DictReader(open(f"{src}/{name}/run_counter_collection.csv")):
            per[r["Kernel_Name"]][key].append(float(r["Counter_Value"]))
    stats = {r["Name"]: r for r in csv.DictReader(open(f"{src}/stats/run_kernel_stats.csv"))}
    out = {}
    for k, v in per.items():
        f = sum(v["fetch_kb"]) / max(1, len(v["fetch_kb"]))
        w = sum(v["write_kb"]) / max(1, len(v["write_kb"]))
        s = stats.get(k)
        out[k] = {"dispatches": len(v["fetch_kb"]), "fetch_size_kb": f, "write_size_kb": w,
                  "hbm_bytes_per_dispatch": 2 * f * 1024 + w * 1024,
                  "avg_ns": float(s["AverageNs"]) if s else None}
    json.dump(out, open(f"profiles/{tag}_pmc.json", "w"), indent=1)
    shutil.copy(f"{src}/stats/run_kernel_stats.csv", f"profiles/{tag}_kernel_stats.csv")
    print(json.dumps({k[:60]: round(v["hbm_bytes_per_dispatch"] / 1e9, 4) for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof", sys.argv[2] if len(sys.argv) > 2 else "r1")
