#!/usr/bin/env python3
"""Fold rocprofv3 outputs (scripts/profile.sh) into profiles/<tag>_*.{csv,json}.

HBM bytes per dispatch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B-per-lane stores.

The three passes (kernel trace + stats, FETCH_SIZE, WRITE_SIZE) are three runs of the same bench.py
command in one gpurun call, on one box; each prints its bench line.  The summary keeps, beside the
traffic, the kernel-trace pass's own bench line (value, ms_per_step, the event-timed kernel average)
and the trace's durations of the headline kernel's TIMED dispatches (the last `steps` launches of
the instance the bench line names; the earlier ones are the warmup), so the profile's kernel time
and that run's step time are one measurement."""
import collections
import csv
import json
import shutil
import statistics
import sys


def bench_line(path):
    line = None
    for ln in open(path, errors="replace"):
        if ln.startswith('{"metric"'):
            line = json.loads(ln)
    return line


def main(src, tag):
    per = collections.defaultdict(lambda: {"fetch_kb": [], "write_kb": []})
    for name, key in (("fetch", "fetch_kb"), ("write", "write_kb")):
        for r in csv.DictReader(open(f"{src}/{name}/run_counter_collection.csv")):
            per[r["Kernel_Name"]][key].append(float(r["Counter_Value"]))
    stats = {r["Name"]: r for r in csv.DictReader(open(f"{src}/stats/run_kernel_stats.csv"))}
    trace = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{src}/stats/run_kernel_trace.csv")):
        trace[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    lines = {p: bench_line(f"{src}/{p}.log") for p in ("stats", "fetch", "write")}
    run = lines["stats"] or {}
    steps = int(run.get("steps", 0))
    head = (run.get("roofline") or {}).get("kernel")
    out = {}
    for k, v in per.items():
        f = sum(v["fetch_kb"]) / max(1, len(v["fetch_kb"]))
        w = sum(v["write_kb"]) / max(1, len(v["write_kb"]))
        s = stats.get(k)
        out[k] = {"dispatches": len(v["fetch_kb"]), "fetch_size_kb": f, "write_size_kb": w,
                  "hbm_bytes_per_dispatch": 2 * f * 1024 + w * 1024,
                  "avg_ns": float(s["AverageNs"]) if s else None}
        if k == head and steps and len(trace.get(k, [])) >= steps:
            timed = trace[k][-steps:]
            out[k].update({"timed_dispatches": steps, "timed_avg_ns": statistics.mean(timed),
                           "timed_median_ns": statistics.median(timed), "timed_min_ns": min(timed),
                           "timed_max_ns": max(timed)})
    if run:
        rf = run.get("roofline") or {}
        out["_run"] = {"pass": "kernel trace + stats", "value": run.get("value"), "ms_per_step": run.get("ms_per_step"),
                       "steps": steps, "warmup": run.get("warmup"), "kernel": head,
                       "kernel_avg_ms_events": rf.get("kernel_avg_ms"),
                       "kernel_timed_avg_ms_trace": (out.get(head) or {}).get("timed_avg_ns", 0) / 1e6 or None,
                       "pmc_pass_ms_per_step": {p: (lines[p] or {}).get("ms_per_step") for p in ("fetch", "write")}}
    json.dump(out, open(f"profiles/{tag}_pmc.json", "w"), indent=1)
    shutil.copy(f"{src}/stats/run_kernel_stats.csv", f"profiles/{tag}_kernel_stats.csv")
    print(json.dumps({k[:60]: round(v["hbm_bytes_per_dispatch"] / 1e9, 4) for k, v in out.items() if k != "_run"},
                     indent=1))
    if run:
        print(json.dumps(out["_run"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof", sys.argv[2] if len(sys.argv) > 2 else "r1")
