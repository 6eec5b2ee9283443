#!/usr/bin/env python3
"""Timeline of the round kernels from a rocprofv3 --kernel-trace CSV: per k_round
dispatch its duration, the gap since the previous one ended, and the other kernels
that ran in that gap or overlapped it (where the side-stream work actually landed).

usage: trace_gaps.py <dir with *kernel_trace.csv> [last_n]"""
import csv
import glob
import sys


def short(name):
    name = name.replace("void ", "").replace("dopt::", "")
    return name.split("(")[0][:48]


def main(d, last=12):
    f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[-1]
    rows = []
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rounds = [r for r in rows if "k_round" in r[2] and "true, " in r[2].split("<")[1].split(">")[0][:40]]
    rounds = [r for r in rows if "k_round<" in r[2]]
    print(f"{f}: {len(rows)} dispatches, {len(rounds)} k_round")
    prev_end = None
    gaps = []
    for (s, e, n) in rounds[-last - 1:]:
        others = [(s2, e2, n2) for (s2, e2, n2) in rows
                  if prev_end is not None and "k_round<" not in n2 and e2 > prev_end - 2000000 and s2 < e]
        g = (s - prev_end) / 1e3 if prev_end is not None else float("nan")
        if prev_end is not None:
            gaps.append(g)
        print(f"k_round {short(n):48s} dur {(e - s) / 1e3:9.1f} us  gap {g:7.1f} us")
        for (s2, e2, n2) in others:
            print(f"    {short(n2):44s} start {(s2 - (prev_end or s)) / 1e3:+9.1f} us  dur {(e2 - s2) / 1e3:7.1f} us"
                  f"  {'(inside round)' if s2 >= s else ''}")
        prev_end = e
    if gaps:
        gaps.sort()
        print(f"gap median {gaps[len(gaps) // 2]:.1f} us, min {gaps[0]:.1f}, max {gaps[-1]:.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
