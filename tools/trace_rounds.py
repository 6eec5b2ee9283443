#!/usr/bin/env python3
"""Per-round view of a rocprofv3 kernel trace (run_kernel_trace.csv): the rounds are delimited by
the launches of the gradient kernel (the k_round dispatch that occurs most often); for the last
half of the rounds it prints the median round period, the gradient kernel's median duration, each
other kernel's median duration and count per round, and the median idle time of the GPU per round
(period minus the union of the busy intervals)."""
import collections
import csv
import statistics
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    counts = collections.Counter(n for _, _, n in ev if "k_round" in n)
    if not counts:
        print("no k_round dispatches")
        return
    grad = counts.most_common(1)[0][0]
    starts = [i for i, e in enumerate(ev) if e[2] == grad]
    rounds = list(zip(starts[:-1], starts[1:]))
    rounds = rounds[len(rounds) // 2:]  # steady state
    per, idle, gdur = [], [], []
    other = collections.defaultdict(list)
    ncount = collections.Counter()
    for a, b in rounds:
        t0, t1 = ev[a][0], ev[b][0]
        per.append((t1 - t0) / 1e3)
        gdur.append((ev[a][1] - ev[a][0]) / 1e3)
        busy, cur_s, cur_e = 0, None, None
        for s, e, n in ev[a:b]:
            e = min(e, t1)
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            if n != grad:
                other[n].append((e - s) / 1e3)
                ncount[n] += 1
        if cur_e is not None:
            busy += cur_e - cur_s
        idle.append((t1 - t0 - busy) / 1e3)
    R = len(rounds)
    print(f"{path}: {R} steady rounds; gradient kernel {grad}")
    print(f"  round period median {statistics.median(per):.2f} us; gradient kernel median "
          f"{statistics.median(gdur):.2f} us; GPU idle per round median {statistics.median(idle):.2f} us")
    for n, v in sorted(other.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {ncount[n] / R:5.2f}/round  median {statistics.median(v):8.2f} us  {n[:110]}")


if __name__ == "__main__":
    main(sys.argv[1])
