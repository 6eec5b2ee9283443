#!/usr/bin/env python3
"""Per-leg view of a rocprofv3 kernel trace (run_kernel_trace.csv) of a process that runs several timed
legs one after another (tools/rank_proxy.py, bench.py): the legs are split at host gaps of more than
`gap_ms` with no kernel running; for each leg's last half of rounds (rounds delimited by the most
frequent k_round instance) it prints the round period, the gradient kernel's median duration, each other
kernel's median duration, count per round and median start offset from the round's gradient kernel
start, and the GPU idle time per round.

  python3 tools/trace_legs.py gpurun_out/<dir>/run_kernel_trace.csv [gap_ms] [round_kernel_substring]

(the rounds of the row-space path: round_kernel_substring = k_rs_rows, one launch per round)
"""
import collections
import csv
import statistics
import sys


def legs(ev, gap_ns):
    out, cur, end = [], [], None
    for e in ev:
        if cur and e[0] - end > gap_ns:
            out.append(cur)
            cur = []
        cur.append(e)
        end = e[1] if end is None or not cur[:-1] else max(end, e[1])
    if cur:
        out.append(cur)
    return out


def leg_stats(ev, key="k_round"):
    counts = collections.Counter(n for _, _, n in ev if key in n)
    if not counts:
        return None
    grad = counts.most_common(1)[0][0]
    starts = [i for i, e in enumerate(ev) if e[2] == grad]
    rounds = list(zip(starts[:-1], starts[1:]))
    rounds = rounds[len(rounds) // 2:]
    if not rounds:
        return None
    per, idle, gdur = [], [], []
    other = collections.defaultdict(list)
    offs = collections.defaultdict(list)
    for a, b in rounds:
        t0, t1 = ev[a][0], ev[b][0]
        per.append((t1 - t0) / 1e3)
        gdur.append((ev[a][1] - ev[a][0]) / 1e3)
        busy, cur_s, cur_e = 0, None, None
        for s, e, n in ev[a:b]:
            if n != grad:
                other[n].append((e - s) / 1e3)
                offs[n].append((s - t0) / 1e3)
            s, e = max(s, t0), min(e, t1)
            if e <= s:
                continue
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        idle.append((t1 - t0 - busy) / 1e3)
    n = len(rounds)
    return {"grad": grad, "rounds": n, "period": statistics.median(per), "grad_us": statistics.median(gdur),
            "idle": statistics.median(idle),
            "other": {k: (len(v) / n, statistics.median(v), statistics.median(offs[k])) for k, v in other.items()}}


def main(path, gap_ms=5.0, key="k_round"):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    for i, leg in enumerate(legs(ev, gap_ms * 1e6)):
        st = leg_stats(leg, key)
        if st is None or st["rounds"] < 5:
            continue
        print(f"leg {i}: {st['rounds']} steady rounds of {st['grad'][:60]}")
        print(f"  period {st['period']:.2f} us, gradient kernel {st['grad_us']:.2f} us, GPU idle {st['idle']:.2f} us")
        for k, (cnt, med, off) in sorted(st["other"].items(), key=lambda kv: -kv[1][1]):
            print(f"  {cnt:5.2f}/round  median {med:8.2f} us  starts +{off:8.2f} us  {k[:80]}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 5.0, sys.argv[3] if len(sys.argv) > 3 else "k_round")
