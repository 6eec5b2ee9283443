#!/usr/bin/env python3
"""A few steady rounds of a rocprofv3 kernel trace as a timeline (start / end / duration in us from
the round's gradient-kernel start, queue id, VGPRs and LDS as the trace reports them): where the
per-round gaps between kernels sit and which queue each kernel ran on."""
import csv
import sys


def main(path, rounds=3):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"],
                 r["VGPR_Count"], r["LDS_Block_Size"]) for r in rows)
    k = [i for i, e in enumerate(ev) if "k_round" in e[2] and "true, true" in e[2]]
    if len(k) < rounds + 2:
        print("too few rounds")
        return
    i0 = k[-(rounds + 2)]
    t0 = ev[i0][0]
    for e in ev[i0:k[-2]]:
        print(f"{(e[0] - t0) / 1e3:9.2f} {(e[1] - t0) / 1e3:9.2f} {(e[1] - e[0]) / 1e3:8.2f}  q{e[3]:>2} vgpr {e[4]:>3} "
              f"lds {e[5]:>6}  {e[2][:70]}")


if __name__ == "__main__":
    main(sys.argv[1])
