#!/usr/bin/env python3
"""Summary of rocprofv3 SQ counter passes for the round kernels (scripts/r4.sh sq).

Arguments: counter-collection output directories (run_counter_collection.csv), then optionally one
kernel-trace directory (run_kernel_trace.csv) for each kernel's VGPR / AGPR / LDS / scratch.  Prints,
per k_round / k_mix / k_colsum kernel, the per-dispatch mean of every counter and the ratios that
say where the wave time goes: issue (SQ_ACTIVE_INST_ANY) vs waiting (SQ_WAIT_ANY) per wave cycle,
VALU utilisation per SQ busy cycle, and the per-SIMD wave occupancy (SQ_LEVEL_WAVES /
SQ_BUSY_CYCLES: SQ_LEVEL_WAVES accumulates the resident waves every cycle, per SE)."""
import collections
import csv
import os
import sys

KEYS = ("k_round", "k_mix", "k_colsum", "k_rs_pass")


def main(dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    res = {}
    for d in dirs:
        p = os.path.join(d, "run_counter_collection.csv")
        if os.path.exists(p):
            for r in csv.DictReader(open(p)):
                if any(k in r["Kernel_Name"] for k in KEYS):
                    acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        p = os.path.join(d, "run_kernel_trace.csv")
        if os.path.exists(p):
            for r in csv.DictReader(open(p)):
                if any(k in r["Kernel_Name"] for k in KEYS):
                    res[r["Kernel_Name"]] = {k: r[k] for k in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                                                "LDS_Block_Size", "Scratch_Size", "Workgroup_Size_X",
                                                                "Grid_Size_X")}
    for k in sorted(acc, key=lambda s: -len(acc[s].get("SQ_WAVE_CYCLES", []))):
        m = {c: sum(v) / len(v) for c, v in acc[k].items()}
        print(k)
        if k in res:
            print("  resources:", res[k])
        print("  per-dispatch means:", {c: round(v) for c, v in sorted(m.items())})
        wc = m.get("SQ_WAVE_CYCLES")
        busy = m.get("SQ_BUSY_CYCLES")
        r = {}
        if wc:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA",
                      "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_INST_CYCLES_VMEM"):
                if c in m:
                    r[c + "/wave_cycle"] = round(m[c] / wc, 3)
        if m.get("SQ_WAVES") and wc:
            r["wave_cycles_per_wave"] = round(wc / m["SQ_WAVES"])
        if busy and m.get("SQ_LEVEL_WAVES"):
            r["resident_waves_per_busy_cycle_per_SE"] = round(m["SQ_LEVEL_WAVES"] / busy, 2)
        if m.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_TRANS_F64",
                      "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_INSTS_SMEM"):
                if c in m:
                    r[c + "/wave"] = round(m[c] / m["SQ_WAVES"], 1)
        if m.get("SQ_ACTIVE_INST_LDS") and "SQ_LDS_BANK_CONFLICT" in m:
            r["lds_bank_conflict/active_lds"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_ACTIVE_INST_LDS"], 3)
        if m.get("GRBM_GUI_ACTIVE") and busy:
            r["sq_busy/gui_active"] = round(busy / m["GRBM_GUI_ACTIVE"], 3)
        print("  ratios:", r)


if __name__ == "__main__":
    main(sys.argv[1:])
