#!/bin/bash
# Round 2: rocprofv3 evidence for configs C4 (65536 workers, torus, float64 over float32 rows)
# and C5 (d = 2^20 column-blocked, float32) on one GPU -> profiles/r2_c4_*, profiles/r2_c5_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--config c4 --steps 5" OUT=gpurun_out/prof_c4 bash scripts/profile.sh > gpurun_out/prof_c4.out 2>&1 || { tail -n 20 gpurun_out/prof_c4.out; exit 1; }
python scripts/pmc_summary.py gpurun_out/prof_c4 r2_c4 || exit $?
BENCH_ARGS="--config c5 --dtype float32 --steps 5" OUT=gpurun_out/prof_c5 bash scripts/profile.sh > gpurun_out/prof_c5.out 2>&1 || { tail -n 20 gpurun_out/prof_c5.out; exit 1; }
python scripts/pmc_summary.py gpurun_out/prof_c5 r2_c5 || exit $?
mkdir -p gpurun_out/profiles && cp profiles/r2_c* gpurun_out/profiles/
echo "=== done"
