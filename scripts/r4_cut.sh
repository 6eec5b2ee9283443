#!/bin/bash
# Round 4, timing only: where k_mixcs's time goes at 512 workers (A/B library, DOPT_MIXCS_CUT ends
# the kernel early: 1 after the worker loop, 2 after xbar, 3 no fold block, 4 before the ticket).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
export DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so
B="bench.py --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 30 --warmup 3"
for cut in 0 4 1 2 3; do
  echo "=== cut $cut"
  DOPT_MIXCS_CUT=$cut timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_cut$cut -o run \
    -- python3 $B > gpurun_out/r4_cut$cut.log 2>&1 || { tail -n 20 gpurun_out/r4_cut$cut.log; exit 1; }
  python3 tools/trace_rounds.py gpurun_out/r4_cut$cut/run_kernel_trace.csv
done
