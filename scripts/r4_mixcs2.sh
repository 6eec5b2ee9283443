#!/bin/bash
# Round 4: k_mixcs as two launches (kernel boundary as the hand-off) -- the multi-GPU tests, then
# one-launch (ticket) vs two-launch kernel traces at 512 workers (A/B library), then
# scripts/r4_mixcs.sh's traces and strong-proxy rows with the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
B="bench.py --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 30 --warmup 3"
for tk in 1 0; do
  echo "=== DOPT_MIXCS_TICKET=$tk (A/B library)"
  DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so DOPT_MIXCS_TICKET=$tk timeout -s KILL 150 rocprofv3 \
    --kernel-trace --output-format csv -d gpurun_out/r4_tk$tk -o run -- python3 $B > gpurun_out/r4_tk$tk.log 2>&1 \
    || { tail -n 20 gpurun_out/r4_tk$tk.log; exit 1; }
  python3 tools/trace_rounds.py gpurun_out/r4_tk$tk/run_kernel_trace.csv
done
bash scripts/r4_mixcs.sh
