#!/bin/bash
# Round-end evidence for profiles/: C3 fused path (kernel stats + FETCH_SIZE / WRITE_SIZE
# passes -> profiles/<tag>_*), and the multi-GPU phase path on one GPU (kernel stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r1}
OUT=gpurun_out/prof bash scripts/profile.sh || exit $?
python scripts/pmc_summary.py gpurun_out/prof $TAG || exit $?
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_phase -o run -- \
  python -u bench.py --no-cpu-baseline --phase --steps 10 --warmup 1 > gpurun_out/prof_phase.log 2>&1 || exit $?
cp gpurun_out/prof_phase/run_kernel_stats.csv profiles/${TAG}_phase_kernel_stats.csv
mkdir -p gpurun_out/profiles && cp profiles/${TAG}_* gpurun_out/profiles/
echo "=== done"
