#!/bin/bash
# C5 at float64 arithmetic on one box: the bench line with float32-stored rows (k_rs_pass_x32, the
# default) and with float64-stored rows (--data-dtype float64), then rocprofv3 kernel stats +
# FETCH_SIZE / WRITE_SIZE of the default run -> profiles/r2_c5x32_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 > gpurun_out/c5x32.json 2> gpurun_out/c5x32.err \
  || { tail -n 20 gpurun_out/c5x32.err; exit 1; }
tail -n 1 gpurun_out/c5x32.json | cut -c 1-400
timeout -k 10 300 python -u bench.py --config c5 --data-dtype float64 --steps 20 --warmup 5 > gpurun_out/c5f64.json \
  2> gpurun_out/c5f64.err || { tail -n 20 gpurun_out/c5f64.err; exit 1; }
tail -n 1 gpurun_out/c5f64.json | cut -c 1-400
BENCH_ARGS="--config c5" PSTEPS=8 OUT=gpurun_out/prof_c5x32 bash scripts/profile.sh > gpurun_out/prof_c5x32.out 2>&1 \
  || { tail -n 20 gpurun_out/prof_c5x32.out; exit 1; }
python scripts/pmc_summary.py gpurun_out/prof_c5x32 r2_c5x32 || exit $?
cp profiles/r2_c5x32_* gpurun_out/profiles/
echo "=== done"
