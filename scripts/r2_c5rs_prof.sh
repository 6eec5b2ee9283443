#!/bin/bash
# C5 evidence on one box: the bench line through the row-space rounds (default) and through the
# direct column-blocked rounds (DOPT_ROWSPACE=0), then rocprofv3 kernel stats + FETCH_SIZE /
# WRITE_SIZE of the row-space run -> profiles/r2_c5rs_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --config c5 --dtype float32 --steps 20 --warmup 3 --no-cpu-baseline \
  > gpurun_out/c5rs.json 2> gpurun_out/c5rs.err || { tail -n 20 gpurun_out/c5rs.err; exit 1; }
tail -n 1 gpurun_out/c5rs.json | cut -c 1-300
DOPT_ROWSPACE=0 timeout -k 10 300 python -u bench.py --config c5 --dtype float32 --steps 20 --warmup 3 \
  --no-cpu-baseline > gpurun_out/c5direct.json 2> gpurun_out/c5direct.err || { tail -n 20 gpurun_out/c5direct.err; exit 1; }
tail -n 1 gpurun_out/c5direct.json | cut -c 1-300
BENCH_ARGS="--config c5 --dtype float32" PSTEPS=8 OUT=gpurun_out/prof_c5rs bash scripts/profile.sh > gpurun_out/prof_c5rs.out 2>&1 \
  || { tail -n 20 gpurun_out/prof_c5rs.out; exit 1; }
python scripts/pmc_summary.py gpurun_out/prof_c5rs r2_c5rs || exit $?
cp profiles/r2_c5rs_* gpurun_out/profiles/
echo "=== done"
