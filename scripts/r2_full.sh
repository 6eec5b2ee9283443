#!/bin/bash
# Round 2: every GPU test + smoke, the default bench line, and the rocprofv3 evidence of the
# headline kernel (kernel stats + FETCH_SIZE / WRITE_SIZE passes -> profiles/r2_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAILN=4 bash scripts/gpu_tests.sh || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err || { tail -n 20 gpurun_out/r2_bench.err; exit 1; }
tail -n 1 gpurun_out/r2_bench.json
BENCH_ARGS="--no-secondary --steps 50" OUT=gpurun_out/prof bash scripts/profile.sh || exit $?
python scripts/pmc_summary.py gpurun_out/prof r2 || exit $?
mkdir -p gpurun_out/profiles && cp profiles/r2_* gpurun_out/profiles/
echo "=== done"
