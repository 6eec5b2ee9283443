#!/bin/bash
# x32 round kernel with LDS-staged CSR rows (VAR bit 4): the parity tests of the C3 path, then
# the C3 and C4 profiles (kernel stats + FETCH / WRITE passes -> profiles/r3_*, r3_c4_*) and the
# driver-shaped bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale_parity.py tests/test_gpu_distributed.py tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pre_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/pre_tests.log; [ $rc -eq 0 ] || exit $rc
PSTEPS=10 OUT=gpurun_out/prof_c3 bash scripts/profile.sh > gpurun_out/prof_c3.out 2>&1 || { tail -n 20 gpurun_out/prof_c3.out; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/prof_c3 r3 || exit $?
BENCH_ARGS="--config c4" PSTEPS=6 OUT=gpurun_out/prof_c4 bash scripts/profile.sh > gpurun_out/prof_c4.out 2>&1 || { tail -n 20 gpurun_out/prof_c4.out; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/prof_c4 r3_c4 || exit $?
cp profiles/r3_pmc.json profiles/r3_kernel_stats.csv profiles/r3_c4_pmc.json profiles/r3_c4_kernel_stats.csv gpurun_out/profiles/
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/pre_bench.json 2> gpurun_out/pre_bench.err || { tail -n 20 gpurun_out/pre_bench.err; exit 1; }
tail -n 1 gpurun_out/pre_bench.json | cut -c 1-300
