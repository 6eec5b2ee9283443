#!/bin/bash
# Round 2 evidence on one box: the default bench line, the phase path (--phase) on the same
# box, rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE of the headline (profiles/r2_*), and
# of C4 / C5 (profiles/r2_c4_*, r2_c5_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err || { tail -n 20 gpurun_out/r2_bench.err; exit 1; }
tail -n 1 gpurun_out/r2_bench.json | cut -c 1-300
timeout -k 10 300 python -u bench.py --phase --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/r2_phase.json 2> gpurun_out/r2_phase.err || { tail -n 20 gpurun_out/r2_phase.err; exit 1; }
BENCH_ARGS="--steps 50" OUT=gpurun_out/prof bash scripts/profile.sh > gpurun_out/prof.out 2>&1 || { tail -n 20 gpurun_out/prof.out; exit 1; }
python scripts/pmc_summary.py gpurun_out/prof r2 || exit $?
BENCH_ARGS="--config c4 --steps 5" OUT=gpurun_out/prof_c4 bash scripts/profile.sh > gpurun_out/prof_c4.out 2>&1 || { tail -n 20 gpurun_out/prof_c4.out; exit 1; }
python scripts/pmc_summary.py gpurun_out/prof_c4 r2_c4 || exit $?
BENCH_ARGS="--config c5 --dtype float32 --steps 8" OUT=gpurun_out/prof_c5 bash scripts/profile.sh > gpurun_out/prof_c5.out 2>&1 || { tail -n 20 gpurun_out/prof_c5.out; exit 1; }
python scripts/pmc_summary.py gpurun_out/prof_c5 r2_c5 || exit $?
cp profiles/r2_* gpurun_out/profiles/
for f in gpurun_out/prof/stats.log gpurun_out/prof_c4/stats.log gpurun_out/prof_c5/stats.log; do tail -n 1 $f | cut -c 1-400; done
echo "=== done"
