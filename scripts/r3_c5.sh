#!/bin/bash
# Round-3 C5 evidence: row-space x32 line (tiled rows, 2 / 8 pass), float32 line, kernel stats +
# FETCH / WRITE passes -> profiles/r3_c5x32_*, then the C3 phase path at RCCL world 1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"; local rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -n 20 "gpurun_out/$name.err"; exit $rc; }
  tail -n 1 "gpurun_out/$name.json" | cut -c 1-240
}
step f_c5 300 python3 -u bench.py --config c5 --steps 20 --warmup 3
step f_c5_f32 300 python3 -u bench.py --config c5 --dtype float32 --steps 20 --warmup 3
BENCH_ARGS="--config c5" PSTEPS=8 OUT=gpurun_out/prof_c5f bash scripts/profile.sh > gpurun_out/prof_c5f.out 2>&1 \
  || { tail -n 20 gpurun_out/prof_c5f.out; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/prof_c5f r3_c5x32 || exit $?
echo "=== phase trace"
DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_phase3 \
  -o run -- python3 -u bench.py --no-cpu-baseline --phase --steps 20 --warmup 3 > gpurun_out/prof_phase3.log 2>&1 \
  || { tail -n 20 gpurun_out/prof_phase3.log; exit 1; }
cp gpurun_out/prof_phase3/run_kernel_stats.csv profiles/r3_phase_kernel_stats.csv
tail -n 1 gpurun_out/prof_phase3.log | cut -c 1-240
cp profiles/r3_* gpurun_out/profiles/
echo "=== done"
