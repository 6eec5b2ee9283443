#!/bin/bash
# Round 3 evidence for profiles/: C3 kernel stats + FETCH_SIZE / WRITE_SIZE (r3_*), the C5 direct
# column-blocked round over float32 rows at float64 arithmetic (k_split_step<double, float>,
# DOPT_ROWSPACE=0: r3_c5x32direct_*), and C5 through the multi-GPU row-space schedule at RCCL world 1
# (collectives forced) with the pass in 1 and 4 column chunks next to the single-context round.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles
export PYTHONUNBUFFERED=1
step() {  # step <name> <timeout> <cmd...>: one GPU step, its own limit, stop at the first failure
  local name=$1 t=$2; shift 2
  echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"; local rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -n 20 "gpurun_out/$name.err"; exit $rc; }
  tail -n 1 "gpurun_out/$name.json" | cut -c 1-300
}
OUT=gpurun_out/prof_r3 bash scripts/profile.sh > gpurun_out/prof_r3.out 2>&1 || { tail -n 20 gpurun_out/prof_r3.out; exit 1; }
python scripts/pmc_summary.py gpurun_out/prof_r3 r3 || exit $?
step c5x32_direct 300 env DOPT_ROWSPACE=0 python -u bench.py --config c5 --steps 10 --warmup 2
DOPT_ROWSPACE=0 BENCH_ARGS="--config c5" PSTEPS=5 OUT=gpurun_out/prof_c5d bash scripts/profile.sh > gpurun_out/prof_c5d.out 2>&1 \
  || { tail -n 20 gpurun_out/prof_c5d.out; exit 1; }
python scripts/pmc_summary.py gpurun_out/prof_c5d r3_c5x32direct || exit $?
step c5_single 300 python -u bench.py --config c5 --steps 20 --warmup 3
step c5_phase_k1 300 env DOPT_FORCE_COLLECTIVES=1 python -u bench.py --config c5 --phase --rs-chunks 1 --steps 20 --warmup 3
step c5_phase_k4 300 env DOPT_FORCE_COLLECTIVES=1 python -u bench.py --config c5 --phase --rs-chunks 4 --steps 20 --warmup 3
step c5_single_b 300 python -u bench.py --config c5 --steps 20 --warmup 3
cp profiles/r3_* gpurun_out/profiles/
echo "=== done"
