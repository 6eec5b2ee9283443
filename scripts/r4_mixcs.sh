#!/bin/bash
# Round 4: k_mixcs with every load of a wave's workers issued before use and the ranks' sums
# staged through LDS -- the multi-GPU tests, the 512-worker traces, the strong-leg proxy rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
echo "=== multi-GPU tests"
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py \
  tests/test_gpu_rowspace.py -k "ranks or strong or lagged or pipelined or flag or rccl" > gpurun_out/r4_mx_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/r4_mx_tests.log | head -20
tail -n 2 gpurun_out/r4_mx_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/r4_strong_trace.sh || exit $?
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"; local rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -n 20 "gpurun_out/$name.err"; exit $rc; }
  tail -n 1 "gpurun_out/$name.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
}
for w in 4096 512; do
  step r4mx_fused_$w 200 python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --workers $w --steps 100 --warmup 5
  DOPT_FORCE_COLLECTIVES=1 step r4mx_phase_$w 200 python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
    --workers $w --steps 100 --warmup 5
  step r4mx_phase1_$w 200 python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
    --workers $w --steps 100 --warmup 5
done
echo "=== done"
