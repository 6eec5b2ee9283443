#!/bin/bash
# Round-3 closing evidence: every GPU test + smoke, the driver-shaped N = 1 line, the
# self-launched 2-rank rehearsal, the phase path at world 1 (bench --phase), C5 x32 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit $?
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"; local rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -n 20 "gpurun_out/$name.err"; exit $rc; }
  tail -n 1 "gpurun_out/$name.json" | cut -c 1-200
}
step g_bench 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
step g_phase 300 python3 bench.py --phase --no-cpu-baseline --no-secondary --steps 20 --warmup 5
step g_rehearsal2 300 python3 bench.py --gpus 2 --backend gloo --workers 512 --steps 20 --warmup 3
step g_c5 300 python3 -u bench.py --config c5 --steps 20 --warmup 3
echo "=== done"
