#!/bin/bash
# Column-block tiled shard layout (round 3): the column-blocked / row-space GPU tests, then C5 lines
# (row-space x32 twice, float32 engine, direct x32) for the per-round time and the pass's roofline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_d.py tests/test_gpu_rowspace.py tests/test_gpu_fullsize.py \
  "tests/test_gpu_distributed.py::test_column_blocked_ranks_match_single_context" -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/tiled_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/tiled_tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/tiled_tests.log | head -30; exit $rc; }
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"; local rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -n 20 "gpurun_out/$name.err"; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('ms/round %.3f  kernel %.3f ms  frac %.4f  %s' % (d['ms_per_step'], r['kernel_avg_ms'], r['frac'], r['kernel']))"
}
step t_c5 300 python -u bench.py --config c5 --steps 20 --warmup 3
step t_c5_f32 300 python -u bench.py --config c5 --dtype float32 --steps 20 --warmup 3
step t_c5_direct 300 env DOPT_ROWSPACE=0 python -u bench.py --config c5 --steps 10 --warmup 2
step t_c5_b 300 python -u bench.py --config c5 --steps 20 --warmup 3
echo "=== done"
