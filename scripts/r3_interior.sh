#!/bin/bash
# Interior workers stepped in the phase path's gradient kernel: the multi-rank GPU tests (bitwise
# one context), the C3 parity tests, then bench --phase at world 1 and the 2-rank rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_scale_parity.py tests/test_gpu_rowspace.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/int_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/int_tests.log; [ $rc -eq 0 ] || exit $rc
for s in phase rehearsal2; do
  if [ $s = phase ]; then a="--phase --no-cpu-baseline --no-secondary --steps 20 --warmup 5"; else a="--gpus 2 --backend gloo --workers 512 --steps 20 --warmup 3"; fi
  timeout -k 10 300 python3 bench.py $a > gpurun_out/int_$s.json 2> gpurun_out/int_$s.err || { tail -n 20 gpurun_out/int_$s.err; exit 1; }
  tail -n 1 gpurun_out/int_$s.json | cut -c 1-200
done
