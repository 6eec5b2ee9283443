#!/bin/bash
# Halo exchange as one RCCL all_to_all_single: the multi-rank / RCCL-world-1 GPU tests, then the
# phase path at RCCL world 1 (collectives forced: a zero-count all-to-all every round) at the strong
# leg's 512 and the weak leg's 4096 workers per rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/a2a_tests.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/a2a_tests.log | tail -n 3; [ $rc -eq 0 ] || exit $rc
for w in 512 4096; do
  echo "=== phase $w"
  DOPT_FORCE_COLLECTIVES=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
    --workers $w --steps 200 --warmup 5 > gpurun_out/a2a_phase_$w.json 2> gpurun_out/a2a_phase_$w.err || exit $?
  tail -n 1 gpurun_out/a2a_phase_$w.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
done
echo "=== rehearsal 2 ranks"
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --workers 512 --steps 20 --warmup 3 > gpurun_out/a2a_reh2.json \
  2> gpurun_out/a2a_reh2.err || { tail -n 20 gpurun_out/a2a_reh2.err; exit 1; }
tail -n 1 gpurun_out/a2a_reh2.json | cut -c 1-300
