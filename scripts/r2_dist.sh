#!/bin/bash
# Round 2: the multi-GPU code path on one GPU -- distributed GPU tests (gloo ranks sharing the
# device; RCCL at world 1 with forced collectives), bench.py --phase over RCCL (world 1), and
# the 2 / 4-rank gloo rehearsal of bench.py --gpus N (bench's default dtype).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r2_dist_tests.log 2>&1 || { grep -E "PASS|FAIL|Error" gpurun_out/r2_dist_tests.log | tail -n 30; exit 1; }
grep -E "passed|failed" gpurun_out/r2_dist_tests.log | tail -n 2
timeout -k 10 300 python -u bench.py --phase --steps 20 --warmup 3 --no-secondary > gpurun_out/r2_phase.json 2> gpurun_out/r2_phase.err \
  || { tail -n 30 gpurun_out/r2_phase.err; exit 1; }
tail -n 1 gpurun_out/r2_phase.json | cut -c 1-400
WORKERS=1024 bash scripts/dist_rehearsal.sh
