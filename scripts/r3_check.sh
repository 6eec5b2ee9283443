#!/bin/bash
# Round 3 first GPU check: all GPU tests + smoke, the self-launched 2-rank rehearsal (gloo, both
# ranks on this one GPU), then the driver-shaped N = 1 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_tests.sh || exit $?
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --workers 512 --steps 20 --warmup 3 \
  > gpurun_out/r3_rehearsal2.json 2> gpurun_out/r3_rehearsal2.log || { echo "rehearsal rc=$?"; tail -20 gpurun_out/r3_rehearsal2.log; exit 1; }
cut -c1-400 gpurun_out/r3_rehearsal2.json
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.log || { echo "bench rc=$?"; tail -20 gpurun_out/r3_bench.log; exit 1; }
cut -c1-300 gpurun_out/r3_bench.json
