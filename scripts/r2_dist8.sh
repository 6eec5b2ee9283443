#!/bin/bash
# Multi-rank rehearsals on ONE GPU (gloo transport, ranks share device 0): bench.py's C3 at
# N = 8 at full size (4096 workers per rank: the driver's 8-GPU command shape), then C5 at N = 2
# through the row-space rounds across ranks.  RCCL with peers runs only on a multi-GPU node.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29731 bench.py --gpus 8 --backend gloo --steps 4 --warmup 1 > gpurun_out/dist8.log 2>&1 \
  || { tail -n 30 gpurun_out/dist8.log; exit 1; }
grep -E "^\{" gpurun_out/dist8.log | tail -n 1 | cut -c 1-700
grep -E "comm:|rank 0" gpurun_out/dist8.log | head -n 5 | cut -c 1-400
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29741 bench.py --gpus 2 --backend gloo --config c5 --dtype float32 --steps 3 --warmup 1 \
  > gpurun_out/dist2_c5.log 2>&1 || { tail -n 30 gpurun_out/dist2_c5.log; exit 1; }
grep -E "^\{" gpurun_out/dist2_c5.log | tail -n 1 | cut -c 1-900
echo "=== done"
