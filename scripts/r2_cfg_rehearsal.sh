#!/bin/bash
# Round 2: bench.py --config c4 / c5 at N = 2 on ONE GPU (gloo transport, both ranks share
# device 0): the multi-GPU paths of the torus strips (halo) and the complete graph
# (all-reduced column sums, serial phase order) end to end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in c4 c5; do
  timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29701 bench.py --gpus 2 --backend gloo --config $cfg --steps 3 --warmup 1 \
    > gpurun_out/rehearse_$cfg.log 2>&1 || { tail -n 30 gpurun_out/rehearse_$cfg.log; exit 1; }
  tail -n 1 gpurun_out/rehearse_$cfg.log | cut -c 1-400
done
