#!/bin/bash
# Multi-rank rehearsal on ONE GPU (gloo transport, ranks share device 0): 2 and 4 ranks,
# spectral partition and contiguous ranges.  The RCCL path runs only on a multi-GPU node.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
port=29611
for np_ in 2 4; do
  for part in spectral ranges; do
    port=$((port + 1))
    timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $np_ --backend gloo --workers ${WORKERS:-512} --steps 4 --warmup 1 \
      --partition $part > gpurun_out/dist${np_}_$part.log 2>&1 || { tail -n 20 gpurun_out/dist${np_}_$part.log; exit 1; }
    python - "gpurun_out/dist${np_}_$part.log" "n=$np_ $part" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value %.4g" % d["value"], "halo rows/gpu", d["config"]["halo_rows_per_gpu"],
      "obj %.9g cons %.6g" % (d["final_objective"], d["final_consensus"]))
PY
  done
done
