#!/bin/bash
# Distributed GPU tests, then the phase path on one GPU: serial vs lagged schedule
# (world 1: no transport, so this isolates the kernel sequence), then a 2-rank gloo run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TESTS=${TESTS:-"tests/test_gpu_distributed.py tests/test_gpu_parity.py"}
if [ "$TESTS" != none ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
  rc=$?; tail -n 12 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in a b; do
  for l in 0 1; do
    DOPT_LAGGED=$l timeout -k 10 300 python -u bench.py --no-cpu-baseline --phase ${BENCH_ARGS:-} > gpurun_out/ph$l$rep.log 2>&1 || exit $?
    python - "gpurun_out/ph$l$rep.log" "lagged=$l rep=$rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value %.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"], "kernel", d["roofline"]["kernel_avg_ms"],
      "obj %.9g cons %.6g" % (d["final_objective"], d["final_consensus"]))
PY
  done
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/fused.log 2>&1 || exit $?
tail -n 1 gpurun_out/fused.log | cut -c 1-400
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --backend gloo --workers 1024 --steps 5 --warmup 1 > gpurun_out/dist2.log 2>&1 || exit $?
tail -n 1 gpurun_out/dist2.log | cut -c 1-300
