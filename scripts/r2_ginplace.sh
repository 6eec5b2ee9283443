#!/bin/bash
# Phase path with the gradients in place (default) vs the separate G array, interleaved on one
# box (bench.py --phase, world 1), next to the fused path; then the distributed GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B="python -u bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline"
for rep in 1 2; do
  for g in 1 0; do
    DOPT_G_INPLACE=$g timeout -k 10 300 $B --phase > gpurun_out/ph_$g.json 2> gpurun_out/ph_$g.err || { tail -n 20 gpurun_out/ph_$g.err; exit 1; }
    python - gpurun_out/ph_$g.json "phase G_INPLACE=$g" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
print(sys.argv[2], "ms/step %.4f kernel %.4f" % (d["ms_per_step"], r["kernel_avg_ms"]), "obj %.12g cons %.12g" % (d["final_objective"], d["final_consensus"]))
PY
  done
  timeout -k 10 300 $B > gpurun_out/fu.json 2> gpurun_out/fu.err || { tail -n 20 gpurun_out/fu.err; exit 1; }
  python - gpurun_out/fu.json "fused" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
print(sys.argv[2], "ms/step %.4f kernel %.4f" % (d["ms_per_step"], r["kernel_avg_ms"]), "obj %.12g cons %.12g" % (d["final_objective"], d["final_consensus"]))
PY
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/dist_tests.log 2>&1 || { tail -n 30 gpurun_out/dist_tests.log; exit 1; }
tail -n 1 gpurun_out/dist_tests.log
