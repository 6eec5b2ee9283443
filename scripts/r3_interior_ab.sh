#!/bin/bash
# Same box, alternated: the fused N = 1 line, the phase path at world 1 with the interior workers
# stepped in the gradient kernel (default) and without (DOPT_PHASE_INTERIOR=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
A="--no-cpu-baseline --no-secondary --steps 40 --warmup 10"
for rep in 1 2; do
  for v in fused int1 int0; do
    case $v in
      fused) env_=""; extra="";;
      int1) env_="DOPT_PHASE_INTERIOR=1"; extra="--phase";;
      int0) env_="DOPT_PHASE_INTERIOR=0"; extra="--phase";;
    esac
    env $env_ timeout -k 10 300 python3 bench.py $A $extra > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -n 20 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$rep $v', round(d['ms_per_step'],4), round(d['roofline']['kernel_avg_ms'],4))"
  done
done
