#!/bin/bash
# Does the 20-round driver window see a clock ramp?  C3 main leg only, interleaved: --steps 20 with
# --warmup 5 / 100, and --steps 200 --warmup 5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do for cfg in "20 5" "20 100" "200 5"; do set -- $cfg
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary --steps $1 --warmup $2 > gpurun_out/w_$1_$2.json 2> gpurun_out/w.err || exit $?
  printf "steps=%s warmup=%s " $1 $2; tail -n 1 gpurun_out/w_$1_$2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
done; done
