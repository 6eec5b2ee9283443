#!/bin/bash
# The driver's N = 1 command interleaved with the main leg alone (--no-secondary: nothing before the
# timed leg).  Run once with the f(x*) solve and both drop-in legs moved ahead of the timed leg (bench.py
# round-3 A/B, reverted: no difference, profiles/r3_warm_check.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/wc_full_$rep.json 2> gpurun_out/wc.err || exit $?
  printf "driver-cmd " ; tail -n 1 gpurun_out/wc_full_$rep.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['suboptimality']['final_suboptimality'])"
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 > gpurun_out/wc_cold_$rep.json 2> gpurun_out/wc.err || exit $?
  printf "cold       " ; tail -n 1 gpurun_out/wc_cold_$rep.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
done
