#!/bin/bash
# Strong-scaling proxy on one GPU: the per-rank shapes of N = 4096 over 1/2/4/8 ranks (4096 / 2048 /
# 1024 / 512 workers) through the fused single-context round and through the multi-GPU phase path at
# RCCL world 1 (collectives forced on), plus a kernel trace of the 512-worker phase path, so the
# schedule's fixed per-round cost (launches, collectives) shows beside the shrinking round kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"; local rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -n 20 "gpurun_out/$name.err"; exit $rc; }
  tail -n 1 "gpurun_out/$name.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
}
for w in 4096 2048 1024 512; do
  step sp_fused_$w 200 python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --workers $w --steps 200 --warmup 5
  DOPT_FORCE_COLLECTIVES=1 step sp_phase_$w 200 python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
    --workers $w --steps 200 --warmup 5
done
echo "=== phase trace 512"
DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_prof \
  -o run -- python3 -u bench.py --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 50 --warmup 3 \
  > gpurun_out/sp_prof.log 2>&1 || { tail -n 20 gpurun_out/sp_prof.log; exit 1; }
echo "=== done"
