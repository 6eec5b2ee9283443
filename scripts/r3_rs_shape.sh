#!/bin/bash
# Row-space pass shapes on the tiled layout (A/B build tools/ab/libdopt_ab.so: DOPT_RS_CB / _NBUF),
# C5 at float64 arithmetic over float32 rows, alternated twice on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
AB="$PWD/tools/ab/libdopt_ab.so"
one() {  # one <name> <cb> <nbuf>
  local name=$1
  DOPT_LIB="$AB" DOPT_RS_CB=$2 DOPT_RS_NBUF=$3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --config c5 \
    --steps 20 --warmup 3 > "gpurun_out/$name.json" 2> "gpurun_out/$name.err" \
    || { echo "$name failed"; tail -n 20 "gpurun_out/$name.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-12s ms/round %.3f  kernel %.3f ms  frac %.4f %s' % ('$name', d['ms_per_step'], r['kernel_avg_ms'], r['frac'], r['kernel']))"
}
for k in 1 2; do
  one s26_$k 2 6
  one s28w_$k 2 8
  one s24w_$k 2 4
  one s18w_$k 1 8
  one s116w_$k 1 16
done
echo "=== done"
