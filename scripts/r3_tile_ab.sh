#!/bin/bash
# Same-box A/B of the shard layout of column-blocked contexts: the tiled build (libdopt.so) vs the
# row-major build of the commit before it (tools/ab/libdopt_rowmajor.so, DOPT_LIB), C5 row-space
# x32 (the C5 default) and the direct x32 step, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
RM="$PWD/tools/ab/libdopt_rowmajor.so"
one() {  # one <name> <lib or ''> <args...>
  local name=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export DOPT_LIB="$lib"; else unset DOPT_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err" \
    || { echo "$name failed"; tail -n 20 "gpurun_out/$name.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-16s ms/round %.3f  kernel %.3f ms  frac %.4f' % ('$name', d['ms_per_step'], r['kernel_avg_ms'], r['frac']))"
}
for k in 1 2; do
  one ab_tiled_$k "" --config c5 --steps 20 --warmup 3
  one ab_rowmaj_$k "$RM" --config c5 --steps 20 --warmup 3
done
export DOPT_ROWSPACE=0
one ab_tiled_direct "" --config c5 --steps 10 --warmup 2
one ab_rowmaj_direct "$RM" --config c5 --steps 10 --warmup 2
echo "=== done"
