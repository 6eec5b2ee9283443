#!/bin/bash
# Kernel trace of a short bench run + the round-kernel gap analysis (tools/trace_gaps.py).
# ENVS="A=1 A=0" runs one trace per setting (A/B of runtime knobs such as DOPT_BIP).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
k=0
for e in ${ENVS:-NONE=0}; do
  env $e timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace$k -o run -- \
    python -u bench.py --no-cpu-baseline --steps 12 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/trace$k.log 2>&1 || exit $?
  echo "=== $e"
  python tools/trace_gaps.py gpurun_out/trace$k 8
  k=$((k + 1))
done
