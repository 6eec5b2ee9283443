#!/bin/bash
# Kernel traces of the serial and the pipelined schedule (short bench runs) + gap analysis.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in 0 1; do
  DOPT_PIPELINE=$p timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace$p -o run -- \
    python -u bench.py --no-cpu-baseline --steps 12 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/trace$p.log 2>&1 || exit $?
  echo "=== DOPT_PIPELINE=$p"
  python tools/trace_gaps.py gpurun_out/trace$p 8
done
