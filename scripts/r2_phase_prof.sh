#!/bin/bash
# The multi-GPU phase path on one GPU (bench.py --phase, RCCL world 1): bench line next to the
# fused path's on the same box, and rocprofv3 kernel stats of the phase run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_phase
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/fused.json \
  2> gpurun_out/fused.err || { tail -n 20 gpurun_out/fused.err; exit 1; }
timeout -k 10 300 python -u bench.py --phase --steps 50 --warmup 5 --no-secondary --no-cpu-baseline \
  > gpurun_out/phase.json 2> gpurun_out/phase.err || { tail -n 20 gpurun_out/phase.err; exit 1; }
for f in fused phase; do tail -n 1 gpurun_out/$f.json | cut -c 1-200; done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_phase -o run -- \
  python -u bench.py --phase --steps 50 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/prof_phase.log 2>&1 \
  || { tail -n 20 gpurun_out/prof_phase.log; exit 1; }
echo "=== done"
