#!/bin/bash
# C5 in float64 (the reference's precision, 137 GB of shards): row-space vs direct rounds, then
# the default C3 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5f64rs.json \
  2> gpurun_out/c5f64rs.err || { tail -n 20 gpurun_out/c5f64rs.err; exit 1; }
tail -n 1 gpurun_out/c5f64rs.json | cut -c 1-200
DOPT_ROWSPACE=0 timeout -k 10 400 python -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/c5f64direct.json 2> gpurun_out/c5f64direct.err || { tail -n 20 gpurun_out/c5f64direct.err; exit 1; }
tail -n 1 gpurun_out/c5f64direct.json | cut -c 1-200
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/c3.json 2> gpurun_out/c3.err \
  || { tail -n 20 gpurun_out/c3.err; exit 1; }
tail -n 1 gpurun_out/c3.json | cut -c 1-200
