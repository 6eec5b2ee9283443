#!/bin/bash
# Kernel trace of the phase path at RCCL world 1 (collectives forced) with the halo all-to-all, 512
# workers: where the ~10 us per round over the P2P-era schedule goes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
  -d gpurun_out/a2a_prof -o run -- python3 -u bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
  --workers 512 --steps 50 --warmup 3 > gpurun_out/a2a_prof.log 2>&1 || { tail -n 20 gpurun_out/a2a_prof.log; exit 1; }
tail -n 1 gpurun_out/a2a_prof.log | cut -c 1-200
ls gpurun_out/a2a_prof
