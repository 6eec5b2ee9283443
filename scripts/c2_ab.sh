#!/bin/bash
# Small-config round time (tools/c2_breakdown.py), quadratic and logistic, with the
# few-workers wide k_round on (default) and off (DOPT_KR_FEW_WIDE=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for prob in quadratic logistic; do
  for wide in 1 0; do
    echo "=== $prob wide=$wide"
    C2_PROBLEM=$prob DOPT_KR_FEW_WIDE=$wide timeout -k 10 200 python -u tools/c2_breakdown.py > gpurun_out/c2_${prob}_$wide.log 2>&1 || exit $?
    grep "us/round" gpurun_out/c2_${prob}_$wide.log
  done
done
