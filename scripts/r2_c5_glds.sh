#!/bin/bash
# Round 2: C5 column-blocked step, LDS-DMA kernel (DOPT_SPLIT_GLDS = D blocks in flight per wave)
# vs the register-prefetch kernel, in-process interleaved (tools/split_ab.py, results bitwise
# equal), at 4 and 3 column-block groups per worker; then the large-d tests with it forced on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_KNOB=DOPT_SPLIT_GLDS AB_VALUES=0,2,3 AB_EXACT=1 timeout -k 10 300 python -u tools/split_ab.py \
  > gpurun_out/r2_glds_g4.json 2> gpurun_out/r2_glds_g4.err || { tail -n 20 gpurun_out/r2_glds_g4.err; exit 1; }
cat gpurun_out/r2_glds_g4.json
DOPT_SPLIT_WGS=3072 AB_KNOB=DOPT_SPLIT_GLDS AB_VALUES=0,2 AB_EXACT=1 timeout -k 10 300 python -u tools/split_ab.py \
  > gpurun_out/r2_glds_g3.json 2> gpurun_out/r2_glds_g3.err || { tail -n 20 gpurun_out/r2_glds_g3.err; exit 1; }
cat gpurun_out/r2_glds_g3.json
DOPT_SPLIT_GLDS=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_large_d.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_glds_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/r2_glds_tests.log | tail -n 20
exit $rc
