#!/bin/bash
# Round 2: C5 column-blocked step A/B (tools/split_ab.py, in-process, interleaved), then the
# large-d parity tests with the candidate kernel forced on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
KNOB=${KNOB:-DOPT_SPLIT_COLWAVE}
AB_KNOB=$KNOB AB_VALUES=0,1 timeout -k 10 300 python -u tools/split_ab.py > gpurun_out/r2_c5_ab.json 2> gpurun_out/r2_c5_ab.err || { tail -n 20 gpurun_out/r2_c5_ab.err; exit 1; }
cat gpurun_out/r2_c5_ab.json; tail -n 4 gpurun_out/r2_c5_ab.err
env $KNOB=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_large_d.py tests/test_gpu_fullsize.py -v --timeout 300 --timeout-method thread > gpurun_out/r2_large_ab.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/r2_large_ab.log | tail -n 14
exit $rc
