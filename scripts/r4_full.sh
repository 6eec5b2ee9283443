#!/bin/bash
# Round 4: the driver's round-end GPU checks on one box -- every `-m gpu` test (no -x: all failures
# listed), then smoke() and the driver-shaped bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "=== pytest -m gpu"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r4_full_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/r4_full_tests.log | head -30
tail -n 3 gpurun_out/r4_full_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "=== smoke"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 \
  || { tail -n 20 gpurun_out/r4_smoke.log; exit 1; }
tail -n 2 gpurun_out/r4_smoke.log
echo "=== bench (driver shape)"
timeout -k 10 420 python3 bench.py > gpurun_out/r4_full_bench.json 2> gpurun_out/r4_full_bench.err \
  || { tail -n 30 gpurun_out/r4_full_bench.err; exit 1; }
tail -n 1 gpurun_out/r4_full_bench.json | cut -c 1-300
exit $rc
