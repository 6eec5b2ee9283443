#!/bin/bash
# Setup kernels: MFMA Gram matrices + float Box-Muller generation -- the tests that touch them,
# then kernel stats of a C5 and a C3 bench run (k_rs_gram / k_generate durations).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rowspace.py tests/test_gpu_large_d.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gg_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/gg_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in c5 c3; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gg_$cfg -o run -- \
    python3 -u bench.py --config $cfg --no-cpu-baseline --no-secondary --steps 10 --warmup 2 > gpurun_out/gg_$cfg.log 2>&1 \
    || { tail -n 20 gpurun_out/gg_$cfg.log; exit 1; }
  python3 - "$cfg" <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/gg_{sys.argv[1]}/run_kernel_stats.csv")):
    if any(k in r["Name"] for k in ("gram", "generate", "k_round<", "rs_pass")):
        print(sys.argv[1], r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
done
