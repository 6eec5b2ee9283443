#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Stops at the first crash-type exit (abort/segv/timeout); ordinary test failures continue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" ; date +%T
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc($name)=$rc"; tail -n 25 "gpurun_out/$name.log"
  case $rc in 0|1|5) return 0 ;; *) echo "STOP after $name (rc=$rc)"; exit $rc ;; esac
}
STEPS=${STEPS:-"smoke tests bench prof"}
for s in $STEPS; do
  case $s in
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ;;
    bench) step bench 600 python -u bench.py ${BENCH_ARGS:-} ;;
    dist2) step dist2 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --workers 1024 --steps 5 --warmup 1 ;;
    probe) step probe 120 ./tools/bw_probe ;;
    variants) step variants 600 python -u tools/kr_variants.py ;;
    splitab) step splitab 600 python -u tools/split_ab.py ;;
    phase1) step phase1 600 python -u bench.py --phase --no-cpu-baseline ;;
    c5)    step c5 600 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline ;;
    c4)    step c4 900 python -u bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline ;;
    mainpy) step mainpy 600 bash -c 'cd distributed-optimization_amd && MPLBACKEND=Agg python -u -c "import time, runpy; t=time.time(); import matplotlib; matplotlib.use(\"Agg\"); runpy.run_path(\"main.py\", run_name=\"__main__\"); print(\"main.py wall %.1f s\" % (time.time()-t))"' ;;
    prof)  (cd /tmp && export TMPDIR=/tmp) ; step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} ;;
  esac
done
echo "=== done"
