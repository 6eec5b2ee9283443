#!/bin/bash
# Round-6 evidence, one gpurun call for any list of steps:
#   /usr/local/graft/bin/gpurun -- 'bash scripts/r6.sh dist_tests rehearsal8'
# Every step runs from the repository root on the GPU box, writes under gpurun_out/, and stops the
# script on a failure.  The summaries judged are copied into profiles/ (named in each step's comment).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp

die() { echo "step $1 failed (rc $2)"; exit "$2"; }
json_line() {  # value, ms_per_step, kernel ms, setup / wall seconds of a bench JSON file's last line
  tail -n 1 "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], 'scaling', d['scaling'], 'setup_s', d.get('setup_s'), 'wall_s', d.get('wall_s'))"
}
bench_step() {  # bench_step <name> <timeout> <bench.py args...>  (env assignments before the call apply)
  local name=$1 t=$2; shift 2
  echo "=== $name"
  local t0=$(date +%s.%N)
  timeout -k 10 "$t" python3 bench.py "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err" \
    || { tail -n 20 "gpurun_out/$name.err"; die "$name" 1; }
  echo "command wall $(python3 -c "print(round($(date +%s.%N) - $t0, 1))") s"
  json_line "gpurun_out/$name.json"
}
tests() {  # tests <name> <pytest args...>: a failing test is listed and stops the script
  local name=$1; shift
  timeout -k 10 1000 python3 -u -m pytest -v --timeout 300 --timeout-method thread "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "FAILED|ERROR" "gpurun_out/$name.log" | head -30
  tail -n 2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || die "$name" $rc
}
rehearsal8() {  # rehearsal8 <name> <timeout> <bench.py args...>: the driver's SCALE command shape, 8 gloo ranks
  local name=$1 t=$2; shift 2
  bench_step "$name" "$t" --gpus 8 --backend gloo --steps 20 --warmup 5 "$@"
  tail -n 1 "gpurun_out/$name.json" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('value', d['value'], 'scaling', d['scaling'], 'workers_total', d['config']['workers_total'], 'per_gpu', d['config']['workers_per_gpu'])
print('per_rank', [(r['rank'], r['workers']) for r in d.get('per_rank', [])])
w = d.get('weak'); print('weak', None if w is None else (w['value'], w['n_workers_total'], w['workers_per_gpu']))
print('transport', d.get('comm', {}).get('transport'))
for k in ('alt_exchange', 'alt_transport'):
    s = d.get(k); print(k, None if s is None else (s.get('value'), s.get('ms_per_step'), s.get('exchange_beside_gradient'), s.get('transport'), s.get('final_objective_matches_value')))
print('transport_probe', d.get('transport_probe'))"
}

for step in "$@"; do
  case $step in
  full)  # every -m gpu test, smoke(), the no-flag bench line -> profiles/r6_gpu_tests.txt, r6_bench_default.json
    echo "=== pytest -m gpu"; tests r6_full_tests tests -m gpu
    echo "=== smoke"
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_smoke.log 2>&1 \
      || { tail -n 20 gpurun_out/r6_smoke.log; die smoke 1; }
    tail -n 1 gpurun_out/r6_smoke.log
    bench_step r6_full_bench 420 ;;
  driver_bench)  # the driver's shape -> profiles/r6_bench_driver.json
    bench_step r6_driver_bench 420 --gpus 1 --steps 20 --warmup 5 ;;
  dist_tests)  # the multi-process GPU tests -> profiles/r6_dist_tests.txt
    echo "=== multi-GPU tests"; tests r6_dist_tests tests/test_gpu_distributed.py tests/test_gpu_rowspace.py ;;
  comm_tests)  # the engine transport's tests (bounded setup, self exchange) -> profiles/r6_comm_tests.txt
    echo "=== transport tests"; tests r6_comm_tests tests/test_gpu_distributed.py -k "comm or transport or self_exchange or rccl" ;;
  rehearsal8)  # SCALE's command on one GPU with 8 gloo ranks: value = 4096 workers over 8 ranks, the weak leg under
    # 'weak' -> profiles/r6_rehearsal8.json
    rehearsal8 r6_rehearsal8 900 ;;
  rank_proxy)  # every rank of the 8-rank strong leg on one GPU (tools/rank_proxy.py: the real plan, the exchange
    # to itself over TRANSPORT, default rccl) beside the fused 4096-worker round -> profiles/r6_rank_proxy.txt
    for r in ${RANKS:-0 1 2 3 4 5 6 7}; do
      legs=proxy
      [ $r = 0 ] && legs=fused,proxy
      DOPT_TRANSPORT=${TRANSPORT:-rccl} timeout -k 10 300 python3 tools/rank_proxy.py --world 8 --rank $r --scaling strong \
        --legs $legs --reps 1 --steps ${STEPS:-2000} --warmup 300 > gpurun_out/r6_rp_$r.json 2> gpurun_out/r6_rp_$r.err \
        || { tail -n 20 gpurun_out/r6_rp_$r.err; die rank_proxy 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/r6_rp_$r.json').read().strip().splitlines()[-1]); p=d['plan']; [print('${TRANSPORT:-rccl}', 'strong rank', $r, g['leg'], g['workers'], 'halo', p['halo_rows_in'], 'interior', p['interior'], round(g['value']), round(g['ms_per_round'], 4), round(g['kernel_avg_ms'], 4)) for g in d['legs']]"
    done ;;
  transport_ab)  # rank 0 of the 8-rank strong leg, the engine's non-blocking RCCL communicator vs the process group's
    # all-to-all (DOPT_TRANSPORT=pg), interleaved twice, one process each -> profiles/r6_rank_proxy.txt
    for rep in 1 2; do
      for t in rccl pg; do
        DOPT_TRANSPORT=$t timeout -k 10 300 python3 tools/rank_proxy.py --world 8 --rank 0 --scaling strong --legs proxy \
          --reps 1 --steps ${STEPS:-2000} --warmup 300 > gpurun_out/r6_tab_${t}_$rep.json 2> gpurun_out/r6_tab_${t}_$rep.err \
          || { tail -n 20 gpurun_out/r6_tab_${t}_$rep.err; die transport_ab 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r6_tab_${t}_$rep.json').read().strip().splitlines()[-1]); [print('transport', '$t', 'rep', $rep, g['leg'], g['workers'], round(g['value']), round(g['ms_per_round'], 4), round(g['kernel_avg_ms'], 4)) for g in d['legs']]"
      done
    done ;;
  proxy_trace)  # kernel trace of the strong leg's rank 0 (proxy alone, WORLD ranks, default 8) -> profiles/r6_rank_proxy.txt
    W=${WORLD:-8}; D=gpurun_out/r6_pt${WORLD:+_$WORLD}
    timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- \
      python3 tools/rank_proxy.py --world $W --rank 0 --scaling strong --legs proxy --reps 1 --steps $((600 * 8 / W)) \
      --warmup 100 > $D.log 2>&1 || { tail -n 20 $D.log; die proxy_trace 1; }
    python3 tools/trace_rounds.py $D/run_kernel_trace.csv
    python3 tools/trace_window.py $D/run_kernel_trace.csv ;;
  scale_proxy)  # rank 0 of the strong leg at 2, 4 and 8 ranks (2048 / 1024 / 512 workers) and of the weak leg at 8 beside
    # the fused round of the same workers, over the engine's RCCL transport and the pull transport: the per-rank
    # efficiency the driver's 1/2/4/8-GPU line can reach before xGMI -> profiles/r6_scale_proxy.txt
    for tr in ${TRANSPORTS:-rccl ipc}; do
      for cfg in "strong 2" "strong 4" "strong 8" "weak 8"; do
        sc=${cfg% *}; w=${cfg#* }
        st=$((1000 * 8 / w)); [ $sc = weak ] && st=150
        DOPT_TRANSPORT=$tr timeout -k 10 300 python3 tools/rank_proxy.py --world $w --rank 0 --scaling $sc --legs fused,proxy --reps 1 \
          --steps $st --warmup 200 > gpurun_out/r6_sp_${tr}_$sc$w.json 2> gpurun_out/r6_sp_${tr}_$sc$w.err \
          || { tail -n 20 gpurun_out/r6_sp_${tr}_$sc$w.err; die scale_proxy 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r6_sp_${tr}_$sc$w.json').read().strip().splitlines()[-1]); p=d['plan']; [print('$tr', '$sc', 'world', $w, g['leg'], g['workers'], 'halo', p['halo_rows_in'], 'interior', p['interior'], round(g['value']), round(g['ms_per_round'], 4), round(g['kernel_avg_ms'], 4)) for g in d['legs']]; print('$tr', '$sc', 'world', $w, 'proxy / fused', [round(x, 4) for x in d['proxy_over_fused']])"
      done
    done ;;
  ipc_ab)  # the pull transport (DOPT_TRANSPORT=ipc: k_pull reads the send slots, no RCCL kernel) vs the engine's RCCL
    # transport, side stream (s1) / serial (s0): rank 0 of the strong leg at 4 / 2 / 8 ranks and of the weak leg at 8
    # (world 1, the rank's blocks pulled from its own slot), two interleaved reps; then kernel traces at 4 and 8
    # ranks -> profiles/r6_ipc_ab.txt
    for rep in 1 2; do
      for cfg in "strong 4" "strong 2" "strong 8" "weak 8"; do
        sc=${cfg% *}; w=${cfg#* }
        st=$((1000 * 8 / w)); [ $sc = weak ] && st=150
        for arm in rccl_s1 ipc_s1 ipc_s0 rccl_s0; do
          tr=${arm%_*}; sd=${arm#*_s}
          env DOPT_TRANSPORT=$tr DOPT_LAGGED_SIDE=$sd timeout -k 10 300 python3 tools/rank_proxy.py --world $w --rank 0 --scaling $sc --legs proxy \
            --reps 1 --steps $st --warmup 50 > gpurun_out/r6_ia_${sc}${w}_${arm}_$rep.json 2> gpurun_out/r6_ia_${sc}${w}_${arm}_$rep.err \
            || { tail -n 20 gpurun_out/r6_ia_${sc}${w}_${arm}_$rep.err; die ipc_ab 1; }
          python3 -c "import json; d=json.loads(open('gpurun_out/r6_ia_${sc}${w}_${arm}_$rep.json').read().strip().splitlines()[-1]); [print('$sc', 'world', $w, '$arm', 'rep', $rep, g['workers'], round(g['value']), round(g['ms_per_round'], 4), round(g['kernel_avg_ms'], 4)) for g in d['legs']]"
        done
      done
    done
    for w in 4 8; do
      D=gpurun_out/r6_ia_tr$w
      DOPT_TRANSPORT=ipc timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- \
        python3 tools/rank_proxy.py --world $w --rank 0 --scaling strong --legs proxy --reps 1 --steps $((300 * 8 / w)) \
        --warmup 100 > $D.log 2>&1 || { tail -n 20 $D.log; die ipc_ab 1; }
      python3 tools/trace_rounds.py $D/run_kernel_trace.csv
      python3 tools/trace_window.py $D/run_kernel_trace.csv
    done ;;
  pull_tests)  # the pull transport's multi-process tests (2-8 processes on the one GPU) -> profiles/r6_pull_tests.txt
    echo "=== pull transport tests"; tests r6_pull_tests tests/test_gpu_distributed.py -k pull ;;
  xq_probe)  # what a cross-stream hand-off costs (tools/xq_probe.hip, built in-tree beforehand) -> profiles/r6_xq_probe.txt
    timeout -k 10 120 tools/xq_probe ${REPS:-50} > gpurun_out/r6_xq_probe.txt 2>&1 || { cat gpurun_out/r6_xq_probe.txt; die xq_probe 1; }
    cat gpurun_out/r6_xq_probe.txt ;;
  c3_profile)  # the driver's shape under rocprofv3: kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes
    # -> profiles/r6_kernel_stats.csv, r6_pmc.json (scripts/pmc_summary.py)
    OUT=gpurun_out/prof_r6 PSTEPS=20 PWARM=5 bash scripts/profile.sh || die c3_profile 1 ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
