#!/bin/bash
# Round-5 evidence, one gpurun call for any list of steps:
#   /usr/local/graft/bin/gpurun -- 'bash scripts/r5.sh dist_tests rehearsal8_c3full'
# Every step runs from the repository root on the GPU box, writes under gpurun_out/, and stops the
# script on a failure (a GPU test failure lists the failures and goes on to the next step).  The
# summaries judged are copied into profiles/ (named in each step's comment).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
AB=$PWD/distributed-optimization_amd/libdopt_ab.so

die() { echo "step $1 failed (rc $2)"; exit "$2"; }
json_line() {  # value, ms_per_step, kernel ms, setup / wall seconds of a bench JSON file's last line
  tail -n 1 "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], 'setup_s', d.get('setup_s'), 'wall_s', d.get('wall_s'))"
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
tests() {  # tests <name> <pytest args...>
  local name=$1; shift
  timeout -k 10 1000 python3 -u -m pytest -v --timeout 300 --timeout-method thread "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "FAILED|ERROR" "gpurun_out/$name.log" | head -30
  tail -n 2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || die "$name" $rc
}
rehearsal8() {  # rehearsal8 <name> <timeout> <bench.py args...>: the driver's SCALE command shape, 8 gloo ranks
  local name=$1 t=$2; shift 2
  bench_step "$name" "$t" --gpus 8 --backend gloo --steps 20 --warmup 5 "$@"
  tail -n 1 "gpurun_out/$name.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('comm', d.get('comm')); print('per_rank', [(r['rank'], r['workers']) for r in d.get('per_rank', [])]); s=d.get('strong'); print('strong', None if s is None else (s['value'], s['n_workers_total'], [(r['workers'], r['halo_rows_in'], r['peers']) for r in s['per_rank']])); print('transport_probe', d.get('transport_probe')); w=d.get('weak_serial_exchange'); print('weak_serial_exchange', None if w is None else (w['value'], w['ms_per_step'], w['side_stream']), 'weak', d['value'], d['ms_per_step'])"
}

for step in "$@"; do
  case $step in
  full)  # every -m gpu test, smoke(), the no-flag bench line -> profiles/r5_gpu_tests.txt, r5_bench_default.json
    echo "=== pytest -m gpu"; tests r5_full_tests tests -m gpu
    echo "=== smoke"
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1 \
      || { tail -n 20 gpurun_out/r5_smoke.log; die smoke 1; }
    bench_step r5_full_bench 420 ;;
  driver_bench)  # the driver's shape -> profiles/r5_bench_a.json
    bench_step r5_base_bench 420 --gpus 1 --steps 20 --warmup 5 ;;
  dist_tests)  # the multi-GPU and row-space GPU tests (torus strips, self exchange, world 8) -> profiles/r5_dist_tests.txt
    echo "=== multi-GPU tests"; tests r5_dist_tests tests/test_gpu_distributed.py tests/test_gpu_rowspace.py ;;
  rehearsal8_c3full)  # SCALE at its real weak size: 8 ranks x 4096 workers + the strong leg -> profiles/r5_rehearsal8_c3full.json
    rehearsal8 r5_rehearsal8_c3full 900 ;;
  rehearsal8_c4)  # C4 over 8 ranks (65536 workers, 256 x 256 torus, strips of 32 rows) -> profiles/r5_rehearsal8_c4.json
    rehearsal8 r5_rehearsal8_c4 900 --config c4 ;;
  rehearsal8_c5)  # C5 over 8 ranks (1024 workers, d = 2^20, complete graph) -> profiles/r5_rehearsal8_c5.json
    rehearsal8 r5_rehearsal8_c5 900 --config c5 ;;
  c3_profile)  # the driver's shape (--steps 20 --warmup 5) under rocprofv3: kernel trace + stats, FETCH_SIZE, WRITE_SIZE
    # passes, each printing its bench line -> profiles/r5_kernel_stats.csv, r5_pmc.json (scripts/pmc_summary.py)
    OUT=gpurun_out/prof_r5 PSTEPS=20 PWARM=5 bash scripts/profile.sh || die c3_profile 1 ;;
  host_probe)  # host time per round at 512 workers, RCCL world 1 forced, side stream on / off, launch_mixcs's HIP calls
    # timed (A/B library, DOPT_HOST_TIMING) -> profiles/r5_host_probe.txt
    for side in 1 0; do
      echo "=== host probe, DOPT_LAGGED_SIDE=$side"
      DOPT_LIB=$AB DOPT_HOST_TIMING=1 DOPT_LAGGED_SIDE=$side DOPT_FORCE_COLLECTIVES=1 timeout -k 10 200 \
        python3 tools/host_round_probe.py > gpurun_out/r5_host_probe_s$side.json 2> gpurun_out/r5_host_probe_s$side.err \
        || { tail -n 20 gpurun_out/r5_host_probe_s$side.err; die host_probe 1; }
      cat gpurun_out/r5_host_probe_s$side.json; grep "launch_mixcs host" gpurun_out/r5_host_probe_s$side.err || true
    done ;;
  strong_trace)  # kernel traces of the phase path at 512 workers, RCCL world 1 forced (self block) / skipped
    # -> profiles/r5_strong_trace.txt
    B="bench.py --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 50 --warmup 5"
    for f in 1 0; do
      echo "=== trace, DOPT_FORCE_COLLECTIVES=$f"
      DOPT_FORCE_COLLECTIVES=$f timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/r5_st_f$f -o run -- python3 $B > gpurun_out/r5_st_f$f.log 2>&1 || die strong_trace 1
      python3 tools/trace_rounds.py gpurun_out/r5_st_f$f/run_kernel_trace.csv
    done ;;
  a2a_trace)  # the lagged exchange on the current (side) stream, asyncOp=False (DOPT_A2A_STREAM=current), 512 workers,
    # RCCL world 1 forced: kernel trace + proxy line -> profiles/r5_a2a_current.txt
    B="bench.py --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 50 --warmup 5"
    echo "=== trace, DOPT_A2A_STREAM=current"
    DOPT_A2A_STREAM=current DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/r5_st_cur -o run -- python3 $B > gpurun_out/r5_st_cur.log 2>&1 || die a2a_trace 1
    python3 tools/trace_rounds.py gpurun_out/r5_st_cur/run_kernel_trace.csv
    python3 tools/trace_window.py gpurun_out/r5_st_cur/run_kernel_trace.csv
    DOPT_A2A_STREAM=current DOPT_FORCE_COLLECTIVES=1 bench_step r5sp_phase_512_cur 200 --no-cpu-baseline --no-secondary \
      --scaling weak --phase --workers 512 --steps 100 --warmup 5
    DOPT_FORCE_COLLECTIVES=1 bench_step r5sp_phase_512_b 200 --no-cpu-baseline --no-secondary --scaling weak --phase \
      --workers 512 --steps 100 --warmup 5 ;;
  ev_ab)  # the side stream's hand-off with a device-scope release (DOPT_SIDE_EV=dev), the exchange on the current
    # stream (DOPT_A2A_STREAM=current), both; the profiling events (DOPT_PROF_EV=dev), A/B library, interleaved twice
    # -> profiles/r5_ev_ab.txt
    for rep in 1 2; do
      for v in "sys nccl" "dev nccl" "sys current" "dev current"; do
        ev=${v%% *}; st=${v##* }
        DOPT_LIB=$AB DOPT_SIDE_EV=$ev DOPT_A2A_STREAM=$st DOPT_FORCE_COLLECTIVES=1 bench_step r5ev_${ev}_${st}_$rep 200 \
          --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 100 --warmup 5
      done
      for pe in sys dev; do
        DOPT_LIB=$AB DOPT_PROF_EV=$pe bench_step r5pe_${pe}_$rep 200 --no-cpu-baseline --no-secondary --steps 20 --warmup 5
      done
    done
    for v in dev_nccl dev_current; do
      echo "=== trace $v"
      DOPT_LIB=$AB DOPT_SIDE_EV=${v%_*} DOPT_A2A_STREAM=${v#*_} DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 150 rocprofv3 \
        --kernel-trace --output-format csv -d gpurun_out/r5_st_$v -o run -- python3 bench.py --no-cpu-baseline \
        --no-secondary --scaling weak --phase --workers 512 --steps 50 --warmup 5 > gpurun_out/r5_st_$v.log 2>&1 \
        || die ev_ab 1
      python3 tools/trace_rounds.py gpurun_out/r5_st_$v/run_kernel_trace.csv
      python3 tools/trace_window.py gpurun_out/r5_st_$v/run_kernel_trace.csv
    done ;;
  sync_ab)  # the lagged schedule's stream hand-offs by events (default) vs stream memory operations
    # (DOPT_LAGGED_SYNC=value), 512 and 4096 workers, RCCL world 1 forced, interleaved twice; a trace and the host
    # probe of the value mode -> profiles/r5_sync_ab.txt
    for rep in 1 2; do
      for w in 512 4096; do
        for sy in event value; do
          DOPT_LAGGED_SYNC=$sy DOPT_FORCE_COLLECTIVES=1 bench_step r5sy_${sy}_${w}_$rep 200 --no-cpu-baseline \
            --no-secondary --scaling weak --phase --workers $w --steps 100 --warmup 5
        done
      done
    done
    echo "=== trace, value sync"
    DOPT_LAGGED_SYNC=value DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv \
      -d gpurun_out/r5_st_value -o run -- python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
      --workers 512 --steps 50 --warmup 5 > gpurun_out/r5_st_value.log 2>&1 || die sync_ab 1
    python3 tools/trace_rounds.py gpurun_out/r5_st_value/run_kernel_trace.csv
    python3 tools/trace_window.py gpurun_out/r5_st_value/run_kernel_trace.csv
    echo "=== host probe, value sync"
    DOPT_LIB=$AB DOPT_HOST_TIMING=1 DOPT_LAGGED_SYNC=value DOPT_FORCE_COLLECTIVES=1 timeout -k 10 200 \
      python3 tools/host_round_probe.py > gpurun_out/r5_host_probe_value.json 2> gpurun_out/r5_host_probe_value.err \
      || { tail -n 20 gpurun_out/r5_host_probe_value.err; die sync_ab 1; }
    cat gpurun_out/r5_host_probe_value.json; grep "launch_mixcs host" gpurun_out/r5_host_probe_value.err || true ;;
  cpwait_ab)  # value sync with the stream waits on the command processor (GPU_STREAMOPS_CP_WAIT=1) vs events, 512
    # workers, forced, interleaved twice; trace + host probe of the CP-wait form -> profiles/r5_sync_ab.txt
    for rep in 1 2; do
      DOPT_FORCE_COLLECTIVES=1 bench_step r5cp_event_$rep 200 --no-cpu-baseline --no-secondary --scaling weak --phase \
        --workers 512 --steps 100 --warmup 5
      GPU_STREAMOPS_CP_WAIT=1 DOPT_LAGGED_SYNC=value DOPT_FORCE_COLLECTIVES=1 bench_step r5cp_value_$rep 200 \
        --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 100 --warmup 5
    done
    echo "=== trace, value sync, CP waits"
    GPU_STREAMOPS_CP_WAIT=1 DOPT_LAGGED_SYNC=value DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 150 rocprofv3 --kernel-trace \
      --output-format csv -d gpurun_out/r5_st_cp -o run -- python3 bench.py --no-cpu-baseline --no-secondary \
      --scaling weak --phase --workers 512 --steps 50 --warmup 5 > gpurun_out/r5_st_cp.log 2>&1 || die cpwait_ab 1
    python3 tools/trace_rounds.py gpurun_out/r5_st_cp/run_kernel_trace.csv
    python3 tools/trace_window.py gpurun_out/r5_st_cp/run_kernel_trace.csv
    GPU_STREAMOPS_CP_WAIT=1 DOPT_LAGGED_SYNC=value DOPT_FORCE_COLLECTIVES=1 timeout -k 10 200 \
      python3 tools/host_round_probe.py > gpurun_out/r5_host_probe_cp.json 2> gpurun_out/r5_host_probe_cp.err \
      || { tail -n 20 gpurun_out/r5_host_probe_cp.err; die cpwait_ab 1; }
    cat gpurun_out/r5_host_probe_cp.json ;;
  sig_ab)  # event vs signal hand-off (k_mixcs's last workgroup released a value the side stream waited for; the
    # signal form was removed after this A/B, DOPT_LAGGED_SYNC=signal now runs the event form), 512 and 4096
    # workers, RCCL world 1 forced, interleaved three times -> profiles/r5_sync_ab.txt
    for rep in 1 2 3; do
      for w in 512 4096; do
        for sy in event signal; do
          DOPT_LAGGED_SYNC=$sy DOPT_FORCE_COLLECTIVES=1 bench_step r5sg_${sy}_${w}_$rep 200 --no-cpu-baseline \
            --no-secondary --scaling weak --phase --workers $w --steps 100 --warmup 5
        done
      done
    done
    echo "=== trace, signal"
    DOPT_LAGGED_SYNC=signal DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv \
      -d gpurun_out/r5_st_sig -o run -- python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
      --workers 512 --steps 50 --warmup 5 > gpurun_out/r5_st_sig.log 2>&1 || die sig_ab 1
    python3 tools/trace_rounds.py gpurun_out/r5_st_sig/run_kernel_trace.csv
    python3 tools/trace_window.py gpurun_out/r5_st_sig/run_kernel_trace.csv ;;
  cur_ab)  # the all-to-all on the process group's stream (nccl, default) vs on the side stream with the engine's own
    # event behind it (current), 512 and 4096 workers, forced, interleaved three times; traces; host probe of
    # current -> profiles/r5_cur_ab.txt
    for rep in 1 2 3; do
      for w in 512 4096; do
        for st in nccl current; do
          DOPT_A2A_STREAM=$st DOPT_FORCE_COLLECTIVES=1 bench_step r5cu_${st}_${w}_$rep 200 --no-cpu-baseline \
            --no-secondary --scaling weak --phase --workers $w --steps 100 --warmup 5
        done
      done
    done
    for st in nccl current; do
      echo "=== trace, $st"
      DOPT_A2A_STREAM=$st DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv \
        -d gpurun_out/r5_st_cu_$st -o run -- python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
        --workers 512 --steps 50 --warmup 5 > gpurun_out/r5_st_cu_$st.log 2>&1 || die cur_ab 1
      python3 tools/trace_rounds.py gpurun_out/r5_st_cu_$st/run_kernel_trace.csv
      python3 tools/trace_window.py gpurun_out/r5_st_cu_$st/run_kernel_trace.csv
    done
    DOPT_A2A_STREAM=current DOPT_FORCE_COLLECTIVES=1 timeout -k 10 200 python3 tools/host_round_probe.py \
      > gpurun_out/r5_host_probe_cur.json 2> gpurun_out/r5_host_probe_cur.err \
      || { tail -n 20 gpurun_out/r5_host_probe_cur.err; die cur_ab 1; }
    cat gpurun_out/r5_host_probe_cur.json ;;
  mainpy8)  # main.py (the reference's experiment: 4 trainers x 10^4 rounds, N = 25) under torch.distributed.run
    # with 8 gloo ranks sharing the one GPU -> profiles/r5_mainpy8.log (Table II: 5425 / 7214 / 5666 / 5549)
    echo "=== main.py, 8 ranks"
    (cd distributed-optimization_amd && MPLBACKEND=Agg DOPT_BACKEND=gloo DOPT_DEVICE=0 timeout -k 10 900 \
      python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 \
      main.py) > gpurun_out/r5_mainpy8.log 2>&1 || { tail -n 30 gpurun_out/r5_mainpy8.log; die mainpy8 1; }
    grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/r5_mainpy8.log | tail -n 30 ;;
  trainer8)  # the drop-in trainers at 2 and 8 gloo ranks vs the C2 fixture
    echo "=== trainers at 8 ranks"; tests r5_trainer8 tests/test_gpu_distributed.py -k trainers_multiprocess_match ;;
  mixrec_ab)  # (historical: the records were reverted after this A/B showed no difference; DOPT_MIXCS_REC is now
    # ignored) k_mixcs with the per-worker mix records vs the CSR arrays (DOPT_MIXCS_REC=0, A/B library),
    # every worker mixed there (DOPT_PHASE_INTERIOR=0) at 4096 and 512 workers, and the strong proxy (512, forced),
    # kernel traces, interleaved twice -> profiles/r5_mixrec_ab.txt
    for rep in 1 2; do
      for w in 4096 512; do
        for rec in 1 0; do
          echo "=== rep $rep, $w workers, DOPT_MIXCS_REC=$rec, DOPT_PHASE_INTERIOR=0"
          DOPT_LIB=$AB DOPT_MIXCS_REC=$rec DOPT_PHASE_INTERIOR=0 timeout -s KILL 150 rocprofv3 --kernel-trace \
            --output-format csv -d gpurun_out/r5_mr_${w}_${rec}_$rep -o run -- python3 bench.py --no-cpu-baseline \
            --no-secondary --scaling weak --phase --workers $w --steps 30 --warmup 3 \
            > gpurun_out/r5_mr_${w}_${rec}_$rep.log 2>&1 || die mixrec_ab 1
          python3 tools/trace_rounds.py gpurun_out/r5_mr_${w}_${rec}_$rep/run_kernel_trace.csv
        done
      done
      for rec in 1 0; do
        DOPT_LIB=$AB DOPT_MIXCS_REC=$rec DOPT_FORCE_COLLECTIVES=1 bench_step r5mr_phase_512_${rec}_$rep 200 \
          --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 100 --warmup 5
      done
    done ;;
  lb_ab)  # the objective terms in register batches inside the row stream (VAR bit 21, instance 3291187) vs the
    # deferred terms after it (default 1210419), A/B library, interleaved in one process, 512 / 4096 workers
    # -> profiles/r5_lb_ab.txt
    for w in 512 4096 512; do
      echo "=== in-stream objective batches, $w workers"
      DOPT_LIB=$AB timeout -k 10 300 python3 tools/kr_variants.py --mode x32 --variants=-1,3291187 --reps 7 \
        --rounds 20 --workers $w > gpurun_out/r5_lb_ab_$w.json 2> gpurun_out/r5_lb_ab_$w.err \
        || { tail -n 20 gpurun_out/r5_lb_ab_$w.err; die lb_ab 1; }
      cat gpurun_out/r5_lb_ab_$w.json
    done ;;
  round_index)  # are the first rounds of a run slower because of the iterates or of the clocks? two chains from zero
    # iterates back to back, every round kernel timed -> profiles/r5_round_index.json
    timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5_ri -o run -- python3 \
      tools/round_index_probe.py > gpurun_out/r5_round_index.log 2>&1 || { tail -n 20 gpurun_out/r5_round_index.log; die round_index 1; }
    python3 tools/round_index_probe.py --analyse gpurun_out/r5_ri/run_kernel_trace.csv | tee gpurun_out/r5_round_index.json ;;
  pe_ab)  # the sampled profiling events' release: device scope (default) / none (hipEventDisableSystemFence) / system,
    # the no-flag default line's shape (300 rounds, events every 30th launch) and the driver's (20, every 2nd), no
    # secondary legs, A/B library, interleaved twice -> profiles/r5_pe_ab.txt
    for rep in 1 2; do
      for pe in dev nofence sys; do
        DOPT_LIB=$AB DOPT_PROF_EV=$pe bench_step r5pe2_${pe}_300_$rep 200 --no-cpu-baseline --no-secondary --steps 300 --warmup 3
        DOPT_LIB=$AB DOPT_PROF_EV=$pe bench_step r5pe2_${pe}_20_$rep 200 --no-cpu-baseline --no-secondary --steps 20 --warmup 5
      done
    done ;;
  sync_tests)  # the multi-GPU tests of the value-sync mode (and everything beside them in those files)
    echo "=== value-sync tests"; tests r5_sync_tests tests/test_gpu_distributed.py -k "value or current or event or self_exchange or torus" ;;
  rank_proxy)  # rank 0 of the 8-rank SCALE run on one GPU (tools/rank_proxy.py: its real plan, boundary share and
    # send set, the exchange through RCCL to itself) beside the fused 4096-worker round, weak (4096 per rank) and
    # strong (512 per rank) legs, steady state, interleaved twice -> profiles/r5_rank_proxy.txt
    for s in weak strong; do
      st=400; wu=50
      [ $s = strong ] && { st=3000; wu=400; }
      echo "=== rank proxy, $s leg, rank 0 of 8"
      timeout -k 10 400 python3 tools/rank_proxy.py --world 8 --rank 0 --scaling $s --reps 2 --steps $st --warmup $wu \
        > gpurun_out/r5_rp_$s.json 2> gpurun_out/r5_rp_$s.err || { tail -n 20 gpurun_out/r5_rp_$s.err; die rank_proxy 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/r5_rp_$s.json').read().strip().splitlines()[-1]); print('plan', d['plan']); [print(g['leg'], g['workers'], round(g['value']), round(g['ms_per_round'], 4), round(g['kernel_avg_ms'], 4)) for g in d['legs']]; print('proxy / fused', [round(x, 4) for x in d['proxy_over_fused']])"
    done ;;
  proxy_ab)  # what the weak-leg rank pays over the fused round: arms of tools/rank_proxy.py (weak, rank 0 of 8), one
    # process each: default / one stream / RCCL at 8 channels / two runners (the second after the first's legs) with
    # the box's 4 HW queues per process and with 8 (ARMS overrides the list)
    for arm in ${ARMS:-default side0 nch8 reps2 hwq8}; do
      envs=""; extra=""
      case $arm in
        side0) envs="DOPT_LAGGED_SIDE=0" ;;
        nch8) envs="NCCL_MAX_NCHANNELS=8" ;;
        hwq8) envs="GPU_MAX_HW_QUEUES=8"; extra="--reps 2" ;;
        reps2) extra="--reps 2" ;;
        pfirst) extra="--reps 2 --legs proxy,fused" ;;
        palone) extra="--legs proxy" ;;
        pfresh) envs="DOPT_FRESH_STREAMS=1"; extra="--reps 2 --legs proxy,fused" ;;
        nch2) envs="NCCL_MAX_NCHANNELS=2" ;;
        palone_w400) extra="--legs proxy --warmup 400" ;;
        palone_side0) envs="DOPT_LAGGED_SIDE=0"; extra="--legs proxy" ;;
        palone_nch2) envs="NCCL_MAX_NCHANNELS=2"; extra="--legs proxy" ;;
        palone_cur) envs="DOPT_A2A_STREAM=current"; extra="--legs proxy" ;;
        palone_lo) envs="DOPT_NCCL_HIPRI=0"; extra="--legs proxy" ;;
        palone_serial) envs="DOPT_LAGGED_SIDE=0 DOPT_A2A_STREAM=current"; extra="--legs proxy" ;;
        pre_palone) extra="--legs proxy --prealloc" ;;
        palone_cur2) envs="DOPT_A2A_STREAM=current"; extra="--legs proxy" ;;
        palone_simple) envs="NCCL_PROTO=Simple"; extra="--legs proxy" ;;
        palone_ll) envs="NCCL_PROTO=LL"; extra="--legs proxy" ;;
        palone_ll128) envs="NCCL_PROTO=LL128"; extra="--legs proxy" ;;
        early_default) extra="--early-streams" ;;
        fshort_palone) extra="--legs fused,proxy --fused-steps 5" ;;
        falone) extra="--legs fused" ;;
        pre_falone) extra="--legs fused --prealloc" ;;
        fthen_serial) envs="DOPT_LAGGED_SIDE=0 DOPT_A2A_STREAM=current" ;;
        pfirst_w400) extra="--reps 2 --legs proxy,fused --warmup 400" ;;
        simple) envs="NCCL_PROTO=Simple" ;;
      esac
      echo "=== $arm ($envs $extra)"
      env $envs timeout -k 10 300 python3 tools/rank_proxy.py --world 8 --rank 0 --scaling weak --reps 1 --steps 300 \
        --warmup 50 $extra > gpurun_out/r5_pab_$arm.json 2> gpurun_out/r5_pab_$arm.err \
        || { tail -n 20 gpurun_out/r5_pab_$arm.err; die proxy_ab 1; }
      grep '^{"leg"' gpurun_out/r5_pab_$arm.err | python3 -c "import json,sys; [print(d['leg'], d['rep'], round(d['value']), round(d['ms_per_round'], 4), round(d['kernel_avg_ms'], 4)) for d in map(json.loads, sys.stdin)]"
    done ;;
  proxy_legs_trace)  # kernel trace of two proxy legs in one process (the second runner is slower: why?)
    timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5_plt -o run -- \
      python3 tools/rank_proxy.py --world 8 --rank 0 --scaling weak --legs fused,proxy --reps 2 --steps 200 --warmup 20 \
      > gpurun_out/r5_plt.log 2>&1 || { tail -n 20 gpurun_out/r5_plt.log; die proxy_legs_trace 1; }
    grep '^{"leg"' gpurun_out/r5_plt.log || true
    python3 tools/trace_legs.py gpurun_out/r5_plt/run_kernel_trace.csv ;;
  rs_chunks)  # C5 across ranks: the column-chunked rounds pipelined across rounds (dopt_rs_phase_cols_range) -- the
    # row-space GPU tests (incl. the RCCL world-1 bitwise test), then the price of chunking at one rank's shape of 8
    # (128 workers) and at world 1's (1024), RCCL world 1 forced -> profiles/r5_rs_chunks.txt
    echo "=== row-space GPU tests"; tests r5_rs_tests tests/test_gpu_rowspace.py
    for w in 128 1024; do
      echo "=== chunk proxy, $w workers"
      timeout -k 10 300 python3 tools/rs_chunk_proxy.py --workers $w --chunks 1,2,3,4 --reps 2 --steps 40 --warmup 5 \
        > gpurun_out/r5_rsc_$w.json 2> gpurun_out/r5_rsc_$w.err || { tail -n 20 gpurun_out/r5_rsc_$w.err; die rs_chunks 1; }
      grep '^{"K"' gpurun_out/r5_rsc_$w.err
    done ;;
  rs_chunks_trace)  # kernel trace of the C5 rank shape (128 workers, K = 1 and 2) -> profiles/r5_rs_chunks.txt
    timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5_rsct -o run -- \
      python3 tools/rs_chunk_proxy.py --workers 128 --chunks 1,2 --reps 1 --steps 40 --warmup 5 \
      > gpurun_out/r5_rsct.log 2>&1 || { tail -n 20 gpurun_out/r5_rsct.log; die rs_chunks_trace 1; }
    grep '^{"K"' gpurun_out/r5_rsct.log || true
    python3 tools/trace_legs.py gpurun_out/r5_rsct/run_kernel_trace.csv 1 k_rs_rows ;;
  rank_proxy_c4)  # C4's rank 0 of 8 (a strip of 32 torus rows, 8192 workers, 512 boundary) beside a fused 8192-worker
    # round (random 4-regular: the same kernel and degree) -> profiles/r5_rank_proxy.txt
    echo "=== rank proxy, C4 rank 0 of 8"
    timeout -k 10 400 python3 tools/rank_proxy.py --world 8 --rank 0 --config c4 --fused-workers 8192 --reps 2 \
      --steps 100 --warmup 20 > gpurun_out/r5_rp_c4.json 2> gpurun_out/r5_rp_c4.err \
      || { tail -n 20 gpurun_out/r5_rp_c4.err; die rank_proxy_c4 1; }
    grep '^{"leg"' gpurun_out/r5_rp_c4.err | python3 -c "import json,sys; [print(d['leg'], d['rep'], d['workers'], round(d['value']), round(d['ms_per_round'], 4), round(d['kernel_avg_ms'], 4)) for d in map(json.loads, sys.stdin)]" ;;
  rs_wg_ab)  # the row-space pass's row groups at one rank's shape of C5 over 8 (128 workers: 2048 rows, one group of
    # 2048-row workgroups by default), A/B library, K = 2 -> profiles/r5_rs_chunks.txt
    for rep in 1 2; do
      for wg in 1 2 4; do
        echo "=== DOPT_RS_WG=$wg rep $rep"
        DOPT_LIB=$AB DOPT_RS_WG=$wg timeout -k 10 300 python3 tools/rs_chunk_proxy.py --workers 128 --chunks 2 --reps 1 \
          --steps 40 --warmup 5 > gpurun_out/r5_rswg_$wg.json 2> gpurun_out/r5_rswg_$wg.err \
          || { tail -n 20 gpurun_out/r5_rswg_$wg.err; die rs_wg_ab 1; }
        grep '^{"K"' gpurun_out/r5_rswg_$wg.err
      done
    done ;;
  contig_ab)  # (historical, profiles/r5_rank_proxy.txt call 11: DOPT_CONTIG_ROWS, a contiguous-allocation A/B knob for the
    # shard rows, showed no difference and was removed)
    echo "contig_ab: the knob was removed"; exit 2 ;;
  rank_proxy_all)  # every rank of the 8-rank weak and strong legs on one GPU (one process each, the fused leg first
    # and last): the SCALE time is the max over ranks -> profiles/r5_rank_proxy.txt
    for sc in weak strong; do
      st=300; wu=50
      [ $sc = strong ] && { st=2000; wu=300; }
      for r in 0 1 2 3 4 5 6 7; do
        legs=proxy
        [ $r = 0 ] && legs=fused,proxy
        [ $r = 7 ] && legs=proxy,fused
        timeout -k 10 300 python3 tools/rank_proxy.py --world 8 --rank $r --scaling $sc --legs $legs --reps 1 \
          --steps $st --warmup $wu > gpurun_out/r5_rpa_${sc}_$r.json 2> gpurun_out/r5_rpa_${sc}_$r.err \
          || { tail -n 20 gpurun_out/r5_rpa_${sc}_$r.err; die rank_proxy_all 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r5_rpa_${sc}_$r.json').read().strip().splitlines()[-1]); p=d['plan']; [print('$sc', 'rank', $r, g['leg'], g['workers'], 'halo', p['halo_rows_in'], 'interior', p['interior'], round(g['value']), round(g['ms_per_round'], 4), round(g['kernel_avg_ms'], 4)) for g in d['legs']]"
      done
    done ;;
  proxy_pmc)  # HBM traffic of the weak rank proxy's gradient kernel with the exchange beside it vs serialised
    # (FETCH_SIZE / WRITE_SIZE passes, proxy alone, 100 rounds) -> profiles/r5_rank_proxy.txt
    for arm in overlap serial; do
      envs=""
      [ $arm = serial ] && envs="DOPT_LAGGED_SIDE=0 DOPT_A2A_STREAM=current"
      for c in FETCH_SIZE WRITE_SIZE; do
        echo "=== $arm $c"
        env $envs timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r5_ppmc_${arm}_$c -o run -- \
          python3 tools/rank_proxy.py --world 8 --rank 0 --scaling weak --legs proxy --reps 1 --steps 100 --warmup 20 \
          > gpurun_out/r5_ppmc_${arm}_$c.log 2>&1 || { tail -n 20 gpurun_out/r5_ppmc_${arm}_$c.log; die proxy_pmc 1; }
        python3 - gpurun_out/r5_ppmc_${arm}_$c/run_counter_collection.csv <<'PY'
import collections, csv, statistics, sys
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    v[r["Kernel_Name"][:70]].append(float(r["Counter_Value"]))
for k, xs in sorted(v.items(), key=lambda kv: -statistics.median(kv[1])):
    if len(xs) >= 50:
        print(f"  {len(xs):5d} dispatches  median {statistics.median(xs[len(xs)//2:]):14.1f} KB  {k}")
PY
      done
    done ;;
  rank_proxy_trace)  # kernel trace of the weak-leg rank proxy (rank 0 of 8, 200 rounds) -> profiles/r5_rank_proxy.txt
    timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_rpt -o run -- \
      python3 tools/rank_proxy.py --world 8 --rank 0 --scaling weak --legs proxy --reps 1 --steps 200 --warmup 20 \
      > gpurun_out/r5_rpt.log 2>&1 || { tail -n 20 gpurun_out/r5_rpt.log; die rank_proxy_trace 1; }
    python3 tools/trace_rounds.py gpurun_out/r5_rpt/run_kernel_trace.csv ;;
  strong_proxy)  # fused 4096 / fused 512 / phase 512 (forced) / phase1 512 -> profiles/r5_strong_proxy.txt
    for w in 4096 512; do
      bench_step r5sp_fused_$w 200 --no-cpu-baseline --no-secondary --scaling weak --workers $w --steps 100 --warmup 5
    done
    DOPT_FORCE_COLLECTIVES=1 bench_step r5sp_phase_512 200 --no-cpu-baseline --no-secondary --scaling weak --phase \
      --workers 512 --steps 100 --warmup 5
    bench_step r5sp_phase1_512 200 --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 100 \
      --warmup 5 ;;
  strong_long)  # the same four legs in the steady state: ~0.4-0.6 s of rounds each after a ~60 ms warmup,
    # so the 512-worker legs are not timed inside the post-setup transient (section 5) that a 100-round
    # 512-worker leg (18 ms) sits in entirely; interleaved twice -> profiles/r5_strong_long.txt
    for rep in 1 2; do
      bench_step r5sl_fused_4096_$rep 200 --no-cpu-baseline --no-secondary --scaling weak --workers 4096 \
        --steps 400 --warmup 50
      bench_step r5sl_fused_512_$rep 200 --no-cpu-baseline --no-secondary --scaling weak --workers 512 \
        --steps 3000 --warmup 400
      DOPT_FORCE_COLLECTIVES=1 bench_step r5sl_phase_512_$rep 200 --no-cpu-baseline --no-secondary --scaling weak \
        --phase --workers 512 --steps 3000 --warmup 400
      bench_step r5sl_phase1_512_$rep 200 --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 \
        --steps 3000 --warmup 400
    done ;;
  strong_long_tr)  # strong_long's legs with the engine's own RCCL communicator (default) and the process group's
    # all-to-all (DOPT_TRANSPORT=pg) for the forced 512-worker phase round, interleaved twice -> profiles/r5_transport.txt
    for rep in 1 2; do
      bench_step r5slt_fused_4096_$rep 200 --no-cpu-baseline --no-secondary --scaling weak --workers 4096 \
        --steps 400 --warmup 50
      bench_step r5slt_fused_512_$rep 200 --no-cpu-baseline --no-secondary --scaling weak --workers 512 \
        --steps 3000 --warmup 400
      DOPT_FORCE_COLLECTIVES=1 bench_step r5slt_phase_512_rccl_$rep 200 --no-cpu-baseline --no-secondary --scaling weak \
        --phase --workers 512 --steps 3000 --warmup 400
      DOPT_TRANSPORT=pg DOPT_FORCE_COLLECTIVES=1 bench_step r5slt_phase_512_pg_$rep 200 --no-cpu-baseline --no-secondary \
        --scaling weak --phase --workers 512 --steps 3000 --warmup 400
    done ;;
  handoff_long)  # the hand-off forms of section 6 again in the steady state (512 workers, RCCL world 1 forced,
    # 3000 rounds after 400): events + side stream (default), one stream (DOPT_LAGGED_SIDE=0), the all-to-all on
    # the engine's stream (DOPT_A2A_STREAM=current), stream memory operations (DOPT_LAGGED_SYNC=value);
    # interleaved twice, then a kernel trace of the default -> profiles/r5_handoff_long.txt
    for rep in 1 2; do
      for arm in event side0 current value; do
        case $arm in
          event) envs="" ;; side0) envs="DOPT_LAGGED_SIDE=0" ;; current) envs="DOPT_A2A_STREAM=current" ;;
          value) envs="DOPT_LAGGED_SYNC=value" ;;
        esac
        ( if [ -n "$envs" ]; then export "$envs"; fi
          DOPT_FORCE_COLLECTIVES=1 bench_step r5hl_${arm}_$rep 200 --no-cpu-baseline --no-secondary --scaling weak \
            --phase --workers 512 --steps 3000 --warmup 400 ) || exit 1
      done
    done
    echo "=== trace, default, steady state"
    DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv \
      -d gpurun_out/r5_hl_trace -o run -- python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
      --workers 512 --steps 1500 --warmup 400 > gpurun_out/r5_hl_trace.log 2>&1 || die handoff_long 1
    python3 tools/trace_rounds.py gpurun_out/r5_hl_trace/run_kernel_trace.csv ;;
  rccl_probe)  # host cost of RCCL's own group of sends / receives (tools/rccl_probe, built here beforehand:
    # hipcc -O2 -o tools/rccl_probe tools/rccl_probe.cpp -I/opt/rocm/include/rccl -L/opt/rocm/lib -lrccl) vs the
    # process group's all-to-all (tools/pg_a2a_probe.py), same sizes -> the head of profiles/r5_transport.txt
    timeout -k 10 120 ./tools/rccl_probe > gpurun_out/r5_rccl_probe.txt 2>&1 || { tail -n 20 gpurun_out/r5_rccl_probe.txt; die rccl_probe 1; }
    timeout -k 10 150 python3 tools/pg_a2a_probe.py >> gpurun_out/r5_rccl_probe.txt 2>&1 || { tail -n 20 gpurun_out/r5_rccl_probe.txt; die rccl_probe 1; }
    grep -E "^bytes|^pg alltoall" gpurun_out/r5_rccl_probe.txt ;;
  transport_ab)  # the engine's own RCCL communicator (dopt_lagged_exchange, DOPT_TRANSPORT=rccl) vs the process
    # group's all-to-all-v (pg): the RCCL GPU tests, the host cost per round at 512 workers, and the rank proxy's
    # weak / strong legs, interleaved twice -> profiles/r5_transport.txt
    timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_distributed.py \
      -k "rccl" > gpurun_out/r5_transport_tests.txt 2>&1 || { tail -n 30 gpurun_out/r5_transport_tests.txt; die transport_ab 1; }
    tail -n 2 gpurun_out/r5_transport_tests.txt
    for rep in 1 2; do
      for tr in rccl pg; do
        echo "=== host probe, DOPT_TRANSPORT=$tr (rep $rep)"
        DOPT_LIB=$AB DOPT_HOST_TIMING=1 DOPT_TRANSPORT=$tr DOPT_FORCE_COLLECTIVES=1 timeout -k 10 200 \
          python3 tools/host_round_probe.py > gpurun_out/r5_tr_host_$tr.json 2> gpurun_out/r5_tr_host_$tr.err \
          || { tail -n 20 gpurun_out/r5_tr_host_$tr.err; die transport_ab 1; }
        cat gpurun_out/r5_tr_host_$tr.json
      done
    done
    for rep in 1 2; do
      for s in strong weak; do
        st=400; wu=50
        [ $s = strong ] && { st=3000; wu=400; }
        for tr in rccl pg; do
          echo "=== rank proxy, $s leg, rank 0 of 8, DOPT_TRANSPORT=$tr (rep $rep)"
          DOPT_TRANSPORT=$tr timeout -k 10 300 python3 tools/rank_proxy.py --world 8 --rank 0 --scaling $s --steps $st \
            --warmup $wu > gpurun_out/r5_tr_rp.json 2> gpurun_out/r5_tr_rp.err || { tail -n 20 gpurun_out/r5_tr_rp.err; die transport_ab 1; }
          python3 -c "import json; d=json.loads(open('gpurun_out/r5_tr_rp.json').read().strip().splitlines()[-1]); [print(g['leg'], g['workers'], round(g['value']), round(g['ms_per_round'], 4), round(g['kernel_avg_ms'], 4)) for g in d['legs']]; print('proxy / fused', [round(x, 4) for x in d['proxy_over_fused']])"
        done
      done
    done ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
