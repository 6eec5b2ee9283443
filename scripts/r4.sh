#!/bin/bash
# Round-4 evidence, one gpurun call for any list of steps:
#   /usr/local/graft/bin/gpurun -- 'bash scripts/r4.sh full strong_trace'
# Every step runs from the repository root on the GPU box, writes under gpurun_out/, and stops the
# script on a failure (a GPU test failure in `full` / `dist_tests` lists the failures and goes on).
# The summaries judged are copied into profiles/ (named in each step's comment).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
AB=$PWD/distributed-optimization_amd/libdopt_ab.so

die() { echo "step $1 failed (rc $2)"; exit "$2"; }
json_line() {  # value, ms_per_step, kernel ms of a bench JSON file's last line
  tail -n 1 "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
}
bench_step() {  # bench_step <name> <timeout> <bench.py args...>  (env assignments before the call apply)
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" python3 bench.py "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err" \
    || { tail -n 20 "gpurun_out/$name.err"; die "$name" 1; }
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
rs_ab() {  # rs_ab <name> <reps> <shapes>: C5 row-space pass shapes (tools/rs_ab.py), A/B library, interleaved
  DOPT_LIB=$AB timeout -k 10 400 python3 tools/rs_ab.py --dtype float64 --data-dtype float32 --reps "$2" \
    --shapes "$3" > "gpurun_out/$1.txt" 2>&1 || { tail -n 20 "gpurun_out/$1.txt"; die "$1" 1; }
  grep -v amdgpu.ids "gpurun_out/$1.txt" | tail -n 4
}

for step in "$@"; do
  case $step in
  full)  # every -m gpu test, smoke(), the no-flag bench line -> profiles/r4_gpu_tests.txt, r4_bench_default.json
    echo "=== pytest -m gpu"; tests r4_full_tests tests -m gpu
    echo "=== smoke"
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 \
      || { tail -n 20 gpurun_out/r4_smoke.log; die smoke 1; }
    bench_step r4_full_bench 420 ;;
  driver_bench)  # the driver's shape -> profiles/r4_bench_a.json
    bench_step r4_base_bench 420 --gpus 1 --steps 20 --warmup 5 ;;
  dist_tests)  # the multi-GPU and row-space GPU tests
    echo "=== multi-GPU tests"; tests r4_dist_tests tests/test_gpu_distributed.py tests/test_gpu_rowspace.py ;;
  early_ab)  # early prologue (-1 = 1210419) vs round 3's 161843 -> profiles/r4_strong_proxy.txt
    for w in 512 4096; do
      echo "=== early-prologue A/B, $w workers"
      DOPT_LIB=$AB timeout -k 10 200 python3 tools/kr_variants.py --mode x32 --variants=-1,161843 --reps 7 --rounds 20 \
        --workers $w > gpurun_out/r4_early_ab_$w.json 2> gpurun_out/r4_early_ab_$w.err || die early_ab 1
      cat gpurun_out/r4_early_ab_$w.json
    done ;;
  ab8)  # 8 waves per workgroup (1210675) vs the default -> profiles/r4_ab8.txt
    for w in 512 1024 4096; do
      echo "=== 8-wave A/B, $w workers"
      DOPT_LIB=$AB timeout -k 10 200 python3 tools/kr_variants.py --mode x32 --variants=-1,1210675 --reps 7 --rounds 20 \
        --workers $w > gpurun_out/r4_ab8_$w.json 2> gpurun_out/r4_ab8_$w.err || die ab8 1
      cat gpurun_out/r4_ab8_$w.json
    done ;;
  strong_proxy)  # fused / phase (collectives forced) / phase1 at 4096 and 512 workers -> profiles/r4_strong_proxy*.txt
    for w in 4096 512; do
      bench_step r4sp_fused_$w 200 --no-cpu-baseline --no-secondary --scaling weak --workers $w --steps 100 --warmup 5
      DOPT_FORCE_COLLECTIVES=1 bench_step r4sp_phase_$w 200 --no-cpu-baseline --no-secondary --scaling weak --phase \
        --workers $w --steps 100 --warmup 5
      bench_step r4sp_phase1_$w 200 --no-cpu-baseline --no-secondary --scaling weak --phase --workers $w --steps 100 \
        --warmup 5
    done ;;
  strong_mid)  # the strong leg's rank shapes at N = 2 and 4 (2048 / 1024 workers): fused, phase (forced) -> profiles/r4_strong_mid.txt
    for w in 2048 1024; do
      bench_step r4sp_fused_$w 200 --no-cpu-baseline --no-secondary --scaling weak --workers $w --steps 100 --warmup 5
      DOPT_FORCE_COLLECTIVES=1 bench_step r4sp_phase_$w 200 --no-cpu-baseline --no-secondary --scaling weak --phase \
        --workers $w --steps 100 --warmup 5
    done
    bench_step r4sp_fused_4096 200 --no-cpu-baseline --no-secondary --scaling weak --workers 4096 --steps 100 --warmup 5 ;;
  host_probe)  # host time per round at 512 workers, collectives forced / skipped -> profiles/r4_host_probe*.json
    for f in 1 0; do
      echo "=== host probe, DOPT_FORCE_COLLECTIVES=$f"
      DOPT_FORCE_COLLECTIVES=$f timeout -k 10 200 python3 tools/host_round_probe.py > gpurun_out/r4_host_probe_f$f.json \
        2> gpurun_out/r4_host_probe_f$f.err || { tail -n 20 gpurun_out/r4_host_probe_f$f.err; die host_probe 1; }
      cat gpurun_out/r4_host_probe_f$f.json
    done ;;
  strong_trace)  # kernel traces of the phase path at 512 workers, collectives skipped / forced -> profiles/r4_strong_trace.txt
    B="bench.py --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 50 --warmup 5"
    for f in 0 1; do
      echo "=== trace, DOPT_FORCE_COLLECTIVES=$f"
      DOPT_FORCE_COLLECTIVES=$f timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/r4_st_f$f -o run -- python3 $B > gpurun_out/r4_st_f$f.log 2>&1 || die strong_trace 1
      python3 tools/trace_rounds.py gpurun_out/r4_st_f$f/run_kernel_trace.csv
    done ;;
  mixcs_ab)  # k_mixcs one launch with the ticket vs two launches, timing-only cuts -> profiles/r4_mixcs_*.txt
    B="bench.py --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 30 --warmup 3"
    for v in "TICKET=1 CUT=0" "TICKET=1 CUT=4" "TICKET=1 CUT=1" "TICKET=1 CUT=2" "TICKET=1 CUT=3" "TICKET=0 CUT=0"; do
      tk=${v%% *}; ct=${v##* }; tag=mx_${tk#TICKET=}_${ct#CUT=}
      echo "=== DOPT_MIXCS_$tk DOPT_MIXCS_$ct"
      DOPT_LIB=$AB DOPT_MIXCS_TICKET=${tk#TICKET=} DOPT_MIXCS_CUT=${ct#CUT=} timeout -s KILL 150 rocprofv3 --kernel-trace \
        --output-format csv -d gpurun_out/r4_$tag -o run -- python3 $B > gpurun_out/r4_$tag.log 2>&1 || die mixcs_ab 1
      python3 tools/trace_rounds.py gpurun_out/r4_$tag/run_kernel_trace.csv
    done ;;
  mixcs_boundary)  # k_mixcs when every worker is mixed in it (DOPT_PHASE_INTERIOR=0: the N = 8 boundary share
    # is 84 %), 4096 and 512 workers, kernel traces -> profiles/r4_mixcs_boundary.txt
    for w in 4096 512; do
      for it in 1 0; do
        echo "=== $w workers, DOPT_PHASE_INTERIOR=$it"
        DOPT_PHASE_INTERIOR=$it timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_mb_${w}_$it \
          -o run -- python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase --workers $w --steps 30 \
          --warmup 3 > gpurun_out/r4_mb_${w}_$it.log 2>&1 || die mixcs_boundary 1
        python3 tools/trace_rounds.py gpurun_out/r4_mb_${w}_$it/run_kernel_trace.csv
      done
    done ;;
  mixcs_r)  # k_mixcs group size at 4096 workers, every worker mixed in it: R = 8 (default) vs 64 (A/B library)
    for r in 8 64; do
      echo "=== DOPT_MIXCS_R=$r, DOPT_PHASE_INTERIOR=0"
      DOPT_LIB=$AB DOPT_MIXCS_R=$r DOPT_PHASE_INTERIOR=0 timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv \
        -d gpurun_out/r4_mr_$r -o run -- python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
        --workers 4096 --steps 30 --warmup 3 > gpurun_out/r4_mr_$r.log 2>&1 || die mixcs_r 1
      python3 tools/trace_rounds.py gpurun_out/r4_mr_$r/run_kernel_trace.csv
    done ;;
  mixcs_cpb)  # k_mixcs column blocks of 1 vs 2 chunks per lane (A/B library), every worker mixed in it, 4096 / 512
    for w in 4096 512; do
      for c in 1 2; do
        echo "=== DOPT_MIXCS_CPB=$c, $w workers, DOPT_PHASE_INTERIOR=0"
        DOPT_LIB=$AB DOPT_MIXCS_CPB=$c DOPT_PHASE_INTERIOR=0 timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv \
          -d gpurun_out/r4_mc_${w}_$c -o run -- python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
          --workers $w --steps 30 --warmup 3 > gpurun_out/r4_mc_${w}_$c.log 2>&1 || die mixcs_cpb 1
        python3 tools/trace_rounds.py gpurun_out/r4_mc_${w}_$c/run_kernel_trace.csv
      done
    done ;;
  rehearsal8)  # the SCALE command shape at 8 gloo ranks on this one GPU -> profiles/r4_rehearsal8.json
    echo "=== 8-rank rehearsal"
    timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 8 --backend gloo --workers 256 --strong-workers 2048 --steps 5 --warmup 3 \
      > gpurun_out/r4_rehearsal8.json 2> gpurun_out/r4_rehearsal8.err || { tail -n 30 gpurun_out/r4_rehearsal8.err; die rehearsal8 1; }
    tail -n 1 gpurun_out/r4_rehearsal8.json | cut -c 1-300 ;;
  sq)  # SQ counters of the C3 round kernel (3 --pmc passes + a kernel trace) -> profiles/r4_c3_sq.txt
    B="bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --scaling weak"
    P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
    P2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT"
    P3="SQ_LEVEL_WAVES SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE GRBM_COUNT"
    n=0
    for P in "$P1" "$P2" "$P3"; do
      n=$((n + 1)); echo "=== sq pass $n"
      timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/r4_sq$n -o run -- python3 $B \
        > gpurun_out/r4_sq$n.log 2>&1 || die sq 1
    done
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_kt -o run -- python3 $B \
      > gpurun_out/r4_kt.log 2>&1 || die sq 1
    python3 tools/sq_summary.py gpurun_out/r4_sq1 gpurun_out/r4_sq2 gpurun_out/r4_sq3 gpurun_out/r4_kt \
      > gpurun_out/r4_c3_sq.txt && cat gpurun_out/r4_c3_sq.txt ;;
  c3_profile)  # C3 kernel stats + FETCH_SIZE / WRITE_SIZE passes -> profiles/r4_kernel_stats.csv, r4_pmc.json
    OUT=gpurun_out/prof_r4 PSTEPS=20 bash scripts/profile.sh || die c3_profile 1 ;;
  c5_profile)  # C5 x32 row-space rounds, same three passes -> profiles/r4_c5x32_*
    OUT=gpurun_out/prof_r4c5 PSTEPS=6 BENCH_ARGS="--config c5" bash scripts/profile.sh || die c5_profile 1 ;;
  c4_profile)  # C4 (65536 workers, torus, one GPU), same three passes -> profiles/r4_c4_*
    OUT=gpurun_out/prof_r4c4 PSTEPS=4 BENCH_ARGS="--config c4" bash scripts/profile.sh || die c4_profile 1 ;;
  c5_ldot)  # row dots: every lane through LDS (1) / lane pairs first (2) / DPP (0) -> profiles/r4_c5_ldot2.txt
    rs_ab r4_c5_ldot2 3 "2,8,2,2 2,8,2,1 2,8,2,0" ;;
  c5_shapes)  # rows in flight, row groups, 4 KiB blocks -> profiles/r4_c5_shapes.txt, r4_c5_groups.txt, r4_c5_cb4.txt
    rs_ab r4_c5_shapes 3 "2,8,2,1 2,16,2,1 2,8,4,1 2,8,1,1"
    rs_ab r4_c5_groups 5 "2,8,1,1 2,8,2,1"
    rs_ab r4_c5_cb4 5 "4,4,1,1 2,8,1,1" ;;
  mainpy)  # the reference's experiment end to end through the drop-in modules (4 trainers x 10^4 rounds)
    echo "=== main.py"
    (cd distributed-optimization_amd && MPLBACKEND=Agg timeout -k 10 600 python3 -u -c "import time, runpy; t=time.time(); import matplotlib; matplotlib.use('Agg'); runpy.run_path('main.py', run_name='__main__'); print('main.py wall %.1f s' % (time.time()-t))") \
      > gpurun_out/r4_mainpy.log 2>&1 || { tail -n 20 gpurun_out/r4_mainpy.log; die mainpy 1; }
    tail -n 25 gpurun_out/r4_mainpy.log ;;
  diag_trainers)  # the C2 trainers at 1 and 2 gloo ranks vs the fixture, every label (the dense-CSR k_mixcs bug)
    timeout -k 10 300 python3 tools/diag_trainers2.py > gpurun_out/r4_diag.log 2>&1 || die diag_trainers 1
    grep -v "amdgpu.ids\|socket.cpp\|Gloo\|Spectral\|Running\|finished" gpurun_out/r4_diag.log | head -60 ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== done"
