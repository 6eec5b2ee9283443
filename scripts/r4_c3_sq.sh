#!/bin/bash
# Round 4 baseline on one box: the driver-shaped bench line, then the SQ counters of the C3 headline
# round kernel in two --pmc passes (SQ block only, <= 8 counters each: occupancy / issue / waits, then
# instruction mix and LDS), then the strong-scaling proxy's 4096 / 512 worker shapes (fused round and
# the phase path at RCCL world 1).  Summary: profiles/r4_c3_sq.txt (tools/sq_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
set -o pipefail
echo "=== bench (driver shape)"
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_base_bench.json \
  2> gpurun_out/r4_base_bench.err || { tail -n 30 gpurun_out/r4_base_bench.err; exit 1; }
tail -n 1 gpurun_out/r4_base_bench.json | cut -c 1-400
BENCH="python3 -u bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --scaling weak"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT"
P3="SQ_LEVEL_WAVES SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE GRBM_COUNT"
n=0
for P in "$P1" "$P2" "$P3"; do
  n=$((n + 1))
  echo "=== sq pass $n"
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/r4_sq$n -o run -- $BENCH \
    > gpurun_out/r4_sq$n.log 2>&1 || { tail -n 20 gpurun_out/r4_sq$n.log; exit 1; }
done
echo "=== kernel trace (VGPR / LDS / scratch per dispatch)"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_kt -o run -- $BENCH \
  > gpurun_out/r4_kt.log 2>&1 || { tail -n 20 gpurun_out/r4_kt.log; exit 1; }
python3 tools/sq_summary.py gpurun_out/r4_sq1 gpurun_out/r4_sq2 gpurun_out/r4_sq3 gpurun_out/r4_kt > gpurun_out/r4_c3_sq.txt \
  && cat gpurun_out/r4_c3_sq.txt
for w in 512 4096; do  # early prologue (new default, -1) vs the round-3 default, interleaved in one process
  echo "=== early-prologue A/B, $w workers"
  DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so timeout -k 10 200 python3 tools/kr_variants.py --mode x32 \
    --variants -1,161843 --reps 7 --rounds 20 --workers $w > gpurun_out/r4_early_ab_$w.json 2> gpurun_out/r4_early_ab_$w.err \
    || { tail -n 20 gpurun_out/r4_early_ab_$w.err; exit 1; }
  cat gpurun_out/r4_early_ab_$w.json
done
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"; local rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -n 20 "gpurun_out/$name.err"; exit $rc; }
  tail -n 1 "gpurun_out/$name.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
}
for w in 4096 512; do
  step r4sp_fused_$w 200 python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --workers $w --steps 100 --warmup 5
  DOPT_FORCE_COLLECTIVES=1 step r4sp_phase_$w 200 python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
    --workers $w --steps 100 --warmup 5
done
echo "=== done"
