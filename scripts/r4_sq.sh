#!/bin/bash
# Round 4: SQ counters of the C3 headline round kernel in three --pmc passes (SQ block only, <= 8
# counters each; GRBM in the third), a kernel trace for its VGPR / LDS / scratch, the summary
# (tools/sq_summary.py -> profiles/r4_c3_sq.txt); then the C5 row-space pass with the row dots
# through LDS vs the DPP butterfly (tools/rs_ab.py, A/B library, interleaved).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
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
echo "=== C5 pass: row dots through LDS (1) vs DPP (0)"
DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so timeout -k 10 300 python3 tools/rs_ab.py --dtype float64 \
  --data-dtype float32 --reps 3 --shapes "2,8,2,1 2,8,2,0" > gpurun_out/r4_c5_ldot.txt 2>&1 \
  || { tail -n 20 gpurun_out/r4_c5_ldot.txt; exit 1; }
cat gpurun_out/r4_c5_ldot.txt | grep -v amdgpu.ids
echo "=== C3 profile: kernel stats + FETCH_SIZE / WRITE_SIZE passes (summarised locally into profiles/r4_*)"
OUT=gpurun_out/prof_r4 bash scripts/profile.sh || exit 1
echo "=== C5 profile (x32 row-space rounds)"
OUT=gpurun_out/prof_r4c5 PSTEPS=6 BENCH_ARGS="--config c5" bash scripts/profile.sh || exit 1
echo "=== done"
