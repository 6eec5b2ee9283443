#!/bin/bash
# Round 4 on one box: the driver-shaped bench line, the early-prologue A/B (interleaved in one
# process, A/B library), and the strong-scaling proxy's 4096 / 512 worker shapes (fused round and
# the phase path at RCCL world 1, collectives forced and not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
echo "=== bench (driver shape)"
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_base_bench.json \
  2> gpurun_out/r4_base_bench.err || { tail -n 30 gpurun_out/r4_base_bench.err; exit 1; }
tail -n 1 gpurun_out/r4_base_bench.json | cut -c 1-600
for w in 512 4096; do  # early prologue (new default, -1) vs the round-3 default, interleaved in one process
  echo "=== early-prologue A/B, $w workers"
  DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so timeout -k 10 200 python3 tools/kr_variants.py --mode x32 \
    --variants=-1,161843 --reps 7 --rounds 20 --workers $w > gpurun_out/r4_early_ab_$w.json 2> gpurun_out/r4_early_ab_$w.err \
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
  step r4sp_phase1_$w 200 python3 bench.py --no-cpu-baseline --no-secondary --scaling weak --phase \
    --workers $w --steps 100 --warmup 5
done
echo "=== host round probe (512 workers, RCCL world 1, collectives forced)"
timeout -k 10 200 python3 tools/host_round_probe.py > gpurun_out/r4_host_probe.json 2> gpurun_out/r4_host_probe.err \
  || { tail -n 20 gpurun_out/r4_host_probe.err; exit 1; }
cat gpurun_out/r4_host_probe.json
echo "=== SCALE command shape at 8 gloo ranks on this one GPU (VERDICT r3 item 2)"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 8 --backend gloo --workers 256 --strong-workers 2048 --steps 5 --warmup 3 \
  > gpurun_out/r4_rehearsal8.json 2> gpurun_out/r4_rehearsal8.err || { tail -n 30 gpurun_out/r4_rehearsal8.err; exit 1; }
tail -n 1 gpurun_out/r4_rehearsal8.json | cut -c 1-400
echo "=== done"
