#!/bin/bash
# Round 4: the headline instance with 8 waves per workgroup (VAR bit 8: two generations of
# workgroups at the strong leg's 512 workers per rank) vs the default, interleaved in one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for w in 512 1024 4096; do
  echo "=== 8-wave A/B, $w workers"
  DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so timeout -k 10 200 python3 tools/kr_variants.py --mode x32 \
    --variants=-1,1210675 --reps 7 --rounds 20 --workers $w > gpurun_out/r4_ab8_$w.json 2> gpurun_out/r4_ab8_$w.err \
    || { tail -n 20 gpurun_out/r4_ab8_$w.err; exit 1; }
  cat gpurun_out/r4_ab8_$w.json
done
