#!/bin/bash
# Paired row-dot butterflies in the row-space pass (DOPT_RS_PAIR=1, new build) vs the committed
# build (tools/_ab/libdopt_old.so), alternated in separate processes, x32 and float32 engines.
# (the baseline: `git stash; make -C distributed-optimization_amd/csrc; cp distributed-optimization_amd/libdopt.so
# tools/_ab/libdopt_old.so; git stash pop; make ...` -- the experiment was reverted, so both are gone)
mkdir -p gpurun_out
for rep in 1 2; do
  for eng in "--dtype float64 --data-dtype float32" "--dtype float32"; do
    tag=$(echo $eng | tr -d ' -' | cut -c 1-20)
    DOPT_LIB=tools/_ab/libdopt_old.so timeout -k 10 200 python -u tools/rs_ab.py $eng --reps 2 --shapes "2,6,2" \
      > gpurun_out/pair_old_${tag}_$rep.log 2>&1 || { tail -n 20 gpurun_out/pair_old_${tag}_$rep.log; exit 1; }
    echo "old $eng: $(tail -n 1 gpurun_out/pair_old_${tag}_$rep.log)"
    timeout -k 10 200 python -u tools/rs_ab.py $eng --reps 2 --shapes "2,6,2,1 2,6,2,0" \
      > gpurun_out/pair_new_${tag}_$rep.log 2>&1 || { tail -n 20 gpurun_out/pair_new_${tag}_$rep.log; exit 1; }
    echo "new $eng: $(tail -n 2 gpurun_out/pair_new_${tag}_$rep.log | tr '\n' ' ')"
  done
done
