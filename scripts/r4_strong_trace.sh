#!/bin/bash
# Round 4: kernel traces of the phase path at the strong leg's rank shape (512 workers, C3 rows), RCCL
# world 1, collectives skipped and forced ("a rocprofv3 trace under profiles/
# shows the kernels per round"), plus the host probe with the collectives skipped.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
B="bench.py --no-cpu-baseline --no-secondary --scaling weak --phase --workers 512 --steps 50 --warmup 5"
echo "=== trace, collectives skipped"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_st1 -o run -- python3 $B \
  > gpurun_out/r4_st1.log 2>&1 || { tail -n 20 gpurun_out/r4_st1.log; exit 1; }
echo "=== trace, collectives forced"
DOPT_FORCE_COLLECTIVES=1 timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_st2 \
  -o run -- python3 $B > gpurun_out/r4_st2.log 2>&1 || { tail -n 20 gpurun_out/r4_st2.log; exit 1; }
echo "=== host probe, collectives skipped"
DOPT_FORCE_COLLECTIVES=0 timeout -k 10 200 python3 tools/host_round_probe.py > gpurun_out/r4_host_probe1.json \
  2> gpurun_out/r4_host_probe1.err || { tail -n 20 gpurun_out/r4_host_probe1.err; exit 1; }
cat gpurun_out/r4_host_probe1.json
python3 tools/trace_rounds.py gpurun_out/r4_st1/run_kernel_trace.csv > gpurun_out/r4_st1.txt && cat gpurun_out/r4_st1.txt
python3 tools/trace_rounds.py gpurun_out/r4_st2/run_kernel_trace.csv > gpurun_out/r4_st2.txt && cat gpurun_out/r4_st2.txt
echo "=== done"
