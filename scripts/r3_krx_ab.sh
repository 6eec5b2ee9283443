#!/bin/bash
# x32 round-kernel variants, interleaved in one process (A/B library): DOPT_KRX_VARIANT values.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so timeout -k 10 240 python3 -u tools/kr_variants.py --mode x32 \
  --variants ${VARIANTS:-161827,161843} --reps ${REPS:-7} > gpurun_out/krx_ab.json 2> gpurun_out/krx_ab.err || { tail -n 20 gpurun_out/krx_ab.err; exit 1; }
cat gpurun_out/krx_ab.json
