#!/bin/bash
# The C5 row-space pass's access pattern alone vs with its arithmetic (tools/rs_probe.hip).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 ./tools/rs_probe > gpurun_out/rs_probe.txt 2>&1; rc=$?
cat gpurun_out/rs_probe.txt; exit $rc
