#!/bin/bash
# tests -> bench -> C5 -> profiles (stats + separate FETCH_SIZE / WRITE_SIZE passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS="${STEPS:-tests bench c5}" bash scripts/gpu_check.sh || exit $?
OUT=gpurun_out/prof bash scripts/profile.sh
