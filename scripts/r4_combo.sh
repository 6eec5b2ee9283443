#!/bin/bash
# Round 4: scripts/r4_strong_trace.sh, scripts/r4_ab8.sh, then scripts/r4_full.sh (one box for all).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/r4_strong_trace.sh || exit $?
bash scripts/r4_ab8.sh || exit $?
bash scripts/r4_full.sh
