#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes (one counter group per pass; no trace domains with --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-secondary --steps ${PSTEPS:-10} --warmup ${PWARM:-1} ${BENCH_ARGS:-}"
run() {  # run <name> <timeout> <args...>
  local name=$1 t=$2; shift 2
  echo "=== $name"; timeout -s KILL "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -n 3 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- $B
run fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $B
run write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $B
echo "=== done"
