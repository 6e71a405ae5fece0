#!/bin/bash
# rocprofv3 summaries for a bench workload (run on the GPU box):
#   pass 1: --kernel-trace --stats        -> per-kernel durations
#   pass 2: --pmc FETCH_SIZE (own pass)   -> HBM read bytes per dispatch
#   pass 3: --pmc WRITE_SIZE (own pass)   -> HBM write bytes per dispatch
# Usage: bash scripts/profile.sh TAG [bench args...]
#        SCRIPT=scripts/bench_joint.py bash scripts/profile.sh TAG [args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# the identity of the build being profiled (bench.py compares it with its own)
python3 -c "from sparc_ldpc_amd._lib import source_hash; print(source_hash())" > $OUT/build.txt || exit 1
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- \
    python3 $SCRIPT "${EXTRA[@]}" "${BENCH_ARGS[@]}" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
BENCH_ARGS=("$@")
SCRIPT=${SCRIPT:-bench.py}
EXTRA=(--no-cpu)
[ "$SCRIPT" = bench.py ] && EXTRA+=(--no-dense --no-legs)
run trace --kernel-trace --stats && \
run fetch --kernel-trace --pmc FETCH_SIZE && \
run write --kernel-trace --pmc WRITE_SIZE
rc=$?
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cat "$f"
exit $rc
