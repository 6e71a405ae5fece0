#!/bin/bash
# rocprofv3 kernel-trace summaries for the bench workloads (run on the GPU box).
# Usage: bash scripts/profile.sh TAG [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o $TAG --output-format csv -- \
  python3 bench.py --no-cpu --no-dense "$@" > $OUT/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -n 2 $OUT/bench.log | cut -c1-600
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cat "$f"
exit $rc
