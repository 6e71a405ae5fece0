#!/bin/bash
# One GPU session: smoke, GPU parity tests, a short bench.  Stops at the first
# step that ends abnormally (fault / abort / timeout); plain test failures
# (exit 1) do not stop the later steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit in $name: stopping"; exit $rc; fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS}
step bench 600 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS}
if [ -n "$EXTRA_BENCH" ]; then step bench_extra 600 python bench.py $EXTRA_BENCH; fi
