#!/bin/bash
# Round-5 first GPU session: the GPU suite, the default bench line (decision in
# the step, dispatch-bound roofline timing), the joint configs[4] step with two
# concurrent halves.  Stops at the first abnormal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit in $name: stopping"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS}
step bench_c2 400 python bench.py --steps 20 --warmup 3 --no-dense
step bench_joint 400 python scripts/bench_joint.py --no-cpu --steps 3
step bench_joint1 400 python scripts/bench_joint.py --no-cpu --steps 3 --parts 1
