#!/bin/bash
# Round 5: the full-size parity tests with every section pinned, then the
# joint step with staggered concurrent slices (2, 3, 4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n ${TAILN:-6} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit in $name: stopping"; exit $rc; fi
  return 0
}
TAILN=30 step pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "golden or batch256"
for p in 2 3 4; do
  step bench_joint_p$p 400 python scripts/bench_joint.py --no-cpu --steps 3 --parts $p
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_joint_p$p.log').read().strip().splitlines()[-1]); print('parts', $p, d['value'], d['ms_per_step'])"
done
