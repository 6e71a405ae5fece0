#!/bin/bash
# Round 5: the joint step's BP stream priority (A/B) with 2 staggered slices.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for pr in 1 0; do
  LDPC_BP_PRIORITY=$pr timeout -k 10 300 python scripts/bench_joint.py --no-cpu --steps 3 --parts 2 > gpurun_out/bj_pr$pr.log 2>&1 || { echo "failed"; tail -5 gpurun_out/bj_pr$pr.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bj_pr$pr.log').read().strip().splitlines()[-1]); print('prio', $pr, d['value'], d['ms_per_step'])"
done
done
timeout -k 10 300 python scripts/bench_joint.py --no-cpu --steps 3 --parts 1 > gpurun_out/bj_p1.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bj_p1.log').read().strip().splitlines()[-1]); print('parts 1', d['value'], d['ms_per_step'])"
