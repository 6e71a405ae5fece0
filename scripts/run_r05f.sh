#!/bin/bash
# Round 5: joint step, BP with and without the tail launches, one decoder and two slices.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in "8 2" "0 2" "8 1" "0 1"; do
  set -- $cfg
  LDPC_BP_TAIL=$1 timeout -k 10 300 python scripts/bench_joint.py --no-cpu --steps 3 --parts $2 > gpurun_out/bj_t$1_p$2.log 2>&1 || { echo "failed"; tail -5 gpurun_out/bj_t$1_p$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bj_t$1_p$2.log').read().strip().splitlines()[-1]); print('tail', $1, 'parts', $2, d['value'], d['ms_per_step'], d['bp']['launch_ms'])"
done
done
