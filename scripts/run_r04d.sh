#!/bin/bash
# LDPC BP tail launches: parity (GPU LDPC tests), BP timing and the joint
# configs[4] step with the tail off / at 8 / 16 / 24 iterations (binary64 AMP
# on its new default plan: WB16 at equal CB + ZIL)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ldpc.py > gpurun_out/ldpc_tail_tests.log 2>&1 || { echo "ldpc tests failed"; tail -30 gpurun_out/ldpc_tail_tests.log; exit 1; }
tail -2 gpurun_out/ldpc_tail_tests.log
for at in 0 8 16; do
  echo "== bp_time tail $at"
  LDPC_BP_TAIL=$at timeout -k 10 300 python scripts/bp_time.py 1,256 || exit 1
done
for at in 0 8 16; do
  LDPC_BP_TAIL=$at timeout -k 10 300 python scripts/bench_joint.py --no-cpu > gpurun_out/joint_tail.log 2>&1 || { echo "joint failed"; tail -5 gpurun_out/joint_tail.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/joint_tail.log').read().strip().splitlines()[-1]); print('joint tail', sys.argv[1], d['value'], d['ms_per_step'], d['step_share_ms'], d['bp'])" "$at"
done
