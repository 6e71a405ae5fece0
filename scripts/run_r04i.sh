#!/bin/bash
# BP: lane-pair check kernel in the tail; parity, BP / joint timing, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ldpc.py tests/test_gpu_joint.py tests/test_gpu_threshold.py tests/test_gpu_ber.py > gpurun_out/bp_parity.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/bp_parity.log; exit 1; }
tail -1 gpurun_out/bp_parity.log
timeout -k 10 300 python scripts/bp_time.py 1,256 || exit 1
timeout -k 10 300 python scripts/bench_joint.py --no-cpu > gpurun_out/joint_i.log 2>&1 || { echo "joint failed"; tail -5 gpurun_out/joint_i.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/joint_i.log').read().strip().splitlines()[-1]); print('joint', d['value'], d['ms_per_step'], d['step_share_ms'], d['bp']['launch_ms'], d['errors'])"
rm -rf gpurun_out/jtri
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/jtri -o jtr --output-format csv -- python3 scripts/bench_joint.py --no-cpu --steps 1 --warmup 1 > gpurun_out/jtri.log 2>&1 || { echo "joint trace failed"; tail -5 gpurun_out/jtri.log; exit 1; }
python3 scripts/bp_tail_trace.py gpurun_out/jtri | tail -6
find gpurun_out/jtri -name "*kernel_trace.csv" -size +20M -delete
