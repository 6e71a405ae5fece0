#!/bin/bash
# Round 5: the BP tail's wave issue priority beside the other slice's AMP (A/B), and a trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for wp in 1 0; do
  LDPC_BP_WAVE_PRIO=$wp timeout -k 10 300 python scripts/bench_joint.py --no-cpu --steps 3 --parts 2 > gpurun_out/bj_wp$wp.log 2>&1 || { echo "failed"; tail -5 gpurun_out/bj_wp$wp.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bj_wp$wp.log').read().strip().splitlines()[-1]); print('wave prio', $wp, d['value'], d['ms_per_step'], d['bp']['launch_ms'])"
done
done
rm -rf gpurun_out/jt_wp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/jt_wp -o jt --output-format csv -- python3 scripts/bench_joint.py --no-cpu --steps 1 --warmup 0 --no-ref --parts 2 > gpurun_out/jt_wp.log 2>&1 || { echo "trace failed"; exit 1; }
python3 scripts/joint_timeline.py $(find gpurun_out/jt_wp -name "*kernel_trace.csv" | head -1)
