#!/bin/bash
# BP tail diagnostic: kernel traces of bp_time (B=256) and the joint step with the tail at 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/bptr gpurun_out/jtr
LDPC_BP_TAIL=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bptr -o bptr --output-format csv -- python3 scripts/bp_time.py 256 > gpurun_out/bptr.log 2>&1 || { echo "bp trace failed"; tail -5 gpurun_out/bptr.log; exit 1; }
cat gpurun_out/bptr.log | grep "B="
python3 scripts/bp_tail_trace.py gpurun_out/bptr
LDPC_BP_TAIL=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/jtr -o jtr --output-format csv -- python3 scripts/bench_joint.py --no-cpu --steps 1 --warmup 1 > gpurun_out/jtr.log 2>&1 || { echo "joint trace failed"; tail -5 gpurun_out/jtr.log; exit 1; }
python3 scripts/bp_tail_trace.py gpurun_out/jtr
find gpurun_out/bptr gpurun_out/jtr -name "*kernel_trace.csv" -size +20M -delete
