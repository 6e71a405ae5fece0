#!/bin/bash
# Round 5: kernel traces of the joint step, one decoder vs two staggered slices.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 1 2; do
  rm -rf gpurun_out/jt_p$p
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/jt_p$p -o jt --output-format csv -- python3 scripts/bench_joint.py --no-cpu --steps 1 --warmup 1 --parts $p > gpurun_out/jt_p$p.log 2>&1 || { echo "trace $p failed"; tail -5 gpurun_out/jt_p$p.log; exit 1; }
  f=$(find gpurun_out/jt_p$p -name "*kernel_trace.csv" | head -1)
  echo "parts $p"; python3 scripts/joint_timeline.py "$f" 0.75
  tail -c 300 gpurun_out/jt_p$p.log
done
