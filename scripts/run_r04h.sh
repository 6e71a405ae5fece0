#!/bin/bash
# BP: branch-free fdlibm-structure log; parity, then two-kernel vs fused tail
# (timing + kernel traces of the joint step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ldpc.py tests/test_gpu_joint.py tests/test_gpu_threshold.py tests/test_gpu_ber.py > gpurun_out/bp_parity.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/bp_parity.log; exit 1; }
tail -1 gpurun_out/bp_parity.log
for fuse in 0 1; do
  echo "== fuse $fuse"
  LDPC_BP_TAIL_FUSE=$fuse timeout -k 10 300 python scripts/bp_time.py 1,256 || exit 1
  LDPC_BP_TAIL_FUSE=$fuse timeout -k 10 300 python scripts/bench_joint.py --no-cpu > gpurun_out/joint_h.log 2>&1 || { echo "joint failed"; tail -5 gpurun_out/joint_h.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/joint_h.log').read().strip().splitlines()[-1]); print('joint', sys.argv[1], d['value'], d['ms_per_step'], d['step_share_ms'], d['bp']['launch_ms'], d['errors'])" "$fuse"
  rm -rf gpurun_out/jtr$fuse
  LDPC_BP_TAIL_FUSE=$fuse timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/jtr$fuse -o jtr --output-format csv -- python3 scripts/bench_joint.py --no-cpu --steps 1 --warmup 1 > gpurun_out/jtr$fuse.log 2>&1 || { echo "joint trace failed"; tail -5 gpurun_out/jtr$fuse.log; exit 1; }
  python3 scripts/bp_tail_trace.py gpurun_out/jtr$fuse | tail -6
  find gpurun_out/jtr$fuse -name "*kernel_trace.csv" -size +20M -delete
done
