#!/bin/bash
# BP: fused tail kernel and the fdlibm-structure log in Lxor.  Parity first
# (every GPU test that decodes LDPC), then BP / joint timing: ROCm log
# (libldpc_bp_ocml.so) with two-kernel and fused tails, and the new default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=sparc_ldpc_amd/libldpc_bp_ocml.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ldpc.py tests/test_gpu_joint.py tests/test_gpu_threshold.py tests/test_gpu_ber.py > gpurun_out/bp_parity.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/bp_parity.log; exit 1; }
tail -2 gpurun_out/bp_parity.log
LDPC_BP_LIB=$O timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ldpc.py > gpurun_out/bp_parity_ocml.log 2>&1 || { echo "ocml parity failed"; tail -30 gpurun_out/bp_parity_ocml.log; exit 1; }
tail -1 gpurun_out/bp_parity_ocml.log
for v in "$O|0" "$O|1" "sparc_ldpc_amd/libldpc_bp.so|1"; do
  lib=${v%|*}; fuse=${v#*|}
  echo "== $v"
  LDPC_BP_LIB=$lib LDPC_BP_TAIL_FUSE=$fuse timeout -k 10 300 python scripts/bp_time.py 1,256 || exit 1
  LDPC_BP_LIB=$lib LDPC_BP_TAIL_FUSE=$fuse timeout -k 10 300 python scripts/bench_joint.py --no-cpu > gpurun_out/joint_g.log 2>&1 || { echo "joint failed"; tail -5 gpurun_out/joint_g.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/joint_g.log').read().strip().splitlines()[-1]); print('joint', sys.argv[1], d['value'], d['ms_per_step'], d['step_share_ms'], d['bp']['launch_ms'], d['errors'])" "$v"
done
