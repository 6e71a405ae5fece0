#!/bin/bash
# Round 5: parity suites on a variant library, then interleaved A/B against
# the default (fp32 c3 c4, fp64 c3 c4).  VAR=libsparc_amp_cp (default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sparc_ldpc_amd
V=${VAR:-libsparc_amp_cp}
SPARC_AMP_LIB=$L/$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_joint.py tests/test_gpu_amp_test_reps.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_$V.log 2>&1 || { echo "parity $V failed"; tail -30 gpurun_out/par_$V.log; exit 1; }
tail -1 gpurun_out/par_$V.log
for r in 1 2; do
  WORKLOADS="c3 c4" bash scripts/ab.sh "--steps 8 --warmup 2 --no-fp64" $L/libsparc_amp.so $L/$V.so || exit 1
  WORKLOADS="c3 c4" bash scripts/ab.sh "--steps 6 --warmup 2 --no-fp64 --precision fp64" $L/libsparc_amp.so $L/$V.so || exit 1
done
