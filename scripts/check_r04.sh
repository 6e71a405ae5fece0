#!/bin/bash
# Round-4 check on the GPU box: bit-identity of the current build against the
# round-3 library (scripts/bitcmp.py), the GPU test suite, then an A/B of the
# two builds at c2 / c3 / c4.  Stops at the first abnormal step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=sparc_ldpc_amd/libsparc_amp_r03.so; N=sparc_ldpc_amd/libsparc_amp.so
if [ -z "$NO_BITCMP" ]; then
  SPARC_AMP_LIB=$P timeout -k 10 300 python scripts/bitcmp.py run gpurun_out/bc_prev.npz > gpurun_out/bc_prev.log 2>&1 || { echo "bitcmp prev failed"; tail -5 gpurun_out/bc_prev.log; exit 1; }
  timeout -k 10 300 python scripts/bitcmp.py run gpurun_out/bc_new.npz > gpurun_out/bc_new.log 2>&1 || { echo "bitcmp new failed"; tail -5 gpurun_out/bc_new.log; exit 1; }
  python scripts/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz | tail -3
fi
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/t_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/t_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$NO_AB" ]; then
  WORKLOADS=${WORKLOADS:-"c2 c3 c4"} bash scripts/ab.sh "--steps 20 --warmup 3 --no-fp64" $P $N $P $N || exit 1
fi
