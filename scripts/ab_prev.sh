#!/bin/bash
# A/B of the current library against sparc_ldpc_amd/libsparc_amp_prev.so (the
# previous build, copied before a rebuild) at c2, C4 single codeword and c2
# binary64, two interleaved rounds each; then the GPU parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=sparc_ldpc_amd/libsparc_amp.so; P=sparc_ldpc_amd/libsparc_amp_prev.so
bash scripts/ab.sh "--steps 30 --warmup 3 --no-fp64" $P $N $P $N || exit 1
WORKLOADS=c4 bash scripts/ab.sh "--batch 1 --steps 30 --warmup 3 --no-fp64" $P $N $P $N || exit 1
bash scripts/ab.sh "--precision fp64 --steps 30 --warmup 3 --no-fp64" $P $N $P $N || exit 1
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/t_ab.log 2>&1; rc=$?; tail -3 gpurun_out/t_ab.log; exit $rc
