#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/calib_r04.sh || exit 1
P=sparc_ldpc_amd/libsparc_amp_r03.so; N=sparc_ldpc_amd/libsparc_amp.so
WORKLOADS="c2 c3 c4" bash scripts/ab.sh "--steps 20 --warmup 3 --no-fp64" $P $N $P $N || exit 1
WORKLOADS="c3 c4" bash scripts/ab.sh "--steps 20 --warmup 3 --no-fp64 --plan WB8" $N || exit 1
WORKLOADS="c4" bash scripts/ab.sh "--steps 20 --warmup 3 --no-fp64 --plan ONE_PASS" $N || exit 1
WORKLOADS="c3 c4" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --precision fp64" $P $N || exit 1
WORKLOADS="c3" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --precision fp64 --plan WB16" $N || exit 1
WORKLOADS="c3" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --precision fp64 --plan ZIL" $N || exit 1
WORKLOADS="c3" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --precision fp64" sparc_ldpc_amd/libsparc_amp_khf1.so $N sparc_ldpc_amd/libsparc_amp_khf1.so || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
for lib in sparc_ldpc_amd/libldpc_bp_r03.so sparc_ldpc_amd/libldpc_bp.so; do
  echo "BP $lib"; LDPC_BP_LIB=$lib timeout -k 10 200 python scripts/bp_time.py 1,256 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ldpc.py tests/test_gpu_joint.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ldpc.log 2>&1; rc=$?; tail -3 gpurun_out/t_ldpc.log; exit $rc
