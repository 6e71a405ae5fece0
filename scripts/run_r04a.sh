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
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
