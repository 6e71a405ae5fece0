#!/bin/bash
# Round 5: binary64 variant (VAR) — parity suites, then interleaved A/B
# (fp64 c3 c4) and the joint step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sparc_ldpc_amd
V=${VAR:-libsparc_amp_xt}
SPARC_AMP_LIB=$L/$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_joint.py tests/test_gpu_amp_test_reps.py tests/test_gpu_ber.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_$V.log 2>&1 || { echo "parity $V failed"; tail -30 gpurun_out/par_$V.log; exit 1; }
tail -1 gpurun_out/par_$V.log
for r in 1 2; do
  WORKLOADS="c3 c4" bash scripts/ab.sh "--steps 6 --warmup 2 --no-fp64 --precision fp64" $L/libsparc_amp.so $L/$V.so || exit 1
  for lib in libsparc_amp $V; do
    SPARC_AMP_LIB=$L/$lib.so timeout -k 10 300 python scripts/bench_joint.py --no-cpu > gpurun_out/bjq.log 2>&1 || { tail -5 gpurun_out/bjq.log; exit 1; }
    grep "^{" gpurun_out/bjq.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('joint $lib', d['value'], d['ms_per_step'], d['errors'])"
  done
done
