#!/bin/bash
# Round 5: the big-n operator tests, then the binary64 k_secb variant A/B (run_r05h.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "big_n or maximum_sizes" > gpurun_out/pt_big.log 2>&1
rc=$?; tail -30 gpurun_out/pt_big.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash scripts/run_r05h.sh
