#!/bin/bash
# Final sources: GPU suite, then the first profile set
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/gpu_suite_m.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/gpu_suite_m.log; exit 1; }
tail -1 gpurun_out/gpu_suite_m.log
bash scripts/profile_r04.sh c2 c2f64 c4b1 c3 c3f64 c4
