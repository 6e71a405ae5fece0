#!/bin/bash
# GPU suite on the new binary64 defaults and the BP tail; then C4 k_secb
# traffic with smaller work-order passes (PMC), binary64 C3/C4 traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/gpu_suite.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/gpu_suite.log; exit 1; }
tail -2 gpurun_out/gpu_suite.log
prof() {
  local tag=$1; shift
  rm -rf "gpurun_out/prof_$tag"
  timeout -k 10 300 bash scripts/profile.sh "$tag" "$@" > "gpurun_out/prof_$tag.txt" 2>&1 || { echo "profile $tag failed"; tail -5 "gpurun_out/prof_$tag.txt"; exit 1; }
  python3 - "$tag" <<'PY'
import sys, os
sys.path.insert(0, "scripts")
from pmc_summary import counters
d = os.path.join("gpurun_out", "prof_" + sys.argv[1])
f, w = counters(os.path.join(d, "fetch"), "FETCH_SIZE"), counters(os.path.join(d, "write"), "WRITE_SIZE")
for k in sorted(set(f) | set(w)):
    if k.startswith(("k_sec", "k_row")):
        print(sys.argv[1], k, "read MB (x2)", round(2 * f.get(k, 0) * 1024 / 1e6, 1), "write MB", round(w.get(k, 0) * 1024 / 1e6, 1))
PY
}
prof c4 --workload c4 --steps 3 --warmup 1 --no-fp64
SPARC_AMP_SECB_L2_KB=1700 prof c4l2a --workload c4 --steps 3 --warmup 1 --no-fp64
SPARC_AMP_SECB_L2_KB=900 prof c4l2b --workload c4 --steps 3 --warmup 1 --no-fp64
prof c3f64 --workload c3 --precision fp64 --steps 3 --warmup 1
