#!/bin/bash
# Before the final profiles: the whole GPU suite (lane-pair BP tail, binary64
# defaults), BP / joint timing with a kernel trace, and C4 k_secb traffic with
# smaller work-order passes (PMC)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/gpu_suite.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/gpu_suite.log; exit 1; }
tail -1 gpurun_out/gpu_suite.log
timeout -k 10 300 python scripts/bp_time.py 1,256 || exit 1
timeout -k 10 300 python scripts/bench_joint.py --no-cpu > gpurun_out/joint_j.log 2>&1 || { echo "joint failed"; tail -5 gpurun_out/joint_j.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/joint_j.log').read().strip().splitlines()[-1]); print('joint', d['value'], d['ms_per_step'], d['step_share_ms'], d['bp']['launch_ms'], d['errors'])"
rm -rf gpurun_out/jtrj
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/jtrj -o jtr --output-format csv -- python3 scripts/bench_joint.py --no-cpu --steps 1 --warmup 1 > gpurun_out/jtrj.log 2>&1 || { echo "joint trace failed"; tail -5 gpurun_out/jtrj.log; exit 1; }
python3 scripts/bp_tail_trace.py gpurun_out/jtrj | tail -6
find gpurun_out/jtrj -name "*kernel_trace.csv" -size +20M -delete
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
  grep -h "k_secb" "gpurun_out/prof_$tag/trace/"*/*kernel_stats.csv 2>/dev/null | head -2 || true
}
prof c4x --workload c4 --steps 3 --warmup 1 --no-fp64
SPARC_AMP_SECB_L2_KB=1700 prof c4l2a --workload c4 --steps 3 --warmup 1 --no-fp64
SPARC_AMP_SECB_L2_KB=900 prof c4l2b --workload c4 --steps 3 --warmup 1 --no-fp64
