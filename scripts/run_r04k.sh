#!/bin/bash
# Final-tree check: GPU suite, smoke(), and the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/gpu_suite_final.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/gpu_suite_final.log; exit 1; }
tail -1 gpurun_out/gpu_suite_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_default_final.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_default_final.log; exit 1; }
tail -1 gpurun_out/bench_default_final.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('default bench', d['value'], d['ms_per_step'], r['frac'], r.get('traffic_over_algorithmic'), r['trace']['profile_matches_build'], d['cpu_baseline']['gpu_over_cpu'], list(d['dense_gemv'])[:3])"
