#!/bin/bash
# Round 5: the GPU suite and the bench lines at the current sources.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n ${TAILN:-3} "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit in $name: stopping"; exit $rc; fi
  return 0
}
TAILN=8 step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
for w in c2 c3; do
  step bench_$w 400 python bench.py --workload $w --no-cpu --no-dense
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_$w.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['frac_dispatch'], r['frac_events'], d['decode_only']['value'], d.get('fp64_leg',{}).get('value'))"
done
step bench_joint 400 python scripts/bench_joint.py --no-cpu --steps 3
python3 -c "import json; d=json.loads(open('gpurun_out/bench_joint.log').read().strip().splitlines()[-1]); print('joint', d['value'], d['ms_per_step'], d['roofline']['frac'], d['step_share_ms'])"
