#!/bin/bash
# One GPU session of round-6 checks (run on the GPU box): the whole -m gpu
# suite, the configs[3] l768 10 k-rep sweep twice (one refilled stream), and
# the default bench line.  Each step has its own time limit; the script stops
# at the first abnormal exit (fault, abort, time limit).  Summaries on stdout,
# logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit in $name: stopping"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  tail -3 gpurun_out/pytest_gpu.log
fi
for i in 1 2; do
  step wf_l768_$i 300 python scripts/waterfall.py --sweep l768 --reps 1000 --out gpurun_out/wf_l768_$i
  python3 -c "import json; d=json.load(open('gpurun_out/wf_l768_$i.json')); s=d['split']; print('sweep', round(d['seconds'], 3), 's', {k: (round(v, 4) if isinstance(v, float) else v) for k, v in s.items() if k != 'stream_phases'})"
done
step bp_empty_tail 200 python scripts/bp_empty_tail.py
cat gpurun_out/bp_empty_tail.log
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  step bench 500 python bench.py
  tail -1 gpurun_out/bench.log > gpurun_out/bench.json
  python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench.json"))
print("headline", d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"])
print("fp64_leg", d["fp64_leg"]["value"], d["fp64_leg"]["roofline"]["frac"])
for k, v in d.get("batched_legs", {}).items():
    print(k, v["value"], v["ms_per_step"], v["roofline"]["kernel"], v["roofline"]["frac"])
print("mc", {k: v for k, v in d.get("mc_stream", {}).items() if k not in ("workload", "note")})
j = d.get("joint_leg", {})
print("joint", j.get("value"), j.get("ms_per_step"), j.get("identical_to_one_decoder"), j.get("roofline", {}).get("kernel"), j.get("roofline", {}).get("frac"), j.get("step_share_ms"))
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["gpu_over_cpu"])
PY
fi
