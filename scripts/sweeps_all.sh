#!/bin/bash
# Every BER / EXIT sweep of the results/ directory (run on the GPU box), next to
# the reference's published curves: plain, the joint soft / hard / originalHard
# waterfalls (configs[4]), the threshold-initialised sweeps (0.6 / 0.8, with
# and without unit cancellation), soft_hard_plot's BER_sparc column (l768,
# configs[3], the refilled stream) and the threshold EXIT curve.  Each step has
# its own time limit; stops at the first abnormal exit.  Outputs
# gpurun_out/sweeps/<name>.json (+ .csv).
#   bash scripts/sweeps_all.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sweeps
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/sweeps/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 gpurun_out/sweeps/$name.log)"
  [ $rc -eq 0 ] || exit $rc
}
O=gpurun_out/sweeps
run waterfall_plain 300 python scripts/waterfall.py --sweep plain --out $O/waterfall_plain
run waterfall_soft 300 python scripts/waterfall.py --sweep soft --out $O/waterfall_soft
run waterfall_hard 300 python scripts/waterfall.py --sweep hard --out $O/waterfall_hard
run waterfall_originalHard 300 python scripts/waterfall.py --sweep originalHard --out $O/waterfall_originalHard
run waterfall_threshold06 300 python scripts/waterfall.py --sweep threshold --threshold 0.6 --out $O/waterfall_threshold06
run waterfall_threshold06_unitcancel 300 python scripts/waterfall.py --sweep threshold --threshold 0.6 --unit-cancel --out $O/waterfall_threshold06_unitcancel
run waterfall_threshold08 300 python scripts/waterfall.py --sweep threshold --threshold 0.8 --out $O/waterfall_threshold08
run waterfall_threshold08_unitcancel 300 python scripts/waterfall.py --sweep threshold --threshold 0.8 --unit-cancel --out $O/waterfall_threshold08_unitcancel
run soft_hard_l768 300 python scripts/waterfall.py --sweep soft_hard --out $O/soft_hard_l768
run waterfall_l768 300 python scripts/waterfall.py --sweep l768 --out $O/waterfall_l768
run exit_curve_L256M32_t07 300 python scripts/exit_curve.py --out $O/exit_curve_L256M32_t07
echo "all ok"
