#!/bin/bash
# The profile set of a round (run on the GPU box): per headline workload a rocprofv3
# kernel trace with --stats and separate FETCH_SIZE / WRITE_SIZE passes
# (scripts/profile.sh, which records the sources hash of the build), optional
# SQ counter passes (scripts/pmc_sq.sh) and the PMC calibration probe.  Raw
# output under gpurun_out/; scripts/collect_profiles.py rNN copies the
# summaries to profiles/rNN_*.  Stops at the first step that fails.
#   bash scripts/profile_set.sh STEP ...
#   steps: c2 c2f64 c4b1 c3 c3f64 c4 c4f64 joint dense_l768 c3dense c2matrix c3matrix
#          sq_c2 sq_c3 sq_c4 sq_c3f64 sq_bp calib mc
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
prof() {  # tag, bench args...
  local tag=$1; shift
  rm -rf "gpurun_out/prof_$tag"
  timeout -k 10 600 bash scripts/profile.sh "$tag" "$@" > "gpurun_out/prof_$tag.txt" 2>&1 || { echo "profile $tag failed"; tail -5 "gpurun_out/prof_$tag.txt"; exit 1; }
  echo "profile $tag ok"
}
sq() {  # tag, bench args...
  local tag=$1; shift
  rm -rf "gpurun_out/sq_$tag"
  timeout -k 10 900 bash scripts/pmc_sq.sh "$tag" "$@" > "gpurun_out/sq_$tag.txt" 2>&1 || { echo "sq $tag failed"; exit 1; }
  echo "sq $tag ok"
}
for s in "$@"; do
  case $s in
    c2) prof c2 --steps 20 --warmup 3 --no-fp64 ;;
    c2f64) prof c2f64 --precision fp64 --steps 20 --warmup 3 ;;
    c4b1) prof c4b1 --workload c4 --batch 1 --steps 20 --warmup 3 --no-fp64 ;;
    c3) prof c3 --workload c3 --steps 5 --warmup 1 --no-fp64 ;;
    c3f64) prof c3f64 --workload c3 --precision fp64 --steps 3 --warmup 1 ;;
    c4) prof c4 --workload c4 --steps 3 --warmup 1 --no-fp64 ;;
    c4f64) prof c4f64 --workload c4 --precision fp64 --steps 2 --warmup 1 ;;
    joint) SCRIPT=scripts/bench_joint.py prof joint --steps 1 --warmup 1 ;;
    dense_l768) prof dense_l768 --workload c4 --batch 1 --backend dense --steps 2 --warmup 1 ;;
    c3dense) prof c3dense --workload c3 --backend dense --steps 2 --warmup 1 ;;
    c2matrix) prof c2matrix --backend matrix --steps 3 --warmup 1 --no-fp64 ;;
    c3matrix) prof c3matrix --workload c3 --backend matrix --steps 1 --warmup 1 --no-fp64 ;;
    sq_c2) sq c2 --no-fp64 --steps 5 --warmup 1 ;;
    sq_c3) sq c3 --workload c3 --no-fp64 --steps 1 --warmup 0 ;;
    sq_c4) sq c4 --workload c4 --no-fp64 --steps 1 --warmup 0 ;;
    sq_c3f64) sq c3f64 --workload c3 --precision fp64 --steps 1 --warmup 0 ;;
    sq_bp) SCRIPT=scripts/bp_time.py sq bp 256 ;;
    calib) bash scripts/pmc_calib.sh || exit 1 ;;
    mc)  # the configs[3] rep stream (kernel trace only; the stream's kernels are the batched ones + k_mc_*)
      rm -rf gpurun_out/prof_mc
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mc -o mc --output-format csv -- \
        python3 scripts/waterfall.py --sweep l768 --reps 1000 --out /tmp/wf_prof > gpurun_out/prof_mc.txt 2>&1 \
        || { echo "profile mc failed"; exit 1; }
      echo "profile mc ok" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all ok"
