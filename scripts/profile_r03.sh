#!/bin/bash
# Round-3 profile set (run on the GPU box): for every headline kernel a
# rocprofv3 kernel trace with --stats and separate FETCH_SIZE / WRITE_SIZE
# passes (scripts/profile.sh), SQ / TCC counter passes (scripts/pmc_sq.sh) and
# s_memtime phase stamps of the section kernels.  Raw output under
# gpurun_out/; scripts/collect_profiles.py copies the summaries to profiles/.
# Stops at the first step that fails.
#   bash scripts/profile_r03.sh [STEP ...]   (default: every step; steps:
#   c2 c4b1 c3 dense_l768 c3dense sq_c2 sq_c3 sq_c3dense stamps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
prof() {  # tag, bench args...
  local tag=$1; shift
  rm -rf "gpurun_out/prof_$tag"
  timeout -k 10 600 bash scripts/profile.sh "$tag" "$@" > "gpurun_out/prof_$tag.txt" 2>&1 || { echo "profile $tag failed"; exit 1; }
  echo "profile $tag ok"
}
sq() {  # tag, bench args...
  local tag=$1; shift
  rm -rf "gpurun_out/sq_$tag"
  timeout -k 10 900 bash scripts/pmc_sq.sh "$tag" "$@" > "gpurun_out/sq_$tag.txt" 2>&1 || { echo "sq $tag failed"; exit 1; }
  echo "sq $tag ok"
}
stamps() {
  export SPARC_AMP_LIB=sparc_ldpc_amd/libsparc_amp_stamps.so
  timeout -k 10 120 python scripts/stamps.py c2 > gpurun_out/stamps_c2.txt 2>&1 || { echo "stamps c2 failed"; exit 1; }
  timeout -k 10 120 python scripts/stamps.py c4 1 > gpurun_out/stamps_c4b1.txt 2>&1 || { echo "stamps c4b1 failed"; exit 1; }
  timeout -k 10 120 python scripts/stamps.py c3 > gpurun_out/stamps_c3.txt 2>&1 || { echo "stamps c3 failed"; exit 1; }
  unset SPARC_AMP_LIB
  echo "stamps ok"
}
STEPS=${*:-c2 c4b1 c3 c4 dense_l768 c3dense sq_c2 sq_c3 sq_c3dense stamps}
for s in $STEPS; do
  case $s in
    c2) prof c2 --steps 20 --warmup 3 --no-fp64 ;;
    c4b1) prof c4b1 --workload c4 --batch 1 --steps 20 --warmup 3 --no-fp64 ;;
    c3) prof c3 --workload c3 --steps 5 --warmup 1 --no-fp64 ;;
    c4) prof c4 --workload c4 --steps 3 --warmup 1 --no-fp64 ;;
    dense_l768) prof dense_l768 --workload c4 --batch 1 --backend dense --steps 2 --warmup 1 ;;
    c3dense) prof c3dense --workload c3 --backend dense --steps 2 --warmup 1 ;;
    sq_c2) sq c2 --no-fp64 --steps 5 --warmup 1 ;;
    sq_c3) sq c3 --workload c3 --no-fp64 --steps 1 --warmup 0 ;;
    sq_c3dense) sq c3dense --workload c3 --backend dense --steps 1 --warmup 0 ;;
    stamps) stamps ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all ok"
