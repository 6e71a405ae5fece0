#!/bin/bash
# profiles at HEAD, part 2 (dense / matrix / joint), fp64 batched-kernel counters and stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/profile_r04.sh sq_c3f64 dense_l768 c3dense c2matrix c3matrix joint || exit 1
SPARC_AMP_PRECISION=fp64 SPARC_AMP_LIB=sparc_ldpc_amd/libsparc_amp_stamps.so timeout -k 10 120 python scripts/stamps.py c3 > gpurun_out/stamps_c3f64.txt 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/stamps_c3f64.txt; exit 1; }
cat gpurun_out/stamps_c3f64.txt | head -12
