#!/bin/bash
# profiles at HEAD (part 1) and fp64 batched-kernel diagnostics
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
N=sparc_ldpc_amd/libsparc_amp.so
WORKLOADS="c3" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --precision fp64" sparc_ldpc_amd/libsparc_amp_khf1.so $N sparc_ldpc_amd/libsparc_amp_khf1.so $N || exit 1
bash scripts/profile_r04.sh c4 c3f64 c3 c2 c2f64 c4b1 sq_c3f64 || exit 1
rm -rf gpurun_out/prof_c4onepass
timeout -k 10 600 bash scripts/profile.sh c4onepass --workload c4 --steps 3 --warmup 1 --no-fp64 --plan ONE_PASS > gpurun_out/prof_c4onepass.txt 2>&1 || { echo "c4onepass failed"; exit 1; }
SPARC_AMP_PRECISION=fp64 SPARC_AMP_LIB=sparc_ldpc_amd/libsparc_amp_stamps.so timeout -k 10 120 python scripts/stamps.py c3 > gpurun_out/stamps_c3f64.txt 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/stamps_c3f64.txt; exit 1; }
head -12 gpurun_out/stamps_c3f64.txt
for t in c4 c4onepass c3f64 c3; do python3 scripts/pmc_summary.py $t rtmp x_$t > /dev/null && echo "$t $(python3 -c "import json;d=json.load(open('profiles/rtmp_${t}_pmc.json'));print({k:v['hbm_bytes_per_launch'] for k,v in d.items() if k.startswith(('k_sec','k_row'))})")"; done
