#!/bin/bash
# Round 5: binary64 k_secb variants (table stream two h-steps ahead, Ab-table rows after the gather): bit identity + A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sparc_ldpc_amd
for v in libsparc_amp libsparc_amp_x21 libsparc_amp_x11 libsparc_amp_x211; do
  BITCMP_CASES=8,9,11,12 SPARC_AMP_LIB=$L/$v.so timeout -k 10 300 python scripts/bitcmp.py run gpurun_out/bc_$v.npz > gpurun_out/bc_$v.log 2>&1 || { echo "bitcmp $v failed"; tail -5 gpurun_out/bc_$v.log; exit 1; }
done
python scripts/bitcmp.py cmp gpurun_out/bc_libsparc_amp.npz gpurun_out/bc_libsparc_amp_x21.npz
python scripts/bitcmp.py cmp gpurun_out/bc_libsparc_amp.npz gpurun_out/bc_libsparc_amp_x11.npz
python scripts/bitcmp.py cmp gpurun_out/bc_libsparc_amp.npz gpurun_out/bc_libsparc_amp_x211.npz
WORKLOADS="c3 c4" bash scripts/ab.sh "--precision fp64 --no-fp64 --steps 10 --warmup 2" $L/libsparc_amp.so $L/libsparc_amp_x21.so $L/libsparc_amp_x211.so $L/libsparc_amp_x11.so $L/libsparc_amp.so $L/libsparc_amp_x21.so $L/libsparc_amp_x211.so
