#!/bin/bash
# Round 5: k_secb variants (table stream two h-steps ahead and Ab-table rows
# after the gather in binary64; the gather's sign per loop in the bank-aware
# order): bit identity + interleaved A/B at c3 (both precisions) and c4 fp64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sparc_ldpc_amd
V="libsparc_amp libsparc_amp_xg libsparc_amp_xg11 libsparc_amp_xgs libsparc_amp_x21 libsparc_amp_x211"
for v in $V; do
  BITCMP_CASES=0,3,8,9,11,12 SPARC_AMP_LIB=$L/$v.so timeout -k 10 300 python scripts/bitcmp.py run gpurun_out/bc_$v.npz > gpurun_out/bc_$v.log 2>&1 || { echo "bitcmp $v failed"; tail -5 gpurun_out/bc_$v.log; exit 1; }
  [ $v != libsparc_amp ] && python scripts/bitcmp.py cmp gpurun_out/bc_libsparc_amp.npz gpurun_out/bc_$v.npz | tail -3
done
for rep in 1 2; do
  WORKLOADS="c3" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64" $L/libsparc_amp.so $L/libsparc_amp_xg.so
  WORKLOADS="c3 c4" bash scripts/ab.sh "--precision fp64 --no-fp64 --steps 8 --warmup 2" $L/libsparc_amp.so $L/libsparc_amp_xg11.so $L/libsparc_amp_xgs.so $L/libsparc_amp_x21.so $L/libsparc_amp_x211.so
done
