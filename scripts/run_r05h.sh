#!/bin/bash
# Round 5: k_secb variants — the gather's sign per loop in the bank-aware
# order (xg), binary64 Ab-table rows after the gather (l) and tau_{t-1}
# through the scalar cache (s): bit identity against the default build, then
# interleaved A/B at c3 (both precisions) and c4 binary64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sparc_ldpc_amd
V="libsparc_amp libsparc_amp_xg libsparc_amp_xgl libsparc_amp_xgls libsparc_amp_xls"
for v in $V; do
  BITCMP_CASES=0,1,3,8,9,11,12 SPARC_AMP_LIB=$L/$v.so timeout -k 10 300 python scripts/bitcmp.py run /tmp/bc_$v.npz > gpurun_out/bc_$v.log 2>&1 || { echo "bitcmp $v failed"; tail -5 gpurun_out/bc_$v.log; exit 1; }
  [ $v != libsparc_amp ] && { echo "== $v"; python scripts/bitcmp.py cmp /tmp/bc_libsparc_amp.npz /tmp/bc_$v.npz | grep -v identical; }
done
for rep in 1 2; do
  WORKLOADS="c3 c4" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64" $L/libsparc_amp.so $L/libsparc_amp_xg.so
  WORKLOADS="c3 c4" bash scripts/ab.sh "--precision fp64 --no-fp64 --steps 8 --warmup 2" $L/libsparc_amp.so $L/libsparc_amp_xg.so $L/libsparc_amp_xgl.so $L/libsparc_amp_xgls.so $L/libsparc_amp_xls.so
done
