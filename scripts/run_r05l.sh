#!/bin/bash
# Round 5: binary64 k_secb with the previous estimate loaded after the gather
# (xb1) and then two bucket h-steps in flight (xb2): bit identity + A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sparc_ldpc_amd
for v in libsparc_amp libsparc_amp_xb1 libsparc_amp_xb2; do
  BITCMP_CASES=8,9,11 SPARC_AMP_LIB=$L/$v.so timeout -k 10 300 python scripts/bitcmp.py run /tmp/bc_$v.npz > gpurun_out/bc_$v.log 2>&1 || { echo "bitcmp $v failed"; tail -5 gpurun_out/bc_$v.log; exit 1; }
  [ $v != libsparc_amp ] && { echo "== $v"; python scripts/bitcmp.py cmp /tmp/bc_libsparc_amp.npz /tmp/bc_$v.npz | tail -1; }
done
for rep in 1 2; do
  WORKLOADS="c3 c4" bash scripts/ab.sh "--precision fp64 --no-fp64 --steps 8 --warmup 2" $L/libsparc_amp.so $L/libsparc_amp_xb1.so $L/libsparc_amp_xb2.so
done
