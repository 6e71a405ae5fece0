#!/bin/bash
# Round 5: binary32 k_secb codeword pairs on packed fp32 (v_pk_fma_f32) in the
# bucket gather and the Ab rows: bit identity + interleaved A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sparc_ldpc_amd
VARS=${VARS:-"libsparc_amp_base libsparc_amp_pk"}
base=${VARS%% *}
for v in $VARS; do
  BITCMP_CASES=${CASES:-0,1,3,4,5,6,7,13} SPARC_AMP_LIB=$L/$v.so timeout -k 10 300 python scripts/bitcmp.py run /tmp/bc_$v.npz > gpurun_out/bc_$v.log 2>&1 || { echo "bitcmp $v failed"; tail -5 gpurun_out/bc_$v.log; exit 1; }
  [ $v != $base ] && { echo "== $v"; python scripts/bitcmp.py cmp /tmp/bc_$base.npz /tmp/bc_$v.npz | tail -1; }
done
libs=""; for v in $VARS; do libs="$libs $L/$v.so"; done
for rep in 1 2; do
  WORKLOADS=${WL:-"c3 c4"} bash scripts/ab.sh "${ARGS:---steps 10 --warmup 2 --no-fp64}" $libs || exit 1
done
