#!/bin/bash
# Round 5: which outputs of the binary64 k_secb variants differ from the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sparc_ldpc_amd
for v in libsparc_amp libsparc_amp_xg11 libsparc_amp_xgs libsparc_amp_x21; do
  BITCMP_CASES=8,9 SPARC_AMP_LIB=$L/$v.so timeout -k 10 300 python scripts/bitcmp.py run /tmp/bc_$v.npz > gpurun_out/bc2_$v.log 2>&1 || { echo "bitcmp $v failed"; tail -5 gpurun_out/bc2_$v.log; exit 1; }
  [ $v != libsparc_amp ] && { echo "== $v"; python scripts/bitcmp.py cmp /tmp/bc_libsparc_amp.npz /tmp/bc_$v.npz; }
done
exit 0
