#!/bin/bash
# Round 5: phase stamps of k_secb at c3, binary64 and binary32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in fp64 fp32; do
  STAMPS_PREC=$p SPARC_AMP_LIB=sparc_ldpc_amd/libsparc_amp_stamps.so timeout -k 10 300 python scripts/stamps.py c3 > gpurun_out/stamps_c3_$p.txt 2>&1 || { echo "stamps $p failed"; tail -5 gpurun_out/stamps_c3_$p.txt; exit 1; }
  echo "== $p"; cat gpurun_out/stamps_c3_$p.txt
done
