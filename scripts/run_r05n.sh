#!/bin/bash
# Round 5: k_secb Ab rows in a bank-aware step order per row (fb) — parity
# suite on the variant, then interleaved A/B; and the W8 stagger experiment.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sparc_ldpc_amd
SPARC_AMP_LIB=$L/libsparc_amp_fb.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_fb.log 2>&1 || { echo "parity fb failed"; tail -30 gpurun_out/par_fb.log; exit 1; }
tail -2 gpurun_out/par_fb.log
for r in 1 2; do
  WORKLOADS="c3 c4" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64" $L/libsparc_amp.so $L/libsparc_amp_fb.so || exit 1
  WORKLOADS="c3" bash scripts/ab.sh "--steps 8 --warmup 2 --no-fp64 --precision fp64" $L/libsparc_amp.so $L/libsparc_amp_fb.so || exit 1
done
WORKLOADS="c3" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --plan WB8" $L/libsparc_amp.so $L/libsparc_amp_st1.so $L/libsparc_amp_st2.so || exit 1
