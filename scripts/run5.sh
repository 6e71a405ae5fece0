#!/bin/bash
# A/B of the current build against libsparc_amp_prev.so at C4 single codeword
# (binary32 and binary64) and c2 binary64, then bit-identity
P=sparc_ldpc_amd/libsparc_amp_prev.so; N=sparc_ldpc_amd/libsparc_amp.so
WORKLOADS=c4 bash scripts/ab.sh "--batch 1 --steps 30 --warmup 3 --no-fp64" $P $N $P $N || exit 1
WORKLOADS=c4 bash scripts/ab.sh "--batch 1 --precision fp64 --steps 20 --warmup 3 --no-fp64" $P $N || exit 1
bash scripts/ab.sh "--precision fp64 --steps 30 --warmup 3 --no-fp64" $P $N || exit 1
SPARC_AMP_LIB=$P timeout -k 10 200 python scripts/bitcmp.py run gpurun_out/bc_prev.npz > /dev/null 2>&1 || exit 1
timeout -k 10 200 python scripts/bitcmp.py run gpurun_out/bc_new.npz > /dev/null 2>&1 || exit 1
python scripts/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz | tail -1
