#!/bin/bash
# A/B of the current build against libsparc_amp_prev.so at c2 and C4 single codeword, then bit-identity
P=sparc_ldpc_amd/libsparc_amp_prev.so; N=sparc_ldpc_amd/libsparc_amp.so
bash scripts/ab.sh "--steps 30 --warmup 3 --no-fp64" $P $N $P $N $P $N || exit 1
WORKLOADS=c4 bash scripts/ab.sh "--batch 1 --steps 30 --warmup 3 --no-fp64" $P $N $P $N || exit 1
SPARC_AMP_LIB=$P timeout -k 10 200 python scripts/bitcmp.py run gpurun_out/bc_prev.npz > /dev/null 2>&1 || exit 1
timeout -k 10 200 python scripts/bitcmp.py run gpurun_out/bc_new.npz > /dev/null 2>&1 || exit 1
python scripts/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz | tail -1
