L=sparc_ldpc_amd/libsparc_amp.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "lds_bucket or triple or partial_layouts" > gpurun_out/t_ib.log 2>&1; rc=$?; tail -3 gpurun_out/t_ib.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab.sh "--steps 20 --warmup 3 --no-fp64" $L SPARC_AMP_IB=1@$L $L SPARC_AMP_IB=1@$L || exit 1
WORKLOADS=c4 bash scripts/ab.sh "--batch 1 --steps 20 --warmup 3 --no-fp64" $L SPARC_AMP_IB=1@$L $L SPARC_AMP_IB=1@$L || exit 1
bash scripts/ab.sh "--precision fp64 --steps 20 --warmup 3 --no-fp64" $L SPARC_AMP_IB=1@$L $L SPARC_AMP_IB=1@$L
