cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python bench.py --workload c4 --batch 1 --steps 10 --warmup 2 --no-cpu --no-dense > gpurun_out/c4_b1.json 2> gpurun_out/c4_b1.err && \
timeout -k 10 300 python bench.py --workload c4 --batch 1 --backend dense --steps 3 --warmup 1 --no-cpu --no-dense > gpurun_out/c4_b1_dense.json 2> gpurun_out/c4_b1_dense.err
rc=$?; cat gpurun_out/c4_b1.json gpurun_out/c4_b1_dense.json; tail -n 3 gpurun_out/c4_b1*.err; exit $rc
