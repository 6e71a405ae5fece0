cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bitcmp.py run gpurun_out/bitcmp_r03head.npz > gpurun_out/bitcmp_r03head.log 2>&1 || { echo bitcmp failed; tail -20 gpurun_out/bitcmp_r03head.log; exit 1; }
for wl in c2 c3 c4; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu --no-dense --steps 20 --warmup 3 > gpurun_out/base_$wl.log 2>&1 || { echo bench $wl failed; tail -5 gpurun_out/base_$wl.log; exit 1; }
  tail -1 gpurun_out/base_$wl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', d['value'], d['ms_per_step'], d.get('fp64_leg',{}).get('value'), d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
