#!/bin/bash
# Every bench line of the round (GPU box): the default headline (c2, with the
# CPU baseline and the dense GEMV probe), c3, c4 (256 reps), c4 single
# codeword, binary64 c3 / c4, the dense backend at c3 (int8 MFMA GEMMs) and
# c4 single (fp32 GEMVs), a caller's Gaussian design (matrix backend) at c2 /
# c3, the joint configs[4] step (scripts/bench_joint.py), and a 2-rank rehearsal of the N-rank path on one GPU over the
# socket all-reduce.  Lines land in gpurun_out/bench_<tag>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
b() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > "gpurun_out/bench_$tag.log" 2>&1 || { echo "bench $tag failed"; tail -5 "gpurun_out/bench_$tag.log"; exit 1; }
  tail -1 "gpurun_out/bench_$tag.log" > "gpurun_out/bench_$tag.json"
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$tag.json')); r=d['roofline']; print('$tag', d['value'], d['unit'], d['ms_per_step'], 'ms/step', r['kernel'], r['frac'])"
}
GROUP=${1:-all}  # a: the factorised-operator lines; b: dense / matrix / joint / rehearsal / sweep
if [ "$GROUP" != b ]; then
b c2
b c3 --workload c3 --no-cpu --no-dense
b c4 --workload c4 --no-cpu --no-dense
b c4b1 --workload c4 --batch 1 --no-cpu --no-dense
b c3f64 --workload c3 --precision fp64 --no-fp64 --no-cpu --no-dense
b c4f64 --workload c4 --precision fp64 --no-fp64 --no-cpu --no-dense --steps 10 --warmup 2
fi
[ "$GROUP" = a ] && exit 0
b c3dense --workload c3 --backend dense --no-cpu --no-dense --steps 5 --warmup 1
b c4b1dense --workload c4 --batch 1 --backend dense --no-cpu --no-dense --steps 3 --warmup 1
b c2matrix --backend matrix --no-cpu --no-dense --no-fp64 --steps 5 --warmup 1
b c3matrix --workload c3 --backend matrix --no-cpu --no-dense --no-fp64 --steps 2 --warmup 1
timeout -k 10 600 python scripts/bench_joint.py > gpurun_out/bench_joint.log 2>&1 || { echo "joint failed"; tail -5 gpurun_out/bench_joint.log; exit 1; }
grep '^{' gpurun_out/bench_joint.log | tail -1 > gpurun_out/bench_joint.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_joint.json')); print('joint', d['value'], d['ms_per_step'], d['step_share_ms'], d['cpu_baseline']['value'])"
SPARC_DIST_BACKEND=socket timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-fp64 \
  > gpurun_out/bench_c2_rehearse_socket2.log 2>&1 || { echo "rehearsal failed"; tail -20 gpurun_out/bench_c2_rehearse_socket2.log; exit 1; }
grep '^{' gpurun_out/bench_c2_rehearse_socket2.log | tail -1 > gpurun_out/bench_c2_rehearse_socket2.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2_rehearse_socket2.json')); print('rehearsal', d['n_gpus'], d['value'], d['config']['parallelism'])"
# BASELINE configs[3]: the 10 k-rep L = 768 Monte-Carlo sweep (10 sigma points x 1000 reps, early stop)
timeout -k 10 300 python scripts/waterfall.py --sweep l768 --reps 1000 --out gpurun_out/waterfall_l768_10k > gpurun_out/waterfall_l768_10k.log 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/waterfall_l768_10k.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/waterfall_l768_10k.json')); print('sweep l768 10k reps', round(d['seconds'], 3), 's')"
