#!/bin/bash
# binary64 batched kernel A/B: previous build vs KH=1 / KR=1 + vector non-temporal beta, then plan options
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export LDPC_BP_TAIL=0  # the BP tail launches are measured in run D
mkdir -p gpurun_out
P=sparc_ldpc_amd/libsparc_amp_prev.so; N=sparc_ldpc_amd/libsparc_amp.so
WORKLOADS="c3 c4" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --precision fp64" $P $N $P $N || exit 1
WORKLOADS="c3 c4" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --precision fp64 --plan ZIL" $N || exit 1
WORKLOADS="c3" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --precision fp64 --plan WB16" $N || exit 1
WORKLOADS="c3" bash scripts/ab.sh "--steps 10 --warmup 2 --no-fp64 --precision fp64 --plan WB16,ZIL" $N || exit 1
for v in "$P|" "$N|" "$N|ZIL" "$N|WB16,ZIL"; do
  lib=${v%|*}; plan=${v#*|}
  SPARC_AMP_LIB=$lib timeout -k 10 300 python scripts/bench_joint.py --no-cpu ${plan:+--plan $plan} > gpurun_out/joint_ab.log 2>&1 || { echo "joint failed"; tail -5 gpurun_out/joint_ab.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/joint_ab.log').read().strip().splitlines()[-1]); print('joint', sys.argv[1], d['value'], d['ms_per_step'], d['step_share_ms'])" "$v"
done
SPARC_AMP_LIB=$P timeout -k 10 300 python scripts/bitcmp.py run gpurun_out/bc_prev.npz > gpurun_out/bc_prev.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bitcmp.py run gpurun_out/bc_new.npz > gpurun_out/bc_new.log 2>&1 || exit 1
python scripts/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz | tail -3
rm -f gpurun_out/bc_prev.npz gpurun_out/bc_new.npz
