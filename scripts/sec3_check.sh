#!/bin/bash
# k_sec43 check: GPU parity tests, then C4 single-codeword A/B (pairs vs triples) and the c2 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sec3_pytest.log 2>&1
rc=$?; tail -n 15 gpurun_out/sec3_pytest.log
[ $rc -ne 0 ] && exit $rc
for v in 0 1 0 1; do
  SPARC_AMP_SEC3=$v timeout -k 10 120 python bench.py --workload c4 --batch 1 --steps 20 --warmup 3 --no-cpu --no-dense > gpurun_out/sec3_c4_$v.json 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['kernel'], r['kernel_ms'], r['frac'])" gpurun_out/sec3_c4_$v.json SEC3=$v
done
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --no-dense > gpurun_out/sec3_c2.json 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c2', d['value'], r['kernel'], r['kernel_ms'], r['frac'])" gpurun_out/sec3_c2.json
