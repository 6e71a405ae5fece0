#!/bin/bash
# A/B of library variants / env settings:
#   bash scripts/ab.sh "<bench args>" VARIANT ...   VARIANT = lib.so or ENV=VAL,ENV2=VAL2@lib.so
# (one bench run per variant and workload; stops on an abnormal exit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=$1; shift
i=0
for var in "$@"; do
  lib=${var##*@}; envs=""
  [ "$lib" != "$var" ] && envs=${var%@*}
  for wl in ${WORKLOADS:-c2}; do
    i=$((i+1)); log=gpurun_out/ab_${i}_$wl.log
    env ${envs//,/ } SPARC_AMP_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-dense --workload $wl $ARGS > $log 2>&1
    rc=$?
    python - "$var" "$wl" $log <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"{sys.argv[1]:50s} {sys.argv[2]} {d['value']:10.1f} cw/s  {d['ms_per_step']:.4f} ms/step  {r['kernel']} {r.get('kernel_ms_dispatch')}")
except Exception as e:
    print(sys.argv[1], sys.argv[2], "FAILED", e)
PY
    if [ $rc -ne 0 ]; then echo "rc=$rc: stopping"; tail -5 $log; exit $rc; fi
  done
done
