#!/bin/bash
# SQ/LDS counter passes for one bench workload (each pass its own rocprofv3 run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-sq}; shift
# SCRIPT=scripts/bp_time.py runs another program with its own arguments
if [ -n "$SCRIPT" ]; then PROG=("$SCRIPT" "$@"); else PROG=(bench.py --no-cpu --no-dense "$@"); fi
OUT=gpurun_out/sq_$TAG; mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" \
           "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- \
     python3 "${PROG[@]}" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(sys.argv[1])), "..", "scripts"))
sys.path.insert(0, "scripts")
from pmc_summary import short
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    if not k.startswith(("k_sec", "k_row", "k_gemm", "k_dense", "k_i8", "k_bp")):
        continue
    print(k, "(per launch, mean over launches; SQ_* cycle counters in quad-cycles)")
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}")
PY
