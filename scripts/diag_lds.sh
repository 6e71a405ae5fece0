#!/bin/bash
# Diagnostic: LDS bank-conflict cycles and kernel time of k_secb builds whose
# gather or Ab-row LDS reads are replaced by conflict-free addresses (wrong
# results; counters only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=sparc_ldpc_amd
for v in libsparc_amp ${DIAG_VARS:-libsparc_amp_dGATHER libsparc_amp_dROWS}; do
  rm -rf gpurun_out/dl_$v
  SPARC_AMP_LIB=$L/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/dl_$v -o p --output-format csv -- python3 bench.py --workload ${WL:-c3} --steps 2 --warmup 0 --no-fp64 --no-cpu --no-dense > gpurun_out/dl_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/dl_$v.log; exit 1; }
  python3 - gpurun_out/dl_$v $v <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list); dur = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_secb" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_secb" in r["Kernel_Name"]:
            dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
import statistics
print(sys.argv[2], {k: round(statistics.mean(v) / 1e6, 2) for k, v in acc.items()}, "median us", statistics.median(dur) / 1e3 if dur else None)
PY
done
