#!/bin/bash
# PMC calibration (scripts/pmc_calib.hip): FETCH_SIZE and WRITE_SIZE per
# access pattern, one rocprofv3 pass each; summary in gpurun_out/pmc_calib.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/calib
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/calib/f -o f --output-format csv -- ./scripts/pmc_calib > gpurun_out/calib_f.log 2>&1 || { echo "calib fetch failed"; tail -5 gpurun_out/calib_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/calib/w -o w --output-format csv -- ./scripts/pmc_calib > gpurun_out/calib_w.log 2>&1 || { echo "calib write failed"; tail -5 gpurun_out/calib_w.log; exit 1; }
python3 scripts/pmc_calib.py gpurun_out/calib gpurun_out/pmc_calib.json
