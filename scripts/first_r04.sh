cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_matrix.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_matrix.log 2>&1; rc=$?; tail -25 gpurun_out/t_matrix.log
[ $rc -gt 1 ] && exit $rc
NO_AB=1 bash scripts/check_r04.sh
