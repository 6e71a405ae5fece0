#!/bin/bash
# Round 5 profile set, part 1 (scripts/profile_r05.sh): the factorised-operator workloads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 1100 bash scripts/profile_r05.sh c2 c2f64 c4b1 c3 c3f64 c4 c4f64
