#!/bin/bash
# Final sources: every bench line of the round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/bench_all.sh a && bash scripts/bench_all.sh b
