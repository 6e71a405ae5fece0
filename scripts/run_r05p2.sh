#!/bin/bash
# Round 5 profile set, part 2: the joint step, the dense / matrix backends, SQ counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 1100 bash scripts/profile_r05.sh joint dense_l768 c3dense c2matrix c3matrix sq_c3 sq_c3f64 sq_c4
