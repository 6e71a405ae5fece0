#!/bin/bash
# Final sources: the second profile set and the SQ counter passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/profile_r04.sh c4f64 joint dense_l768 c3dense c2matrix c3matrix sq_c2 sq_c3 sq_c4 sq_c3f64 sq_bp
