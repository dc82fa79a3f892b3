#!/bin/bash
# round 4: G = 128 and B = 8 bench lines, then the W4A16 lane-stagger sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_final_c.sh || exit 1
bash tools/gpu_r4_u.sh || exit 1
