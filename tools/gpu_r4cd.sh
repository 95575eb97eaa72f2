#!/bin/bash
# r04c (single-call request path) then r04d (large values, full -m gpu suite)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4c.sh && bash tools/gpu_r4d.sh
