#!/bin/bash
# r04b (v4 decoder tests + A/B + traces) then r04c (single-call request path)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4b.sh && bash tools/gpu_r4c.sh
