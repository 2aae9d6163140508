#!/bin/bash
# Wire-path kernel trace, then the headline A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/w2_kt.sh && bash scripts/gpu_ab.sh
