#!/bin/bash
# BA rooflines of the final tree (16 pass-B replicas): c2 and c3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MVBA_CG_GRAPH=0 bash tools/gpu_ba_roofline.sh c2 r05bb || exit 1
MVBA_CG_GRAPH=0 bash tools/gpu_ba_roofline.sh c3 r05bb || exit 1
