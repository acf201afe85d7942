#!/bin/bash
# PMC evidence of the final tree, part 2: c4 summaries and the c3 BA roofline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MVBA_CG_GRAPH=0 PMC_CFGS="c4" bash tools/gpu_pmc_r05.sh r05p2 || exit 1
MVBA_CG_GRAPH=0 bash tools/gpu_ba_roofline.sh c3 r05p2 || exit 1
