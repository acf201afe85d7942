#!/bin/bash
# PMC evidence of the final tree, part 1: c2, c5, c3 per-kernel fp64 / traffic
# summaries (tools/gpu_pmc_r05.sh) and the c2 BA roofline (tools/gpu_ba_roofline.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MVBA_CG_GRAPH=0 PMC_CFGS="c2 c5 c3" bash tools/gpu_pmc_r05.sh r05p1 || exit 1
MVBA_CG_GRAPH=0 bash tools/gpu_ba_roofline.sh c2 r05p1 || exit 1
