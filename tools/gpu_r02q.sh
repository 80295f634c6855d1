#!/bin/bash
# EPM profile refresh after the 16-age blocks: PMC + bench + stats for exp_pist_flow and exp_pist_flow-piston
set -o pipefail
cd "$GRAFT_REPO_ROOT"
SKIP_TESTS=1 BENCH_ARGS="--mod-type1 exp_pist_flow" bash tools/gpu_profile.sh r02q_epm || exit 1
SKIP_TESTS=1 BENCH_ARGS="--mod-type1 exp_pist_flow --mod-type2 piston" bash tools/gpu_profile.sh r02q_epmp || exit 1
echo done
