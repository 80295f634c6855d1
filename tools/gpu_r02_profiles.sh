#!/bin/bash
# Round-2 profile set: headline (with all GPU tests) + the published RTD models, PMC + stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_profile.sh r02p_exp || exit 1
SKIP_TESTS=1 BENCH_ARGS="--mod-type1 exp_pist_flow" bash tools/gpu_profile.sh r02p_epm || exit 1
SKIP_TESTS=1 BENCH_ARGS="--mod-type1 exponential --mod-type2 piston" bash tools/gpu_profile.sh r02p_bmm || exit 1
echo done
