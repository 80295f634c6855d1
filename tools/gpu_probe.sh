#!/bin/bash
# Diagnostics session: FETCH_SIZE calibration (tools/fetch_calib.hip) and the section-timing
# probe of logp_fused_kernel.  Usage: bash tools/gpu_probe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-probe}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/calib -o calib -- ./tools/fetch_calib > $OUT/calib.log 2>&1 || { echo "calib failed rc=$?"; exit 1; }
timeout -k 10 300 python tools/section_probe.py > $OUT/section.json 2> $OUT/section.err || { echo "probe failed rc=$?"; exit 1; }
cat $OUT/section.json
