#!/bin/bash
# DZ step timing variants (tools/dz_probe.py): full step, no partner loads (diag 1), no history
# store (2), no commit (4), no staging (8); natural and transformed space.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-dzdiag}
mkdir -p $OUT
for j in "" 1; do for d in 0 1 8 16; do
  DZ_JAC=$j NGRTD_DZ_DIAG=$d timeout -k 10 120 python tools/dz_probe.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
done; done
cat $OUT/probe.jsonl


