#!/bin/bash
# Multi-step DEMetropolisZ step time for the published RTD models at the c4 shape (natural space).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-dzmodels}
mkdir -p $OUT
for m in "" bmm epm epm_piston; do
  DZ_MODEL=$m timeout -k 10 180 python tools/dz_probe.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
done
cat $OUT/probe.jsonl
