#!/bin/bash
# DZ probe: step time vs history length (fused and pair), rocprof stats of the fused sampler bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02h}
mkdir -p $OUT
timeout -k 10 300 python tools/dz_probe.py > $OUT/probe.json 2> $OUT/probe.err || exit 1
cat $OUT/probe.json
NGRTD_DZ_MODE=pair timeout -k 10 300 python tools/dz_probe.py > $OUT/probe_pair.json 2> $OUT/probe_pair.err || exit 1
cat $OUT/probe_pair.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o dz -- python3 $GRAFT_REPO_ROOT/tools/dz_probe.py > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/$OUT/prof -name "*kernel_stats.csv" | head -1 | xargs cut -c1-150 | head -8
