#!/bin/bash
# A/B of library builds on per-launch kernel time (tools/model_probe.py): 3 rounds, each round
# over the product library and every variant .so named after the model list.
#   bash tools/gpu_ab_models.sh TAG MODELS [variant.so ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}; MODELS=${2:?models}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 120 python tools/model_probe.py --models $MODELS --rounds 1 > $OUT/default.$i.json || exit 1
  echo "round $i default $(cat $OUT/default.$i.json)" | tee -a $OUT/ab.txt
  for v in "$@"; do
    n=$(basename $v .so)
    timeout -k 10 120 env NGRTD_LIB=$PWD/$v python tools/model_probe.py --models $MODELS --rounds 1 > $OUT/$n.$i.json || exit 1
    echo "round $i $n $(cat $OUT/$n.$i.json)" | tee -a $OUT/ab.txt
  done
done
