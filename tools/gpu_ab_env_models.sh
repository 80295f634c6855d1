#!/bin/bash
# A/B of environment switches on per-launch kernel time (tools/model_probe.py): 3 rounds, each
# round the default and every "K=V[+K2=V2]" variant in turn (same library).
#   bash tools/gpu_ab_env_models.sh TAG MODELS "NGRTD_NO_REFB=1" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}; MODELS=${2:?models}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 120 python tools/model_probe.py --models $MODELS --rounds 1 > $OUT/envdefault.$i.json || exit 1
  echo "round $i default $(cat $OUT/envdefault.$i.json)" | tee -a $OUT/env_ab.txt
  for v in "$@"; do
    timeout -k 10 120 env ${v//+/ } python tools/model_probe.py --models $MODELS --rounds 1 > $OUT/env.$i.json || exit 1
    echo "round $i $v $(cat $OUT/env.$i.json)" | tee -a $OUT/env_ab.txt
  done
done
