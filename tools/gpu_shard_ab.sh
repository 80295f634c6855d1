#!/bin/bash
# c5 shard geometry A/B: per-launch kernel time of the c4 plan at 256 walkers (one strong-scaled
# shard of 8) with the adaptive walkers-per-block (fused_wb: 256 one-walker blocks) and with the
# full blocks (NGRTD_FUSED_WB=max: 32 blocks of 8 walkers), 3 interleaved rounds; then 2048.
#   bash tools/gpu_shard_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:?tag}
mkdir -p $OUT
M=exponential:0,exponential:123,exp_pist_flow:0
for i in 1 2 3; do
  timeout -k 10 120 python tools/model_probe.py --models $M --walkers 256 --steps 400 --rounds 1 > $OUT/wb_auto.$i.json || exit 1
  echo "round $i W=256 auto $(cat $OUT/wb_auto.$i.json)" | tee -a $OUT/shard_ab.txt
  timeout -k 10 120 env NGRTD_FUSED_WB=max python tools/model_probe.py --models $M --walkers 256 --steps 400 --rounds 1 > $OUT/wb_max.$i.json || exit 1
  echo "round $i W=256 max  $(cat $OUT/wb_max.$i.json)" | tee -a $OUT/shard_ab.txt
done
timeout -k 10 120 python tools/model_probe.py --models $M --walkers 2048 --steps 400 --rounds 2 > $OUT/w2048.json || exit 1
echo "W=2048 $(cat $OUT/w2048.json)" | tee -a $OUT/shard_ab.txt
