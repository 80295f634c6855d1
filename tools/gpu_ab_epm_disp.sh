#!/bin/bash
# A/B of two compile-time knobs against the product library (tools/build_variant.py builds
# libngrtd_tp16.so with -DNGRTD_EPM_TAIL_PRE=16 and libngrtd_du8.so with -DNGRTD_GEN_DISP_UNROLL=8):
# exp_pist_flow per-launch times and dispersion per-launch times, two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/r04zb
for i in 1 2; do
  timeout -k 10 200 python tools/model_probe.py --models exp_pist_flow:0,exp_pist_flow-piston:0 --steps 200 --rounds 2 > gpurun_out/r04zb/epm_def$i.json || exit 1
  timeout -k 10 200 env NGRTD_LIB=noblegas_rtd_mcmc_amd/libngrtd_tp16.so python tools/model_probe.py --models exp_pist_flow:0,exp_pist_flow-piston:0 --steps 200 --rounds 2 > gpurun_out/r04zb/epm_tp16_$i.json || exit 1
  timeout -k 10 200 python tools/model_probe.py --models dispersion:0,dispersion:123 --steps 20 --rounds 2 > gpurun_out/r04zb/disp_def$i.json || exit 1
  timeout -k 10 200 env NGRTD_LIB=noblegas_rtd_mcmc_amd/libngrtd_du8.so python tools/model_probe.py --models dispersion:0,dispersion:123 --steps 20 --rounds 2 > gpurun_out/r04zb/disp_du8_$i.json || exit 1
done
for f in gpurun_out/r04zb/*.json; do echo "$f $(cat $f)"; done
