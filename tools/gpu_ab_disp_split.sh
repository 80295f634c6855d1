#!/bin/bash
# A/B of the dispersion age split between the unit's theta and RTD waves
# (NGRTD_DISP_SPLIT_FRAC: the theta waves' share), 2 interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for f in ${FRACS:-0.5 0.45 0.4 0.55}; do
    echo -n "frac $f "; NGRTD_DISP_SPLIT_FRAC=$f timeout -k 10 120 python tools/model_probe.py --models dispersion:0,dispersion:123,dispersion-piston:0 --steps 100 --rounds 1 2>/dev/null | grep '^{' || exit 1
  done
done
