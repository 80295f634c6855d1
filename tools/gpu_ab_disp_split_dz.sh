#!/bin/bash
# The dispersion age split (NGRTD_DISP_SPLIT_FRAC) for the DEMetropolisZ step and the log-prob:
# the generic DZ step (tools/dz_generic_ab.py, single launch only) and tools/model_probe.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in ${FRACS:-0.5 0.55 0.6 0.65}; do
  echo -n "frac $f "; NGRTD_DISP_SPLIT_FRAC=$f DZ_AB_PAIRS=dispersion DZ_AB_SINGLE=1 timeout -k 10 200 python tools/dz_generic_ab.py --rounds 1 2>/dev/null | grep '^{' | tr -d '\n' || exit 1
  NGRTD_DISP_SPLIT_FRAC=$f timeout -k 10 120 python tools/model_probe.py --models dispersion:0,dispersion-piston:0 --steps 100 --rounds 1 2>/dev/null | grep '^{' || exit 1
done
