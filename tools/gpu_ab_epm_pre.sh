for i in 1 2; do
  for v in default lw8 lw2 tp10 tp20; do
    if [ $v = default ]; then L=""; else L="NGRTD_LIB=$PWD/noblegas_rtd_mcmc_amd/libngrtd_$v.so"; fi
    echo -n "$v "; env $L timeout -k 10 120 python tools/model_probe.py --models exp_pist_flow:123,exp_pist_flow:0,exp_pist_flow-piston:123,exp_pist_flow-piston:0 --steps 200 --rounds 1 2>/dev/null | grep '^{' || exit 1
  done
done
