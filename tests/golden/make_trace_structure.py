#!/usr/bin/env python3
"""Freeze the structure (group / variable / dimension / attribute names and types, storage
filters; no values) of the reference's shipped trace
age_ens_runs_mcmc/conv_traces/PLM1.CFC12.SF6.H3.He4_ter.exponential.123.netcdf (written by
az.to_netcdf, run_age_mcmc_utils.py:425) into trace_structure_exponential_123.json, and the
sampling_time / tuning_steps attributes of every shipped trace into trace_attrs.json.
Run in the build container (it reads /root/reference).  tests/golden/traces/ also holds one
shipped trace as-is (PLM1.H3.exponential.0.netcdf, a data file) for the reader tests."""
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from noblegas_rtd_mcmc_amd import h5lite  # noqa: E402

REF = "/root/reference/age_ens_runs_mcmc/conv_traces"

if __name__ == "__main__":
    st = h5lite.structure(os.path.join(REF, "PLM1.CFC12.SF6.H3.He4_ter.exponential.123.netcdf"))
    with open(os.path.join(HERE, "trace_structure_exponential_123.json"), "w") as f:
        json.dump(st, f, indent=1, sort_keys=True)
    attrs = {}
    for p in sorted(glob.glob(os.path.join(REF, "*.netcdf"))):
        r = h5lite.H5Reader(p)
        a = r.attrs(r.links(r.root)["posterior"])
        attrs[os.path.basename(p)] = {"sampling_time": float(a["sampling_time"][0]),
                                      "tuning_steps": int(a["tuning_steps"][0])}
    with open(os.path.join(HERE, "trace_attrs.json"), "w") as f:
        json.dump(attrs, f, indent=1, sort_keys=True)
