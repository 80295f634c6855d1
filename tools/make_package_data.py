#!/usr/bin/env python3
"""Extract the small data tables the engine ships with from the reference's own data
files (run once, in the build container, where /root/reference exists).

Outputs (committed, tiny):
  noblegas_rtd_mcmc_amd/data/plm_field_data.json
      Noble-gas observations of Field_Data/PLM_noblegas_2021.xlsx sheet1 rows 3-7
      (read at ng_interp/noble_gas_mcmc.py:72-78), parsed with zipfile+xml (no
      openpyxl, nothing executed from the file), the percent errors
      (noble_gas_mcmc.py:107), the well elevations (noble_gas_mcmc.py:80-82) and the
      MAP tracer observations of age_ens_runs_mcmc/map_dict.pk (prep.py:453-494),
      every tracer x well, at full float64 precision.
  noblegas_rtd_mcmc_amd/data/atmos_series.npz
      The shipped input series age_ens_runs_mcmc/C_in_dict.pk (written by
      age_modeling_mcmc.prep.py:165-219; read at run_age_mcmc.py:46), all 6 tracers.
      Both pickles are read WITHOUT unpickling: tools/pickle_extract.py walks their
      opcode stream symbolically (nothing is imported or called) and decodes the float64
      block buffers and int64 indices with numpy.frombuffer.
      Stored age-first (age k = np.flip(C_in_dict[t].values)[k], the flip that
      convolution_integral_utils.py:336 applies) and compactly, bit for bit: every series
      is a constant fill for all ages >= its tail length, so the file holds the fill value
      and the ages before it.  tests/test_package_data_cpu.py re-extracts the pickle and
      checks the reconstruction bitwise.
"""
import json
import os
import sys
import xml.etree.ElementTree as ET
import zipfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pickle_extract import read_frame_dict  # noqa: E402

REF = os.environ.get("NGRTD_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "noblegas_rtd_mcmc_amd", "data")
N_FULL = 25256          # len(C_in_dict[...])
SAMPLE_YEAR = 2021      # age 0 == 2021 (prep.py:163)


def read_xlsx_sheet1(path):
    ns = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main"}
    z = zipfile.ZipFile(path)
    sst = ET.fromstring(z.read("xl/sharedStrings.xml"))
    strs = ["".join(t.text or "" for t in si.iter("{%s}t" % ns["m"])) for si in sst.findall("m:si", ns)]
    sh = ET.fromstring(z.read("xl/worksheets/sheet1.xml"))
    rows = {}
    for row in sh.find("m:sheetData", ns).findall("m:row", ns):
        r = int(row.get("r"))
        vals = {}
        for c in row.findall("m:c", ns):
            v = c.find("m:v", ns)
            if v is None:
                continue
            col = "".join(ch for ch in c.get("r") if ch.isalpha())
            vals[col] = strs[int(v.text)] if c.get("t") == "s" else v.text
        rows[r] = vals
    return rows


def field_data():
    rows = read_xlsx_sheet1(os.path.join(REF, "Field_Data", "PLM_noblegas_2021.xlsx"))
    header = rows[2]
    col_of = {name: col for col, name in header.items()}
    wells = {}
    for r in range(3, 8):  # nrows=5 after skiprows=1 (noble_gas_mcmc.py:72)
        site = rows[r]["A"]
        rec = {}
        for key, name in (("He", "4He"), ("Ne", "Ne"), ("Ar", "Ar"), ("Kr", "Kr"), ("Xe", "Xe"),
                          ("He3", "3He"), ("R/Ra", "R/Ra")):
            rec[key] = float(rows[r][col_of[name]])
        wells[site] = rec
    return {
        "source": "Field_Data/PLM_noblegas_2021.xlsx sheet1 rows 3-7 (noble_gas_mcmc.py:72-78)",
        "units": "ccSTP/g(H2O)",
        "obs": wells,
        "err_percent": {"He": 1.5, "Ne": 1.5, "Ar": 2.5, "Kr": 3.1, "Xe": 15.1},   # noble_gas_mcmc.py:107
        "well_elev": {"PLM1": 2786.889893, "PLM6": 2759.569824, "PLM7": 2782.550049},  # :80-82
        # MAP tracer observations map_dict[tracer].loc[well] (run_age_mcmc.py:44,128)
        "map_obs": map_obs(),
        "map_source": "age_ens_runs_mcmc/map_dict.pk (no-code read, tools/pickle_extract.py)",
    }


def map_obs():
    """{tracer column: {well: value}} of every DataFrame in map_dict.pk."""
    out = {}
    for _key, fr in read_frame_dict(os.path.join(REF, "age_ens_runs_mcmc", "map_dict.pk")).items():
        for j, col in enumerate(fr["columns"]):
            out[col] = {str(w): float(fr["values"][j][i]) for i, w in enumerate(fr["index"])}
    return out


def series():
    """{tracer: (fill, tail)} of C_in_dict.pk, age-first, bit-exact."""
    out = {}
    for key, fr in read_frame_dict(os.path.join(REF, "age_ens_runs_mcmc", "C_in_dict.pk")).items():
        if fr["values"].shape[0] != 1:
            raise ValueError("%s: expected one column, got %r" % (key, fr["columns"]))
        v = np.flip(fr["values"][0]).copy()            # age 0 first (:336)
        idx = np.flip(fr["index"])
        if len(v) != N_FULL or not np.array_equal(idx, np.arange(N_FULL)):
            raise ValueError("%s: index is not 25255..0" % key)
        fill = v[-1]
        diff = np.nonzero(v != fill)[0]
        k0 = int(diff.max()) + 1 if len(diff) else 0
        out[key] = (fill, v[:k0], fr["columns"][0])
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "plm_field_data.json"), "w") as f:
        json.dump(field_data(), f, indent=1, sort_keys=True)
    s = series()
    arrays = {"N_full": np.array(N_FULL), "sample_year": np.array(SAMPLE_YEAR),
              "tracers": np.array(sorted(s))}
    for k, (fill, tail, col) in s.items():
        arrays[k + "_fill"] = np.array(fill)
        arrays[k + "_tail"] = np.asarray(tail, dtype=np.float64)
        arrays[k + "_column"] = np.array(col)
    np.savez_compressed(os.path.join(OUT, "atmos_series.npz"), **arrays)
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
