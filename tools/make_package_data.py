#!/usr/bin/env python3
"""Extract the small data tables the engine ships with from the reference's own
TEXT/XML data files (run once, in the build container, where /root/reference exists).

Outputs (committed, tiny):
  noblegas_rtd_mcmc_amd/data/plm_field_data.json
      Noble-gas observations of Field_Data/PLM_noblegas_2021.xlsx sheet1 rows 3-7
      (read at ng_interp/noble_gas_mcmc.py:72-78), parsed with zipfile+xml (no
      openpyxl, nothing executed from the file), the percent errors
      (noble_gas_mcmc.py:107) and the well elevations (noble_gas_mcmc.py:80-82).
  noblegas_rtd_mcmc_amd/data/atmos_series.npz
      Yearly atmospheric input series in the shape of age_ens_runs_mcmc/C_in_dict.pk
      (age index 25255..0, built by age_modeling_mcmc.prep.py:165-219).  The pickle
      itself is NOT loaded (pickle-only format, no safe loader); instead the series are
      rebuilt from the reference's shipped CSV histories:
        CFC12/SF6/CFC11/CFC113: Input_Series/NOAA_cfc_sf6/cfc_sf6_atmhist_1765-2021.csv
        H3: Input_Series/Tritium/TritiumInQuadrangeles_Jurgens2018.csv column
            '39-37,110-105' (the Crested Butte cell used at Gen_atmos_tracers_v3.py:57-60),
            annual means, 2013-2021 continued by 12.34-yr decay of the 2012 value,
            pre-1953 fill 3.3273 TU (the constant prefix SURVEY.md §8a-a15 recorded).
        He4_ter: zeros (run_age_mcmc.py:212 multiplies the series by 0.0).
      Ages older than the CSV coverage take the constant fill recorded in SURVEY.md
      §8a-a15 (1e-10 for the CFC/SF6 family).  Stored compactly as (fill, tail).
"""
import json
import os
import sys
import xml.etree.ElementTree as ET
import zipfile

import numpy as np

REF = os.environ.get("NGRTD_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "noblegas_rtd_mcmc_amd", "data")
N_FULL = 25256          # len(C_in_dict[...])
SAMPLE_YEAR = 2021      # age 0 == 2021 (CSV coverage ends there)


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
        # MAP tracer observations map_dict[tracer].loc[well] as recorded in SURVEY.md §8d c3
        # (map_dict.pk is a pickle and is not loaded here).
        "map_obs_PLM1": {"CFC12": 36.3828, "SF6": 1.24528, "H3": 4.86877, "He4_ter": 8.82174e-9},
    }


def series():
    import csv
    years, cols = [], {"CFC11": [], "CFC12": [], "CFC113": [], "SF6": []}
    with open(os.path.join(REF, "Input_Series", "NOAA_cfc_sf6", "cfc_sf6_atmhist_1765-2021.csv")) as f:
        for rec in csv.DictReader(f):
            years.append(int(rec["year"]))
            for k, c in (("CFC11", "cfc11_ppt"), ("CFC12", "cfc12_ppt"), ("CFC113", "cfc113_ppt"), ("SF6", "sf6_ppt")):
                cols[k].append(float(rec[c]))
    years = np.array(years)
    out = {}
    for k, v in cols.items():
        v = np.array(v)
        ages = SAMPLE_YEAR - years          # 256..0
        tail = np.zeros(ages.max() + 1)
        tail[ages] = v
        tail[tail == 0.0] = 1e-10           # constant-fill convention of C_in_dict
        out[k] = (1e-10, tail)
    # tritium: annual means of the Crested Butte quadrangle cell
    h3 = {}
    with open(os.path.join(REF, "Input_Series", "Tritium", "TritiumInQuadrangeles_Jurgens2018.csv")) as f:
        for rec in csv.DictReader(f):
            y, v = rec["Year"], rec["39-37,110-105"]
            if y and v:
                h3.setdefault(int(float(y)), []).append(float(v))
    yrs = sorted(h3)
    ann = {y: float(np.mean(h3[y])) for y in yrs}
    lam = -np.log(0.5) / 12.34
    for y in range(yrs[-1] + 1, SAMPLE_YEAR + 1):
        ann[y] = ann[yrs[-1]] * np.exp(-lam * (y - yrs[-1]))
    first = min(ann)
    tail = np.array([ann[SAMPLE_YEAR - a] for a in range(SAMPLE_YEAR - first + 1)])
    out["H3"] = (3.3273, tail)
    out["He4_ter"] = (0.0, np.zeros(1))
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "plm_field_data.json"), "w") as f:
        json.dump(field_data(), f, indent=1, sort_keys=True)
    s = series()
    arrays = {"N_full": np.array(N_FULL), "sample_year": np.array(SAMPLE_YEAR),
              "tracers": np.array(sorted(s))}
    for k, (fill, tail) in s.items():
        arrays[k + "_fill"] = np.array(fill)
        arrays[k + "_tail"] = np.asarray(tail, dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "atmos_series.npz"), **arrays)
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
