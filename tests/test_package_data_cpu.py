"""The shipped data tables: the input series ARE age_ens_runs_mcmc/C_in_dict.pk and the
MAP observations ARE map_dict.pk, bit for bit.  The pickles are read with the no-code
reader tools/pickle_extract.py (opcode walk, nothing unpickled).  CPU only; the checks
against the reference's files skip where /root/reference is absent (the GPU box)."""
import os
import pickle
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from pickle_extract import read_frame_dict, symbolic_load  # noqa: E402

from noblegas_rtd_mcmc_amd import workloads as wl  # noqa: E402

REF = os.environ.get("NGRTD_REFERENCE", "/root/reference")
need_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "age_ens_runs_mcmc")),
                              reason="reference data not present")


@need_ref
def test_series_equal_shipped_pickle_bitwise():
    frames = read_frame_dict(os.path.join(REF, "age_ens_runs_mcmc", "C_in_dict.pk"))
    assert sorted(frames) == sorted(["CFC11", "CFC12", "CFC113", "SF6", "He4_ter", "H3"])
    for key, fr in frames.items():
        assert np.array_equal(fr["index"], np.arange(25255, -1, -1))
        want = np.flip(fr["values"][0])
        got = wl.atmos_series(key).c_by_age
        assert got.view(np.int64).tolist() == want.view(np.int64).tolist(), key
        # c3/c4 use the last 1200 rows of the DataFrame
        assert np.array_equal(wl.atmos_series(key, 1200).c_by_age, want[:1200])


@need_ref
def test_map_obs_equal_shipped_pickle():
    frames = read_frame_dict(os.path.join(REF, "age_ens_runs_mcmc", "map_dict.pk"))
    for _key, fr in frames.items():
        for j, col in enumerate(fr["columns"]):
            for i, well in enumerate(fr["index"]):
                assert wl.map_obs(str(well))[col] == fr["values"][j][i]
    # SURVEY.md §8d c3 quotes these PLM1 values to 6 digits
    spec, _ = wl.c3(W=4)
    np.testing.assert_allclose(spec.rtd.obs[0], [36.3828, 1.24528, 4.86877, 8.82174e-9], rtol=1e-5)


def test_symbolic_reader_on_own_pickle(tmp_path):
    """The reader decodes a pickle this test writes itself (pandas frames of known data)."""
    pd = pytest.importorskip("pandas")
    rng = np.random.default_rng(5)
    d = {"A": pd.DataFrame({"x": rng.normal(size=37)}, index=np.arange(36, -1, -1)),
         "B": pd.DataFrame({"p": rng.normal(size=3), "q": rng.normal(size=3)}, index=["u", "v", "w"])}
    path = tmp_path / "own.pk"
    with open(path, "wb") as f:
        pickle.dump(d, f, protocol=4)
    got = read_frame_dict(str(path))
    assert np.array_equal(got["A"]["values"][0], d["A"]["x"].to_numpy())
    assert np.array_equal(got["A"]["index"], d["A"].index.to_numpy())
    assert got["B"]["columns"] == ["p", "q"] and list(got["B"]["index"]) == ["u", "v", "w"]
    assert np.array_equal(got["B"]["values"], d["B"].to_numpy().T)


def test_symbolic_reader_never_calls(tmp_path):
    """A pickle naming a callable yields an inert record; nothing is imported or run."""
    class Boom:
        def __reduce__(self):
            return (os.system, ("echo should-not-run",))
    path = tmp_path / "boom.pk"
    with open(path, "wb") as f:
        pickle.dump({"k": Boom()}, f, protocol=4)
    top = symbolic_load(path.read_bytes())
    (k, rec), = top.items
    assert k == "k" and rec.func.qual in ("posix.system", "os.system", "nt.system")
