"""The trace container (f4): the reference's runs are ONE netCDF-4 / HDF5 file each
(az.to_netcdf, age_ens_runs_mcmc/run_age_mcmc_utils.py:425), read back by az.from_netcdf
(:434, run_age_mcmc.post_plots.comp.py:171).  h5lite reads the reference's shipped
conv_traces/*.netcdf (all 22 when /root/reference is present; the committed
tests/golden/traces/PLM1.H3.exponential.0.netcdf always) and writes ours; the structure of our
file is diffed against the frozen structure of
conv_traces/PLM1.CFC12.SF6.H3.He4_ter.exponential.123.netcdf
(tests/golden/make_trace_structure.py)."""
import glob
import json
import os
import re

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF = "/root/reference/age_ens_runs_mcmc/conv_traces"

# sampling_time ranges per model family (s, all chains, tune included)
RANGES = {"exponential.0": (67.0, 101.0), "exponential.123": (230.0, 241.0), "exp_pist_flow.123": (296.0, 324.0),
          "exponential-piston.123": (401.0, 401.5), "exp_pist_flow-piston.123": (438.0, 494.0)}


def _shipped():
    paths = sorted(glob.glob(os.path.join(REF, "*.netcdf")))
    return paths or [os.path.join(GOLD, "traces", "PLM1.H3.exponential.0.netcdf")]


def test_lookup3_known_values():
    """HDF5's metadata checksum (Jenkins lookup3 hashlittle, initval 0)."""
    from noblegas_rtd_mcmc_amd.h5lite import lookup3
    assert lookup3(b"") == 0xDEADBEEF
    assert lookup3(b"Four score and seven years ago") == 0x17770551        # lookup3.c driver5
    assert lookup3(b"Four score and seven years ago", 1) == 0xCD628161


@pytest.mark.parametrize("path", _shipped(), ids=os.path.basename)
def test_reader_decodes_shipped_trace(path):
    """Every shipped trace decodes (superblock v2, dense link / attribute storage, chunked
    shuffle + deflate datasets, global-heap DIMENSION_LIST): 3 chains x 10 000 draws per
    posterior variable, finite, tau1 positive (the single-tracer runs of savenum 0 predate the
    U(1, 1000) bounds of run_age_mcmc.py:145-146: their tau1 reaches 4400); accepted in {0, 1};
    tuning_steps = 10 000 and sampling_time in SURVEY.md §6's range for its model."""
    from noblegas_rtd_mcmc_amd import trace
    t = trace.from_netcdf(path)
    assert set(t) >= {"posterior", "sample_stats", "attrs", "coords"}
    assert t["attrs"]["tuning_steps"] == 10000 and t["attrs"]["inference_library"] == "pymc3"
    name = os.path.basename(path)
    key = next(k for k in RANGES if name.endswith(k + ".netcdf") and not (k == "exponential.123" and "piston" in name))
    lo, hi = RANGES[key]
    assert lo <= t["attrs"]["sampling_time"] <= hi, (name, t["attrs"]["sampling_time"])
    frozen = json.load(open(os.path.join(GOLD, "trace_attrs.json")))[name]
    assert t["attrs"]["sampling_time"] == frozen["sampling_time"]
    assert np.array_equal(t["coords"]["chain"], [0, 1, 2]) and np.array_equal(t["coords"]["draw"], np.arange(10000))
    for v, (dims, a) in t["posterior"].items():
        assert dims == ("chain", "draw") and a.shape == (3, 10000) and np.isfinite(a).all(), v
    tau = t["posterior"]["tau1"][1]
    assert (tau >= 1).all() and (tau <= 15000).all()
    acc = t["sample_stats"]["accepted"][1]
    assert set(np.unique(acc)) <= {0, 1} and 0 < acc.mean() < 1
    assert set(t["sample_stats"]) == {"accept", "accepted", "lambda", "scaling"}


def _norm(st):
    """Structure without string lengths (values differ) and without the root provenance."""
    s = json.loads(re.sub(r'"string\d+"', '"string"', json.dumps(st)))
    s.pop("/", None)
    return s


def _our_trace(tmp_path, with_lp=False):
    import torch
    from noblegas_rtd_mcmc_amd import trace
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.spec import ModelSpec
    base = wl.c4_spec(L=1, N=60, par_names=("tau1", "J", "thalf_cfc", "lamsf6"))
    tr = [t for t in base.rtd.tracers if t.name in ("CFC12", "SF6", "H3", "He4_ter")]
    import dataclasses
    rtd = dataclasses.replace(base.rtd, tracers=tr, obs=base.rtd.obs[:, [0, 1, 2, 4]], sd=base.rtd.sd[:, [0, 1, 2, 4]])
    spec = ModelSpec(n_wells=1, rtd=rtd)
    D, W = 40, 3
    rng = np.random.default_rng(3)
    s = np.stack([wl.sample_prior(spec, W, rng) for _ in range(D)])
    res = {"samples": torch.from_numpy(s), "logp": torch.from_numpy(rng.normal(size=(D, 1, W))),
           "accepted": torch.from_numpy(rng.integers(0, 2, (D, 1, W)).astype(np.uint8)),
           "accept": torch.from_numpy(rng.uniform(0, 2, (D, 1, W))),
           "lamb": torch.full((1, W), 0.5, dtype=torch.float64), "scaling": torch.full((1, W), 1e-3, dtype=torch.float64),
           "tuning_steps": 10000, "sampling_time": 12.5}
    idata = trace.inference_data(res, spec, wells=["PLM1"], observed=spec.rtd.obs)
    path = str(tmp_path / "PLM1.CFC12.SF6.H3.He4_ter.exponential.123.netcdf")
    trace.to_netcdf(idata, path)
    return idata, path


def test_our_trace_structure_matches_reference(tmp_path):
    """A trace of the same model (4 tracers, exponential, savenum 123: tau1, J, thalf_cfc,
    lamsf6) written by trace.to_netcdf has the reference file's structure: groups, group
    attributes, variables, dtypes, dimension names, per-variable attributes (netCDF's
    _Netcdf4Dimid / _Netcdf4Coordinates, _FillValue, the dimension-scale CLASS / NAME /
    REFERENCE_LIST, DIMENSION_LIST) and storage filters (shuffle, deflate)."""
    from noblegas_rtd_mcmc_amd import h5lite
    _, path = _our_trace(tmp_path)
    ours = _norm(h5lite.structure(path))
    ref = _norm(json.load(open(os.path.join(GOLD, "trace_structure_exponential_123.json"))))
    assert set(ours) == set(ref)
    for g in ref:
        assert ours[g]["attrs"] == ref[g]["attrs"], g
        assert set(ours[g]["vars"]) == set(ref[g]["vars"]), (g, set(ours[g]["vars"]) ^ set(ref[g]["vars"]))
        for v in ref[g]["vars"]:
            assert ours[g]["vars"][v] == ref[g]["vars"][v], (g, v, ours[g]["vars"][v], ref[g]["vars"][v])


def test_our_trace_roundtrip(tmp_path):
    """to_netcdf -> from_netcdf gives back every array bit for bit and the attributes."""
    from noblegas_rtd_mcmc_amd import trace
    idata, path = _our_trace(tmp_path)
    back = trace.from_netcdf(path)
    assert back["attrs"]["tuning_steps"] == 10000 and back["attrs"]["sampling_time"] == 12.5
    for g in ("posterior", "sample_stats"):
        assert set(back[g]) == set(idata[g])
        for k, (dims, arr) in idata[g].items():
            assert back[g][k][0] == dims and np.array_equal(back[g][k][1], arr), (g, k)
    assert np.array_equal(back["observed_data"]["like"][1], idata["observed"])


def test_inference_data_serves_reference_caller(tmp_path):
    """conv_mcmc.sample_mcmc returns trace.InferenceData (what the reference returns:
    az.from_pymc3(trace), run_age_mcmc_utils.py:407-429).  The reference's caller
    (age_ens_runs_mcmc/run_age_mcmc.py:231-276) runs az.summary over it, copies it, takes the
    summary's index as the variable list and reads every posterior draw as
    np.asarray(dd['posterior'][v])[0, :][s]; that loop, restated here, must see the
    sampler's chain-0 draws of every variable, and the object must round-trip through
    to_netcdf."""
    from noblegas_rtd_mcmc_amd import trace
    idd, _ = _our_trace(tmp_path)
    raw = {"samples": np.zeros(3), "accept_rate": 0.25}
    mc_out = trace.InferenceData.from_dict(idd, raw=raw)
    trace_summary = trace.summary(mc_out, round_to=6)                     # az.summary(mc_out, round_to=6)
    assert list(trace_summary.columns[:2]) == ["mean", "sd"]
    dd = mc_out.copy()
    pp = {'tau1': False, 'tau2': False, 'f1': False, 'f2': False, 'eta1': False, 'eta2': False, 'J': False,
          'D1': False, 'D2': False, 'thalf_cfc': False, 'lamsf6': False}
    vrs = list(trace_summary.index)
    assert {"tau1", "J", "thalf_cfc", "lamsf6", "nu"} <= set(vrs)
    seen = {v: [] for v in vrs}
    for s in range(np.asarray(dd['posterior']['tau1']).shape[1]):
        for v in vrs:
            pp[v] = np.asarray(dd['posterior'][v])[0, :][s]
            seen[v].append(pp[v])
    for v in vrs:
        assert np.array_equal(seen[v], idd["posterior"][v][1][0]), v
    assert np.array_equal(np.asarray(mc_out.posterior["tau1"]), idd["posterior"]["tau1"][1])
    assert mc_out.posterior.var_dims["tau1"] == ("chain", "draw")
    assert np.array_equal(mc_out["sample_stats"]["accepted"], idd["sample_stats"]["accepted"][1])
    assert mc_out["accept_rate"] == 0.25 and set(mc_out.groups()) == {"posterior", "sample_stats", "observed_data"}
    # the copy is independent of the original
    dd["posterior"]["tau1"][0, 0] = -1.0
    assert mc_out["posterior"]["tau1"][0, 0] != -1.0
    back = trace.from_netcdf(trace.to_netcdf(mc_out, str(tmp_path / "again.netcdf")))
    for k, (dims, arr) in idd["posterior"].items():
        assert back["posterior"][k][0] == dims and np.array_equal(back["posterior"][k][1], arr), k


def test_ce_prior_group_roundtrip(tmp_path):
    """The CE trace carries the prior group az.from_pymc3(trace, prior=prior_checks) writes
    (ng_interp/noble_gas_mcmc.py:276-283, :419; its plots read idata.prior[v], :544): every
    posterior variable, Ae / F linear as the reference converts them before storing, one
    chain; it round-trips through the netCDF-4 file without disturbing the posterior's coords."""
    from noblegas_rtd_mcmc_amd import trace
    from noblegas_rtd_mcmc_amd import workloads as wl
    spec, _ = wl.c1(W=4)
    n = 500
    th = wl.sample_prior(spec, n, np.random.default_rng(10))
    g = trace.prior_group(spec, th)
    assert {"Ae_beta", "m", "Ae", "F", "E", "b", "T", "nu"} <= set(g)
    assert g["m"][0] == ("chain", "draw") and g["m"][1].shape == (1, n)
    assert np.array_equal(g["m"][1][0], th[spec.roles.index("m"), 0])
    D, W = 6, 2
    s = np.stack([wl.sample_prior(spec, W, np.random.default_rng(i)) for i in range(D)])
    res = {"samples": s, "accepted": np.ones((D, 1, W), np.uint8), "accept": np.ones((D, 1, W)),
           "lamb": np.full((1, W), 0.5), "scaling": np.full((1, W), 1e-3), "tuning_steps": 5, "sampling_time": 1.0}
    idd = trace.inference_data(res, spec, observed=spec.ce.obs)
    mc = trace.InferenceData.from_dict(idd, prior=g)
    assert "prior" in mc.groups() and mc.prior["m"].shape == (1, n)
    back = trace.from_netcdf(trace.to_netcdf(mc, str(tmp_path / "ce.netcdf")))
    assert np.array_equal(back["prior"]["m"][1], g["m"][1])
    assert np.array_equal(back["coords"]["draw"], np.arange(D)) and np.array_equal(back["coords"]["chain"], np.arange(W))


def test_writer_uncompressed_and_multiwell(tmp_path):
    """Contiguous (unfiltered) datasets and a third (well) dimension read back as written."""
    from noblegas_rtd_mcmc_amd import h5lite
    groups = {"posterior": {"attrs": {"created_at": "x"},
                            "dims": {"chain": np.arange(4), "draw": np.arange(7), "well": np.arange(3)},
                            "vars": {"T": (("chain", "draw", "well"), np.random.default_rng(0).normal(size=(4, 7, 3)), {}),
                                     "n": (("chain", "draw"), np.arange(28, dtype=np.int64).reshape(4, 7), {})}}}
    p = str(tmp_path / "t.nc")
    w = h5lite.H5Writer(compress=False)
    h5lite.write_netcdf4(p, groups, compress=False)
    back = h5lite.read_netcdf4(p)
    for k, (dims, a, _) in groups["posterior"]["vars"].items():
        d2, a2, _ = back["posterior"]["vars"][k]
        assert d2 == dims and np.array_equal(a2, a)
    assert w is not None


def _var_msgs(path, group, var):
    from noblegas_rtd_mcmc_amd import h5lite
    r = h5lite.H5Reader(path)
    a = r.links(r.links(r.root)[group])[var]
    return {t: bytes(d) for t, f, d in r.messages(a) if t != 0x0C}, r


def test_writer_encodings_pinned_to_shipped_trace(tmp_path):
    """The writer's low-level encodings against the bytes of a shipped trace
    (tests/golden/traces/PLM1.H3.exponential.0.netcdf, netCDF 4.8.1 / HDF5): for a (chain,
    draw) float64 variable of the same shape, the dataspace, datatype, fill-value, filter
    pipeline (shuffle + deflate 4) and chunked-layout messages are byte-identical but for the
    B-tree address, and the chunk B-tree node has the same header and keys (the first key's
    stored size aside: a different compressed payload)."""
    import struct
    from noblegas_rtd_mcmc_amd import h5lite
    ref, rr = _var_msgs(os.path.join(GOLD, "traces", "PLM1.H3.exponential.0.netcdf"), "posterior", "tau1")
    groups = {"posterior": {"attrs": {}, "dims": {"chain": np.arange(3), "draw": np.arange(10000)},
                            "vars": {"tau1": (("chain", "draw"), np.random.default_rng(0).normal(size=(3, 10000)), {})}}}
    p = str(tmp_path / "t.nc")
    h5lite.write_netcdf4(p, groups)
    ours, r = _var_msgs(p, "posterior", "tau1")
    for t in (0x01, 0x03, 0x05, 0x0B):
        assert ours[t] == ref[t], hex(t)
    lay_r, lay_o = ref[0x08], ours[0x08]
    assert lay_o[:3] == lay_r[:3] and lay_o[11:] == lay_r[11:]          # version, class, rank; chunk dims
    def node(rd, lay):
        a = int.from_bytes(lay[3:11], "little")
        b = rd.b
        ksz = 8 + 8 * 3
        head = bytes(b[a:a + 8])
        k0 = bytes(b[a + 24:a + 24 + ksz])
        k1 = bytes(b[a + 24 + ksz + 8:a + 24 + 2 * ksz + 8])
        return head, k0, k1
    hr, k0r, k1r = node(rr, lay_r)
    ho, k0o, k1o = node(r, lay_o)
    assert ho == hr and k0o[4:] == k0r[4:] and k1o == k1r
    assert struct.unpack_from("<I", k0o)[0] > 0


def test_writer_tiles_large_variables_and_empty_draws(tmp_path, monkeypatch):
    """Variables above the chunk bound are tiled (chunk_dims) and indexed by a multi-level v1
    B-tree (more than 2K = 64 chunks: the bound is lowered here to force 2 levels); a
    zero-draw variable stores no chunk.  Both read back exactly; the stored chunk sizes stay
    within the 32-bit fields whatever the variable size."""
    from noblegas_rtd_mcmc_amd import h5lite
    monkeypatch.setattr(h5lite, "CHUNK_BYTES", 2048)
    rng = np.random.default_rng(1)
    big = rng.normal(size=(5, 1999, 3))                   # 240 KB -> 2 KB chunks: 125 chunks
    ints = np.arange(3 * 1001, dtype=np.int64).reshape(3, 1001)
    groups = {"posterior": {"attrs": {"x": "y"}, "dims": {"chain": np.arange(5), "draw": np.arange(1999),
                                                          "well": np.arange(3)},
                            "vars": {"T": (("chain", "draw", "well"), big, {})}},
              "sample_stats": {"attrs": {}, "dims": {"chain": np.arange(3), "draw": np.arange(1001),
                                                     "none": np.arange(0)},
                               "vars": {"n": (("chain", "draw"), ints, {}),
                                        "empty": (("chain", "none"), np.zeros((3, 0)), {})}}}
    p = str(tmp_path / "big.nc")
    h5lite.write_netcdf4(p, groups)
    back = h5lite.read_netcdf4(p)
    assert np.array_equal(back["posterior"]["vars"]["T"][1], big)
    assert np.array_equal(back["sample_stats"]["vars"]["n"][1], ints)
    assert back["sample_stats"]["vars"]["empty"][1].shape == (3, 0)
    assert h5lite.chunk_dims((5, 1999, 3), 8, 2048)[1] < 1999
    assert h5lite.chunk_dims((2048, 50000, 6), 8) != (2048, 50000, 6)        # 4.9 GB: tiled at 4 MiB
    r = h5lite.H5Reader(p)
    a = r.links(r.links(r.root)["posterior"])["T"]
    lay = [bytes(d) for t, f, d in r.messages(a) if t == 0x08][0]
    bt = int.from_bytes(lay[3:11], "little")
    assert r.b[bt + 5] == 1                                # the root is an internal node (2 levels)


def test_multilevel_chunk_btree_layout(tmp_path, monkeypatch):
    """The v1 B-tree of a tiled variable, decoded node by node against the format's rules
    (HDF5 spec, "Version 1 B-trees"): every node is a TREE of type 1 with its level, holds
    1..2K entries, its left / right sibling addresses link the nodes of one level in order
    (undefined at the ends); keys are monotone in chunk order; a node's right key (after its
    last child) equals its right sibling's first key (the last node of a level: the dataset's
    end key); a parent's key i is child i's first key and its key i + 1 child i's right key;
    the leaves' chunk addresses cover every chunk once."""
    import struct
    from noblegas_rtd_mcmc_amd import h5lite
    monkeypatch.setattr(h5lite, "CHUNK_BYTES", 2048)
    rng = np.random.default_rng(2)
    big = rng.normal(size=(3, 9001, 2))      # 432 KB in 2 KB chunks: more than 2K = 64 leaves, two levels
    p = str(tmp_path / "tree.nc")
    groups = {"posterior": {"attrs": {}, "dims": {"chain": np.arange(3), "draw": np.arange(9001), "well": np.arange(2)},
                            "vars": {"T": (("chain", "draw", "well"), big, {})}}}
    h5lite.write_netcdf4(p, groups)
    assert np.array_equal(h5lite.read_netcdf4(p)["posterior"]["vars"]["T"][1], big)
    r = h5lite.H5Reader(p)
    a = r.links(r.links(r.root)["posterior"])["T"]
    lay = [bytes(d) for t, f, d in r.messages(a) if t == 0x08][0]
    root = int.from_bytes(lay[3:11], "little")
    b = r.b
    rank = 4                                               # 3 dims + the element dimension
    ksz = 8 + 8 * rank
    K2 = 2 * h5lite._CHUNK_K
    UNDEF = h5lite.UNDEF

    def node(addr):
        assert b[addr:addr + 4] == b"TREE" and b[addr + 4] == 1
        level, n = b[addr + 5], struct.unpack_from("<H", b, addr + 6)[0]
        left, right = struct.unpack_from("<QQ", b, addr + 8)
        q = addr + 24
        keys, kids = [], []
        for _ in range(n):
            keys.append(bytes(b[q:q + ksz]))
            kids.append(struct.unpack_from("<Q", b, q + ksz)[0])
            q += ksz + 8
        keys.append(bytes(b[q:q + ksz]))
        return level, n, left, right, keys, kids

    def offs(key):
        return struct.unpack_from("<%dQ" % rank, key, 8)

    levels = {}
    def walk(addr, depth_level):
        lv, n, left, right, keys, kids = node(addr)
        assert lv == depth_level and 1 <= n <= K2
        levels.setdefault(lv, []).append((addr, left, right, keys))
        for i, kid in enumerate(kids):
            if lv:
                klv, kn, _, _, kkeys, _ = node(kid)
                assert kkeys[0] == keys[i] and kkeys[-1] == keys[i + 1], (lv, i)
                walk(kid, lv - 1)
        return kids
    top = node(root)[0]
    assert top >= 1                                        # the bound above forces 2 levels
    walk(root, top)
    chunks = []
    for lv, nodes in levels.items():
        for j, (addr, left, right, keys) in enumerate(nodes):
            assert left == (nodes[j - 1][0] if j else UNDEF) and right == (nodes[j + 1][0] if j + 1 < len(nodes) else UNDEF)
            if j + 1 < len(nodes):
                assert keys[-1] == nodes[j + 1][3][0], (lv, j)
            ks = [offs(k) for k in keys]
            assert all(x < y for x, y in zip(ks, ks[1:])), (lv, j)
            if lv == 0:
                chunks += ks[:-1]
    cd = h5lite.chunk_dims(big.shape, 8)
    want = [tuple(int(v) for v in o) + (0,) for o in np.array(np.meshgrid(
        *[range(0, d, c) for d, c in zip(big.shape, cd)], indexing="ij")).reshape(3, -1).T]
    assert chunks == want
    last = offs(levels[0][-1][3][-1])
    assert last == tuple(int(o) + int(c) for o, c in zip(want[-1][:3], cd)) + (8,)


def test_summary_hdi_is_narrowest_interval():
    """trace.hdi is ArviZ's HDI (the narrowest window of floor(p n) + 1 order statistics): it
    equals a brute-force search on small samples, for a skewed posterior (Exp(1)) it is
    [~0, ~ln(1/0.06)] where the equal-tailed interval is [0.031, 2.81], and summary() carries
    it under ArviZ's column names; Dataset.dims is {dimension: size} as xarray's."""
    from noblegas_rtd_mcmc_amd import trace
    rng = np.random.default_rng(4)
    for n in (2, 3, 17, 100):
        a = rng.lognormal(0, 1.5, n)
        s = np.sort(a)
        k = int(np.floor(0.94 * n))
        best = min(range(n - k), key=lambda i: (s[i + k] - s[i], i))
        assert trace.hdi(a) == (s[best], s[best + k])
    x = rng.exponential(1.0, 400000)
    lo, hi = trace.hdi(x)
    assert lo < 1e-3 and abs(hi - np.log(1 / 0.06)) < 0.02
    idd = {"posterior": {"tau": (("chain", "draw"), x.reshape(4, -1))},
           "sample_stats": {"accepted": (("chain", "draw"), np.ones((4, 100000), np.uint8))}}
    mc = trace.InferenceData.from_dict(idd)
    df = trace.summary(mc)
    assert list(df.columns) == ["mean", "sd", "hdi_3%", "hdi_97%"]
    assert df.loc["tau", "hdi_3%"] == lo and df.loc["tau", "hdi_97%"] == hi
    assert df.loc["tau", "sd"] == x.std(ddof=1)
    assert mc.posterior.dims == {"chain": 4, "draw": 100000}
