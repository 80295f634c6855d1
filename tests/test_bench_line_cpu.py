"""bench.py's printed line stays driver-parsable: the last stdout line is one JSON object of
at most HEADLINE_MAX_BYTES carrying the contract's fields, with the side legs summarised
(the round-5 line grew to 30 KB and the driver's bounded tail could not parse it)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline",
            "value_amortized_20k", "exact_value")


def _round5_full():
    # the builder's round-5 full line (30 KB): every side leg at its real size
    with open(os.path.join(REPO, "profiles", "r05fin_bench20.json")) as f:
        full = json.load(f)
    # grow it further, as round 6 adds legs: extra reference runs and the CE inference runs
    rr = full["reference_runs"]
    rr["runs"] = rr["runs"] + [dict(rr["runs"][0], run="PLM1.CFC12.SF6.H3.He4_ter.dispersion%s.123" % s)
                               for s in ("", "-piston")]
    full["ce_runs"] = {"runs": [{"run": "%s.CE.4chains" % w, "wall_s": 1.0, "speedup_vs_reference": 100.0,
                                 "accept_rate": 0.3} for w in ("PLM1", "PLM6", "PLM7")], "total_wall_s": 3.0}
    return full


def test_headline_bounded_and_complete():
    full = _round5_full()
    assert len(json.dumps(full)) > 25000
    line = bench.headline(full, "gpurun_out/bench_side.json")
    s = json.dumps(line)
    assert len(s) < bench.HEADLINE_MAX_BYTES <= 8000
    assert "\n" not in s
    for k in REQUIRED:
        assert k in line, k
    assert line["value"] == full["value"] and line["ms_per_step"] == full["ms_per_step"]
    assert line["roofline"] == full["roofline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"]
    side = line["side"]
    assert side["file"] == "gpurun_out/bench_side.json"
    assert len(side["models_kernel_us"]) == len(full["models"])
    assert len(side["reference_runs"]["runs"]) == len(full["reference_runs"]["runs"])
    assert len(side["ce_runs"]["runs"]) == 3
    assert "transformed" in side["sampler"]


def test_headline_drops_summaries_before_overflowing():
    full = _round5_full()
    full["models"] = {"m%03d" % i: dict(full["models"]["exponential"]) for i in range(600)}
    s = json.dumps(bench.headline(full))
    assert len(s) <= bench.HEADLINE_MAX_BYTES
    assert json.loads(s)["value"] == full["value"]


def test_headline_with_failed_legs():
    full = _round5_full()
    full["models"] = {"error": "RuntimeError('x')"}
    full["reference_runs"] = {"error": "RuntimeError('y' * 5000)"}
    full["sampler"] = {"error": "boom"}
    full["cpu_baseline"] = None
    line = bench.headline(full)
    assert len(json.dumps(line)) < bench.HEADLINE_MAX_BYTES
    assert line["cpu_baseline"] is None
    assert line["side"]["reference_runs"]["error"].startswith("RuntimeError")
