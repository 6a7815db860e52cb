"""bench.py's stdout contract: the driver parses ONE compact JSON line (its capture keeps only the tail
of stdout + stderr, so round 3's 24 KB line was unparseable). The headline is built from the full
record and must stay under HEADLINE_MAX_BYTES while keeping roofline and cpu_baseline for every leg."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _record():
    # a full record in the shape bench.py's main() assembles (last round's real line)
    with open(os.path.join(ROOT, "profiles", "r03zc_bench.json")) as f:
        d = json.load(f)
    bench.add_per_core(d, 256, 128)
    return d


def test_headline_fits_and_keeps_contract_fields():
    d = _record()
    h = bench.headline(d, "profiles/x_bench_detail.json")
    s = json.dumps(h)
    assert len(s) < bench.HEADLINE_MAX_BYTES
    assert len(s) < 3500  # room for the stderr progress lines inside the driver's tail
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in h
    assert h["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    for r in (h["roofline"], h["fmi"]["roofline"], h["chain"]["roofline"], h["bsw"]["roofline"]):
        for k in ("bound", "achieved", "peak", "unit", "frac"):
            assert k in r
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 2e-3
    for cb in (h["cpu_baseline"], h["fmi"]["cpu_baseline"], h["chain"]["cpu_baseline"], h["bsw"]["cpu_baseline"]):
        for k in ("value", "cores", "kind"):
            assert k in cb
        assert cb["all_core_physical"][1] == 128
    assert h["value"] == round(d["value"], 2)


def test_headline_drops_optional_parts_when_too_big():
    d = _record()
    d["config"]["workload"] = "x" * 3000
    h = bench.headline(d)
    assert len(json.dumps(h)) <= bench.HEADLINE_MAX_BYTES or "small" not in h
    assert "roofline" in h and "cpu_baseline" in h


def test_headline_partial_legs():
    d = _record()
    for k in ("fmi", "chain", "bsw", "small", "shard_proxy"):
        d[k] = None
    h = bench.headline(d)
    assert h["fmi"] is None and h["roofline"]["frac"] > 0
    json.dumps(h)
