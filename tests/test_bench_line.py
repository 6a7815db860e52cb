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
    # a full record as bench.py writes it to --detail-out (this round's checkpoint)
    with open(os.path.join(ROOT, "profiles", "r04m_bench_detail.json")) as f:
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


def test_pmc_traffic_marks_other_code_stale(tmp_path, monkeypatch):
    # counters stamped with the current sources' digest are current; any other stamp is stale, and a
    # file without one is "unknown" (None); the headline carries the mark beside the number
    prof = tmp_path / "profiles"
    prof.mkdir()
    entry = {"fetch_bytes": 2.0, "fetch_bytes_raw": 1.0, "fetch_factor": 2.0, "fetch_class": "stream",
             "write_bytes": 1.0}
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "source_digest", lambda: "abc")
    (prof / "r09a_pmc.json").write_text(json.dumps({"k": entry}))
    assert bench.pmc_traffic_detail("k")["stale"] is None
    (prof / "r09b_pmc.json").write_text(json.dumps({"k": entry, "_code": "old"}))
    assert bench.pmc_traffic_detail("k")["stale"] is True
    (prof / "r09c_pmc.json").write_text(json.dumps({"k": entry, "_code": "abc"}))
    td = bench.pmc_traffic_detail("k")
    assert td["stale"] is False and td["bytes"] == 3.0 and td["source"] == os.path.join("profiles", "r09c_pmc.json")
    r = bench._roof_short({"bound": "hbm", "achieved": 1.0, "peak": 2.0, "unit": "GB/s", "frac": 0.5,
                           "traffic": 3.0, "traffic_detail": td})
    assert r["traffic_stale"] is False


def test_source_digest_is_stable():
    assert bench.source_digest() == bench.source_digest()
    assert len(bench.source_digest()) == 16


def test_pmc_staleness_is_per_leg(tmp_path, monkeypatch):
    # a file stamped per leg: a kernel is stale only when its own leg's sources changed
    prof = tmp_path / "profiles"
    prof.mkdir()
    entry = {"fetch_bytes": 2.0, "fetch_bytes_raw": 1.0, "fetch_factor": 2.0, "fetch_class": "stream",
             "write_bytes": 1.0}
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "source_digest", lambda leg=None: {"chain": "new"}.get(leg, "same"))
    (prof / "r09a_pmc.json").write_text(json.dumps({
        "chain_rows": entry, "phmm_forward<float>": entry, "_code": "old",
        "_code_legs": {"phmm": "same", "fmi": "same", "chain": "old", "bsw": "same"}}))
    assert bench.pmc_traffic_detail("chain_rows")["stale"] is True
    assert bench.pmc_traffic_detail("phmm_forward<float>")["stale"] is False


def test_leg_sources_cover_every_kernel_file():
    # every kernel source belongs to one leg or is shared, so no change escapes the staleness mark
    for f in bench.source_files():
        rel = os.path.relpath(f, bench.ROOT)
        b = os.path.basename(rel)
        if not rel.endswith((".hip", ".cpp", ".h")) or b.startswith(("gb_common", "gb.h")):
            continue
        assert sum(b.startswith(p) for p in bench.LEG_SOURCES.values()) == 1, rel
