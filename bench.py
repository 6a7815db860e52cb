#!/usr/bin/env python3
"""bench.py -- GenomicsBench hot kernels on MI355X (driver contract: one JSON line on rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batches B] [--no-cpu-baseline]

Metric (BASELINE.json): "GCUPS (phmm) + Mreads/s (fmi) on 'large' set at 1/2/4/8 MI355X".
phmm (the line's `value`): a step = one PairHMM forward pass (f32 kernel + f64 fallback kernel +
log10 epilogue) over this rank's shard of one 'large'-shaped synthetic job of B batches
(gen.phmm_dataset, seed 1) already resident in HBM; value = cells of the whole job x K / max-over-ranks
wall time, in GCUPS.
chain / bsw (the "chain" / "bsw" objects): a step = chain_dp over every call of the rank's shard of a
'large'-shaped set (10k calls, 25 M anchors, seed 5; Manchors/s) / the banded SW extension of every
pair of the rank's shard of a 'large'-shaped set (10 606 460 pairs, seed 11; GCUPS over the
reference's inner-loop cells).
fmi (the line's "fmi" object): a step = the whole fmi.cpp per-batch pipeline (SMEMs, reseeding,
LAST seeds, per-read sort) over every read of the rank's shard (whole 512-read batches) of a 10 M-read
set (gen.fmi_reads, seed 8) against a 512 Mbp genome-like synthetic reference (+RC: 1.024 G BWT rows,
1.02 GB CP_OCC) built on the GPU and replicated on every rank; value = reads x K / max-over-ranks time.
"small" object: the same four legs on the 'small'-shaped sets (phmm small batches, 1 M fmi reads over
the same index, 1 000 chain calls, 100 000 bsw pairs), sharded the same way.
Strong scaling (default): every rank generates the same seeded set and keeps its contiguous shard
(shard.py: testcases by cells, reads by whole batches, calls by anchors, pairs by cell estimate), so
N GPUs share one fixed job and the shards concatenate back into the 1-GPU output. --scaling weak
gives every rank its own full-size set (seed + rank) instead. There is no data-path collective;
torch.distributed only provides the barrier and the max-time / sum-work reductions.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Peaks (MI355X_MICROARCH.md, chip-level parameters): 256 CU x 4 SIMD x 32 lanes x 2.4 GHz
PEAK_F32_OPS = 256 * 4 * 32 * 2.4e9  # non-FMA FP32 VALU ops/s = 78.6e12 (157.3 TF counts FMA as 2)
PEAK_F64_OPS = PEAK_F32_OPS / 2      # FP64 vector peak 78.6 TF (FMA=2) -> 39.3e12 non-FMA ops/s
PHMM_FLOP_PER_CELL = 12              # 12 FP ops per cell, no FMA
PEAK_HBM = 8.0e12                    # HBM3E spec bytes/s (MI355X_MICROARCH.md)
FMI_BYTES_PER_EXT = 128              # 2 x 64-B CP_OCC lines per backwardExt
FMI_OCC_BYTES_PER_EXT = 35           # bytes of the one Occ32 line the kernel gathers per extension (DESIGN.md fmi)
SA_BYTES_PER_STEP = 64               # one 64-B Occ2 line per LF step of an SA lookup
SA_BYTES_PER_COORD = 24              # row in, sampled-SA entry, coordinate out (8 B each)
CHAIN_OPS_PER_PAIR = 25              # ~25 int32/fp64 ops per visited (i, j) pair
PEAK_CHAIN_OPS = PEAK_F64_OPS        # INT32/FP64 VALU, 39.3e12 lane-op/s
BSW_OPS_PER_CELL = 13                # ~13 int ops per scalar inner-loop iteration
PEAK_INT_OPS = PEAK_F32_OPS          # 32-bit integer VALU lane-ops/s = 78.6e12


# kernel sources per leg (file-name prefixes under csrc/ and include/), for the PMC staleness mark
LEG_SOURCES = {"phmm": ("phmm", "gb_phmm", "gkl"), "fmi": ("fmi", "gb_fmi", "FMI_search"),
               "chain": ("chain", "gb_chain", "minimap2_chain"), "bsw": ("bsw", "gb_bsw", "bandedSWA")}
KERNEL_LEG = {"phmm_forward<float>": "phmm", "phmm_forward<double>": "phmm", "smem_search": "fmi",
              "smem_heavy": "fmi", "sa_walk": "fmi", "chain_rows": "chain", "chain_kernel": "chain",
              "verify_lanes": "chain", "bsw_lane_kernel": "bsw", "bsw_extend_kernel": "bsw"}


def source_files():
    import glob
    return sorted(glob.glob(os.path.join(ROOT, "genomicsbench_palisade_amd", "csrc", "*"))
                  + glob.glob(os.path.join(ROOT, "include", "*.h")) + glob.glob(os.path.join(ROOT, "include", "*", "*.h"))
                  + [os.path.join(ROOT, "Makefile")])  # build flags shape the kernels too


def digest_of(named):
    """sha256 (16 hex) over (relative name, bytes) pairs of .hip / .cpp / .h sources, in name order.
    With a leg, only that leg's sources (LEG_SOURCES) and the shared ones (gb_common*, gb.h)."""
    import hashlib
    h = hashlib.sha256()
    for rel, data in sorted(named):
        if rel.endswith((".hip", ".cpp", ".h")) or os.path.basename(rel) == "Makefile":
            h.update(rel.encode())
            h.update(data)
    return h.hexdigest()[:16]


def _leg_match(rel, leg):
    b = os.path.basename(rel)
    return leg is None or b.startswith(LEG_SOURCES[leg]) or b.startswith(("gb_common", "gb.h")) or b == "Makefile"


def source_digest(leg=None) -> str:
    """Digest of the kernel sources (csrc/ and include/), or of one leg's: tools/pmc_summary.py
    stamps them into each profiles/*_pmc.json, and a bench line's traffic_detail says whether its
    counters were taken on the kernel code being measured ("stale": false) or on other code (true;
    null for a file without a stamp)."""
    named = []
    for f in source_files():
        rel = os.path.relpath(f, ROOT)
        if _leg_match(rel, leg):
            with open(f, "rb") as fh:
                named.append((rel, fh.read()))
    return digest_of(named)


def _stale(d, kernel):
    leg = KERNEL_LEG.get(kernel)
    legs = d.get("_code_legs") or {}
    if leg and leg in legs:
        return legs[leg] != source_digest(leg)
    return (d["_code"] != source_digest()) if "_code" in d else None


def pmc_traffic_detail(kernel: str, leg: str = ""):
    """Per-launch HBM bytes of `kernel` from the newest committed profiles/*_pmc.json (rocprofv3
    FETCH_SIZE and WRITE_SIZE passes of this same bench configuration, tools/gpu_prof.sh +
    tools/pmc_summary.py, fetch corrected by the calibrated factor of the kernel's read class);
    None when no profile covers it. PMC cannot run inside the timed process. leg = "human": the
    profiles/*_human_pmc.json passes of `bench.py --only fmi_human` (the same kernel on the human-scale
    index)."""
    import glob
    # checkpoint order is the file name (r01k < r02d < r02k < r03a ...), never mtime: on the GPU box
    # mtimes are the push order. GB_PMC_CHECKPOINT pins one checkpoint.
    suffix = f"_{leg}_pmc.json" if leg else "_pmc.json"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*" + suffix)), key=os.path.basename)
    if not leg:
        files = [f for f in files if os.path.basename(f).count("_") == 1]  # rNNx_pmc.json only
    pin = os.environ.get("GB_PMC_CHECKPOINT")
    if pin:
        files = [f for f in files if os.path.basename(f) == f"{pin}{suffix}"]
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if kernel in d and "fetch_factor" in d[kernel]:
            k = d[kernel]
            return {"bytes": k["fetch_bytes"] + k["write_bytes"], "fetch_bytes": k["fetch_bytes"],
                    "fetch_bytes_raw": k["fetch_bytes_raw"], "fetch_factor": k["fetch_factor"],
                    "fetch_class": k["fetch_class"], "write_bytes": k["write_bytes"],
                    "source": os.path.relpath(f, ROOT),
                    "stale": _stale(d, kernel)}
    return None


def pmc_traffic(kernel: str, leg: str = ""):
    """roofline.traffic: corrected HBM bytes per launch (number), or None."""
    d = pmc_traffic_detail(kernel, leg)
    return None if d is None else d["bytes"]


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return world, rank, local


class Dist:
    def __init__(self, world):
        self.world = world
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group(backend="gloo")
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def device_sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


def cpu_baseline_phmm(ta, sample_seconds: float, gpu=None, threads=None):
    """Reference GKL kernels (oracle/_ref, kind 'reference') -- or the C restatement when the
    reference build is absent (kind 'port') -- on a bounded random sample of the same job.
    gpu = (results, raw f32, raw f64) of the GPU pass over `ta`: the sample's outputs are compared
    with them bit for bit and the run fails on any mismatch."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from genomicsbench_palisade_amd._tc import TestcaseArray  # noqa: F401
    if threads is None:
        threads = max(1, min(16, _cores()))  # the GPU box grants 16 CPUs per GPU
    ref = oracle_lib.ref_phmm()
    rng = np.random.default_rng(123)
    order = rng.permutation(ta.n)
    kind = "reference" if ref is not None else "port"
    engine = 512 if (ref is not None and ref.ref_phmm_has_avx512()) else 256
    last = {}

    def run(sub):
        n = sub.n
        out, rf, rd = np.zeros(n), np.zeros(n, np.float32), np.zeros(n)
        t0 = time.perf_counter()
        if ref is not None:
            ref.ref_phmm_batch(ctypes.addressof(sub.arr), n, out.ctypes.data, rf.ctypes.data,
                               rd.ctypes.data, engine, threads)
        else:
            oracle_lib.oracle().phmm_oracle_batch(ctypes.addressof(sub.arr), n, out.ctypes.data,
                                                  rf.ctypes.data, rd.ctypes.data, None, threads)
        last["out"] = (out, rf, rd)
        return time.perf_counter() - t0

    # warm the reference's static tables (Context ctors) outside the timed region, calibrate on a
    # small sample, then time ~sample_seconds of work: a random subset of the job, or the whole
    # job repeated when it is shorter than that
    run(ta.subset(order[:8]))
    cal = ta.subset(order[:max(threads * 32, 256)])
    t = run(cal)
    rate = cal.cells() / max(t, 1e-6)
    ncells_target = rate * sample_seconds
    cum = np.cumsum(ta.np_arr["rslen"][order].astype(np.int64) * ta.np_arr["haplen"][order])
    m = int(min(ta.n, max(64, np.searchsorted(cum, ncells_target))))
    sub = ta.subset(order[:m])
    reps = max(1, int(round(ncells_target / max(sub.cells(), 1))))
    t = sum(run(sub) for _ in range(reps))
    gcups = reps * sub.cells() / t / 1e9
    eng = {512: "AVX-512", 256: "AVX2"}[engine] if ref is not None else "C"
    res = {"value": gcups, "unit": "GCUPS", "cores": threads, "kind": kind,
           "sample": f"{m} of {ta.n} testcases ({sub.cells() / 1e9:.2f} G cells, random) of the same "
                     f"job x {reps} passes, {eng} GKL kernels, OpenMP {threads} threads, {t:.1f} s"}
    if gpu is not None:
        from genomicsbench_palisade_amd.phmm import parity_mismatches
        sel = order[:m]
        # what computelikelihoodsboth exposes, bit for bit: final log10, raw f64, the fallback choice,
        # raw f32 of the passing testcases (below MIN_ACCEPTED the f32 early exit may leave 0)
        bad = parity_mismatches(tuple(np.ascontiguousarray(g[sel]) for g in gpu), last["out"])
        dropped = bad.pop("f32_dropped")
        res["parity_check"] = {"testcases": int(m), "of": int(ta.n), "mismatches": bad,
                               "f32_early_exit_dropped": dropped,
                               "bit_exact": not any(bad.values()),
                               "against": f"reference GKL {eng}" if ref is not None else "C restatement"}
        if any(bad.values()):
            raise SystemExit(f"phmm parity FAILED on the CPU-baseline sample: {res['parity_check']}")
    return res


def cpu_baseline_fmi(oracle_index, codes, lens, sample_seconds: float, fmi=None, idx=None):
    """The bwa-mem2 SMEM restatement (oracle/fmi_oracle.c, kind 'port': the reference FMI_search.cpp
    is not buildable here without Palisade) over a bounded sample (whole 512-read batches) of the same
    reads. The sample's SMEM lists are compared with the GPU's on the same reads (bit-exact)."""
    threads = max(1, min(16, _cores()))
    cal = min(len(lens), 4000 * threads)
    t0 = time.perf_counter()
    oracle_index.run_threaded(codes[:cal], lens[:cal], threads)
    rate = cal / max(time.perf_counter() - t0, 1e-6)
    m = int(min(len(lens), max(cal, rate * sample_seconds)))
    m = min(len(lens), max(512, m // 512 * 512))
    t0 = time.perf_counter()
    _, ocalls, parts = oracle_index.run_threaded(codes[:m], lens[:m], threads, collect=True)
    t = time.perf_counter() - t0
    check = None
    if fmi is not None:
        rs = fmi.Reads(idx, codes[:m], lens[:m])
        rs.search(19)
        sm, tot, bc, _ = rs.results(batch_size=512)
        _, _, gcalls = rs.timing()
        rs.close()
        exp = np.concatenate(parts) if parts else sm[:0]
        same = tot == len(exp) and all((sm[f] == exp[f]).all() for f in ("rid", "m", "n", "k", "l", "s"))
        check = {"reads": m, "smems": int(tot), "bit_exact": bool(same), "backwardExt_equal": bool(gcalls == ocalls)}
        if not (same and gcalls == ocalls):
            raise SystemExit(f"fmi parity FAILED on the CPU-baseline sample: {check}")
    port = {"value": m / t / 1e6, "unit": "Mreads/s", "cores": threads, "kind": "port",
            "sample": f"first {m} of {len(lens)} reads of the same shard, C restatement of bwa-mem2 "
                      f"FMI_search (batches of 512 over {threads} threads), {t:.1f} s",
            "parity_check": check}
    # reference kind: bwa v1's own mem_collect_intv (tools/bwa, unmodified, oracle/_ref) over a bwt_t
    # rebuilt from the same CP_OCC tables -- same intervals (tests/test_fmi_oracle.py), bwa v1 speed
    import fmi_util
    lib = fmi_util.ref_bwa()
    if lib is None:
        return port
    n_, _, s_ = idx.info() if idx is not None else oracle_index.info()
    bwt = fmi_util.bwa_from_tables(lib, n_, s_, oracle_index._occ)
    t0 = time.perf_counter()
    tot = fmi_util.bwa_collect_threaded(lib, bwt, codes[:m], lens[:m], threads)
    t = time.perf_counter() - t0
    lib.ref_bwa_free(bwt)
    if check is not None and tot != check["smems"]:
        raise SystemExit(f"bwa v1 interval count {tot} != GPU SMEM count {check['smems']} on the baseline sample")
    return {"value": m / t / 1e6, "unit": "Mreads/s", "cores": threads, "kind": "reference",
            "sample": f"first {m} of {len(lens)} reads of the same shard, bwa v1 mem_collect_intv (tools/bwa "
                      f"bwt_smem1 + bwt_seed_strategy1, compiled unmodified) over a bwt_t rebuilt from the same "
                      f"CP_OCC tables, {threads} threads, {t:.1f} s; {tot} intervals == GPU SMEM count",
            "port": port, "parity_check": check}


def _cores():
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def cpu_host():
    """The host the CPU baselines ran on (nproc, affinity, model)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity": _cores(), "model": model,
            "physical_cores": physical_cores(),
            "note": "cpu_baseline.cores = threads used (<= 16, the GPU box's CPU share per GPU); "
                    "per_core = value / cores; all_core_estimate = per_core x nproc "
                    "(linear over every logical CPU, i.e. generous to the CPU: the box only grants 16 CPUs to a run)"}


def physical_cores():
    """Distinct (physical id, core id) pairs of /proc/cpuinfo: the host's physical cores."""
    seen, phys, core = set(), None, None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("physical id"):
                    phys = ln.split(":", 1)[1].strip()
                elif ln.startswith("core id"):
                    core = ln.split(":", 1)[1].strip()
                elif not ln.strip():
                    if core is not None:
                        seen.add((phys, core))
                    phys = core = None
    except OSError:
        return None
    if core is not None:
        seen.add((phys, core))
    return len(seen) or None


def add_per_core(obj, cores_all=None, cores_phys=None):
    """cpu_baseline objects (nested ones too) get value per thread used and the all-core estimates
    of BASELINE.md section 3: per thread x every logical CPU of the host (an upper bound for the CPU,
    SMT siblings do not double a core's rate) and per thread x the physical cores."""
    if cores_all is None:
        cores_all = os.cpu_count()
    if cores_phys is None:
        cores_phys = physical_cores()
    if isinstance(obj, dict):
        if "cpu_baseline" in obj and isinstance(obj["cpu_baseline"], dict):
            cb = obj["cpu_baseline"]
            if cb.get("value") and cb.get("cores"):
                cb["per_core"] = cb["value"] / cb["cores"]
                if cores_all:
                    cb["all_core_estimate"] = {"value": cb["per_core"] * cores_all, "cores": cores_all}
                if cores_phys:
                    cb["all_core_estimate_physical"] = {"value": cb["per_core"] * cores_phys, "cores": cores_phys}
            if isinstance(cb.get("port"), dict) and cb["port"].get("value") and cb["port"].get("cores"):
                cb["port"]["per_core"] = cb["port"]["value"] / cb["port"]["cores"]
        for v in obj.values():
            add_per_core(v, cores_all, cores_phys)


HEADLINE_MAX_BYTES = 4096


def _sig(x, n=4):
    """x rounded to n significant digits (floats only), for the compact headline."""
    if isinstance(x, float):
        if x == 0 or x != x:
            return x
        from math import floor, log10
        return round(x, max(0, n - 1 - int(floor(log10(abs(x))))))
    return x


def _pick(d, keys):
    if not isinstance(d, dict):
        return None
    return {k: _sig(d[k]) for k in keys if k in d and d[k] is not None}


def _cpu_short(cb):
    if not isinstance(cb, dict):
        return None
    out = _pick(cb, ("value", "unit", "cores", "kind", "per_core"))
    pc = cb.get("parity_check") or {}
    if "bit_exact" in pc:
        out["bit_exact"] = bool(pc["bit_exact"])
    for k, short in (("all_core_estimate", "all_core_logical"), ("all_core_estimate_physical", "all_core_physical")):
        if isinstance(cb.get(k), dict):
            out[short] = [_sig(cb[k]["value"]), cb[k]["cores"]]
    return out


def _roof_short(r):
    out = _pick(r, ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic"))
    if out and isinstance(out.get("kernel"), str):
        out["kernel"] = out["kernel"].split(" ")[0]
    td = r.get("traffic_detail") if isinstance(r, dict) else None
    if out and out.get("traffic") is not None and isinstance(td, dict):
        # counters taken on other kernel code than the one measured: say so beside the number
        out["traffic_stale"] = td.get("stale")
    return out


def _proxy_short(sp):
    """of / ratio_min / speedup of the largest N, and the projected speedup at every N timed."""
    out = {"of": sp.get("of"), "ratio_min": _sig(sp.get("ratio_min_vs_full")),
           "speedup": _sig(sp.get("projected_speedup"))}
    if isinstance(sp.get("by_n"), dict):
        out["speedup_by_n"] = {n: _sig(o.get("projected_speedup")) for n, o in sp["by_n"].items()}
    return out


def _leg_short(leg):
    if not isinstance(leg, dict):
        return None
    out = _pick(leg, ("value", "unit", "ms_per_step"))
    wl = (leg.get("config") or {}).get("workload")
    if isinstance(wl, str):
        import re
        w = re.sub(r" \([^)]*\)", "", wl.split(";")[0])
        if len(w) > 140:  # cut at a clause boundary, never inside a token ("minSeedLen 19")
            w = w[:140].rsplit(", ", 1)[0]
        out["workload"] = w
    out["roofline"] = _roof_short(leg.get("roofline"))
    out["cpu_baseline"] = _cpu_short(leg.get("cpu_baseline"))
    if isinstance(leg.get("split_stats"), dict):
        out["fixups"] = leg["split_stats"].get("fixup_blocks")
    sp = leg.get("shard_proxy")
    if isinstance(sp, dict):
        out["shard_proxy"] = _proxy_short(sp)
    return out


def headline(line: dict, detail_path=None) -> dict:
    """The one compact JSON line the driver parses (<= HEADLINE_MAX_BYTES): the contract's fields, the
    phmm headline's roofline and cpu_baseline, and per leg (fmi, chain, bsw, + chain backtrack, fmi
    human-scale and the 'small' values) value / ms_per_step / workload / roofline / cpu_baseline.
    Everything else (shard proxies' per-rank times, drop-ins, traffic_detail, parity-check objects)
    goes to the detail file named in `detail`."""
    h = {k: line.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                  "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    h["value"] = _sig(h["value"], 6)
    cfg = line.get("config") or {}
    h["config"] = {"workload": cfg.get("workload"), "parallelism": cfg.get("parallelism")}
    h["roofline"] = _roof_short(line.get("roofline"))
    h["cpu_baseline"] = _cpu_short(line.get("cpu_baseline"))
    sp = line.get("shard_proxy")
    if isinstance(sp, dict):
        h["shard_proxy"] = _proxy_short(sp)
    if isinstance(line.get("roofline_f64"), dict):
        h["roofline_f64_frac"] = _sig(line["roofline_f64"].get("frac"))
    if line.get("f32_only_gcups"):
        h["f32_only_gcups"] = _sig(line["f32_only_gcups"])
    for leg in ("fmi", "chain", "bsw"):
        h[leg] = _leg_short(line.get(leg))
    fm, ch = line.get("fmi") or {}, line.get("chain") or {}
    if isinstance(ch.get("backtrack"), dict):
        h["chain"]["backtrack"] = _pick(ch["backtrack"], ("value", "unit"))
        h["chain"]["backtrack"]["frac"] = _sig((ch["backtrack"].get("roofline") or {}).get("frac"))
    if isinstance(fm.get("human"), dict):
        hu = fm["human"]
        h["fmi"]["human"] = _pick(hu, ("value", "unit"))
        h["fmi"]["human"]["frac"] = _sig((hu.get("roofline") or {}).get("frac"))
        h["fmi"]["human"]["rows"] = (hu.get("config") or {}).get("workload", "").split("BWT rows ")[-1].split(",")[0]
    if isinstance(line.get("small"), dict):
        h["small"] = {k: _sig(v.get("value")) for k, v in line["small"].items() if isinstance(v, dict)}
    # world > 1: gathered shard outputs vs a 1-rank pass of the whole set, per leg (rank_check)
    rc = {"phmm": line.get("rank_check")}
    for leg in ("fmi", "chain", "bsw"):
        rc[leg] = (line.get(leg) or {}).get("rank_check")
    for leg, v in (line.get("small") or {}).items():
        if isinstance(v, dict):
            rc["small_" + leg] = v.get("rank_check")
    rc = {k: bool(v.get("bit_exact")) for k, v in rc.items() if isinstance(v, dict)}
    if rc:
        h["rank_check_bit_exact"] = rc
    if detail_path:
        h["detail"] = detail_path
    # never let the line outgrow the driver's capture: drop the least important parts first
    for drop in (("small",), ("fmi", "human"), ("chain", "backtrack"), ("data",)):
        if len(json.dumps(h)) <= HEADLINE_MAX_BYTES:
            break
        tgt = h
        for k in drop[:-1]:
            tgt = tgt.get(k) or {}
        tgt.pop(drop[-1], None)
    return h


def cpu_baseline_chain(calls, sample_seconds: float, gpu=None):
    """The reference's scalar chain_dp (tools/minimap2-acceleration/kernel/scalar, compiled from the
    reference tree into oracle/_ref, kind 'reference'; the C restatement when absent, kind 'port')
    over a bounded random sample of the same calls, OpenMP over calls like host_chain_kernel.
    gpu = (scores, parents, targets, peaks) of the GPU pass over `calls`: the reference is run once
    over every call first and its outputs compared bit for bit (the run fails on a mismatch)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from genomicsbench_palisade_amd import gen
    threads = max(1, min(16, _cores()))
    ref = oracle_lib.ref_chain()
    rng = np.random.default_rng(321)
    order = rng.permutation(calls.ncalls)
    check = None
    if gpu is not None:
        exp = oracle_lib.ref_chain_run(ref, calls, threads) if ref is not None else oracle_lib.chain_oracle(calls, threads)
        bad = {name: int((np.asarray(g) != np.asarray(e)).sum())
               for name, g, e in zip(("score", "parent", "target", "peak_score"), gpu, exp[:4])}
        check = {"calls": int(calls.ncalls), "anchors": int(calls.nanchors), "mismatches": bad,
                 "bit_exact": not any(bad.values()),
                 "against": "minimap2-acceleration scalar chain_dp" if ref is not None else "C restatement"}
        if any(bad.values()):
            raise SystemExit(f"chain parity FAILED over the bench set: {check}")

    def sub(idx):
        idx = np.sort(idx)
        lens = calls.offsets[idx + 1] - calls.offsets[idx]
        offs = np.zeros(len(idx) + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        sel = np.concatenate([np.arange(calls.offsets[c], calls.offsets[c + 1]) for c in idx])
        return gen.ChainCalls(offs, calls.x[sel], calls.y[sel], calls.avg_qspan[idx], calls.params4[idx])

    def run(c):
        t0 = time.perf_counter()
        if ref is not None:
            oracle_lib.ref_chain_run(ref, c, threads)
        else:
            oracle_lib.chain_oracle(c, threads)
        return time.perf_counter() - t0

    cal = sub(order[:64])
    rate = cal.nanchors / max(run(cal), 1e-6)
    cum = np.cumsum((calls.offsets[order + 1] - calls.offsets[order]))
    m = int(min(calls.ncalls, max(64, np.searchsorted(cum, rate * sample_seconds))))
    s_ = sub(order[:m])
    t1 = run(s_)  # the whole set can be shorter than the sample budget: repeat it
    reps = max(1, int(sample_seconds / max(t1, 1e-6)))
    t = t1 + sum(run(s_) for _ in range(reps - 1))
    t /= reps
    return {"value": s_.nanchors / t / 1e6, "unit": "Manchors/s", "cores": threads,
            "kind": "reference" if ref is not None else "port",
            "sample": f"{m} of {calls.ncalls} calls ({s_.nanchors} anchors, random) of the same set, "
                      f"{'minimap2-acceleration scalar chain_dp' if ref is not None else 'C restatement'}, "
                      f"OpenMP {threads} threads, {reps} pass(es) of {t:.2f} s",
            "parity_check": check}


def cpu_baseline_bsw(pairs, params, sample_seconds: float, gpu=None):
    """bwa v1 ksw_extend2 compiled from the reference tree (oracle/_ref/libref_bwa.so) -- the function
    the benchmark's scalarBandedSWA (bandedSWA.cpp:130-251) restates; the benchmark's own SSE
    getScores16 needs Palisade and is not buildable here -- on a bounded random sample of the same
    pairs, one pair stream per thread (ctypes releases the GIL). Falls back to the C restatement.
    gpu = out6 [n, 6] of the GPU pass over `pairs`: the sample's outputs are compared bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from concurrent.futures import ThreadPoolExecutor
    threads = max(1, min(16, _cores()))
    ref = oracle_lib.ref_bsw()
    rng = np.random.default_rng(654)

    def run(sub):
        parts = [sub.subset(np.arange(k, sub.n, threads)) for k in range(threads)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            if ref is not None:
                outs = list(ex.map(lambda q: oracle_lib.ref_bsw_run(ref, q, params), parts))
            else:
                outs = list(ex.map(lambda q: oracle_lib.bsw_oracle(q, params, 1)[0], parts))
        t = time.perf_counter() - t0
        out6 = np.zeros((sub.n, 6), np.int32)
        for k in range(threads):
            out6[k::threads] = outs[k]
        return t, out6

    cal = pairs.subset(rng.choice(pairs.n, 4000 * threads, replace=False))
    rate = cal.n / max(run(cal)[0], 1e-6)
    m = int(min(pairs.n, max(cal.n, rate * sample_seconds)))
    idx = np.sort(rng.choice(pairs.n, m, replace=False))
    sub = pairs.subset(idx)
    cells = oracle_lib.bsw_oracle(sub, params, threads)[2]
    t, exp = run(sub)
    check = None
    if gpu is not None:
        bad = int((np.asarray(gpu)[idx] != exp).any(axis=1).sum())
        check = {"pairs": int(m), "of": int(pairs.n), "mismatching_pairs": bad, "bit_exact": bad == 0,
                 "fields": "score, qle, tle, gtle, gscore, max_off",
                 "against": "bwa ksw_extend2" if ref is not None else "C restatement"}
        if bad:
            raise SystemExit(f"bsw parity FAILED on the CPU-baseline sample: {check}")
    return {"value": cells / t / 1e9, "unit": "GCUPS", "cores": threads,
            "kind": "reference" if ref is not None else "port", "pairs_per_s": m / t,
            "sample": f"{m} of {pairs.n} pairs (random) of the same set, "
                      f"{'bwa ksw_extend2 (tools/bwa/ksw.c)' if ref is not None else 'C restatement'}, "
                      f"{threads} threads, {t:.1f} s",
            "parity_check": check}


def set_seed(args, base: int, rank: int) -> int:
    """Strong scaling: one set for the whole job (every rank the same seed, then its shard); weak:
    every rank its own full-size set."""
    return base if args.scaling == "strong" else base + rank


def timed_steps(D, steps: int, step, after=None):
    """Barrier + device sync on both sides of exactly `steps` calls of step() (each returns its kernel
    ms, or enqueues its work and returns None, the kernel ms then coming from after() once the last
    step has finished); returns (max-over-ranks wall seconds, mean kernel ms of this rank)."""
    D.barrier()
    device_sync()
    t0 = time.perf_counter()
    ks = [step() for _ in range(steps)]
    device_sync()
    D.barrier()
    wall = D.max(time.perf_counter() - t0)
    if after is not None:
        return wall, float(after())
    return wall, float(np.mean(ks)) if ks else 0.0


def shard_note(args, what: str, lo: int, hi: int, total: int, world: int) -> str:
    if args.scaling == "strong":
        return f"{what} {lo}..{hi} of {total} (rank 0 shard of {world})" if world > 1 else f"all {total} {what}"
    return f"{total} {what} per rank (own seed)"


def proxy_on(args, world: int) -> bool:
    """The single-GPU proxy of the N-GPU strong-scaling run: on one GPU (world 1), time each shard
    rank r of an N-rank run would get (N in --shard-of), with the same shard.py cut that run takes."""
    return world == 1 and args.scaling == "strong" and bool(args.shard_ns)


def proxy_warm(args, one) -> int:
    """Warm-up of one shard of the proxy: one() runs a step to completion, at least 1 + --warmup times
    and for at least --proxy-warm-ms. A 1/8 shard's step is a few ms, so --warmup steps alone end
    while the GPU is still raising its clocks (phmm 1/8 shard: 4.95 -> 4.2 ms per step over its first
    ~50 ms, profiles/r06y_phmm_shard_ramp.txt) and the proxy timed that ramp, not the shard; an N-GPU
    run's ranks run their shards back to back. Returns the warm-up steps run."""
    t0, k = time.perf_counter(), 0
    while k < 1 + args.warmup or (time.perf_counter() - t0) * 1e3 < args.proxy_warm_ms:
        one()
        k += 1
    return k


def shard_proxy(args, full_ms: float, full_value: float, unit: str, time_rank):
    """time_rank(r, n) -> (ms per step, per-GPU value) for rank r's shard of an n-rank job, for every
    n in --shard-of (default 2, 4, 8: the metric's 1/2/4/8-GPU points). Per n: each shard's per-GPU
    throughput, the lowest one against the full-set rate and (all ranks timed) the projected n-GPU
    strong-scaling speedup = full-set step / slowest shard step. The top-level fields are the largest
    n's; `by_n` carries every n."""
    by_n = {}
    for n in args.shard_ns:
        ranks = range(n) if (args.shard_rank < 0 or n != args.shard_of) else [args.shard_rank]
        per = []
        for r in ranks:
            ms, value = time_rank(r, n)
            per.append({"rank": r, "ms_per_step": round(ms, 4), "value": round(value, 3)})
        low = min(p["value"] for p in per)
        one = {"of": n, "ranks": per, "per_gpu_min": low,
               "ratio_min_vs_full": low / full_value if full_value else None}
        if len(per) == n:
            worst = max(p["ms_per_step"] for p in per)
            one["projected_speedup"] = full_ms / worst
            one["projected_efficiency"] = full_ms / worst / n
        by_n[n] = one
    top = by_n[args.shard_of]
    out = {"of": args.shard_of, "unit": unit + " per GPU", "ranks": top["ranks"], "per_gpu_min": top["per_gpu_min"],
           "ratio_min_vs_full": top["ratio_min_vs_full"],
           "note": f"1 GPU, world size 1: each rank's strong-scaling shard of the same set (shard.py) timed "
                   f"alone, {args.steps} steps after >= {1 + args.warmup} warm-up steps and >= "
                   f"{args.proxy_warm_ms:g} ms of them; ratio = per-GPU rate on the "
                   f"shard / full-set rate (>= 0.94 needed for 7.5x at 8)",
           "by_n": {str(n): {k: v for k, v in o.items() if k != "ranks"} | {"worst_ms": max(p["ms_per_step"] for p in o["ranks"])}
                    for n, o in by_n.items()}}
    for k in ("projected_speedup", "projected_efficiency"):
        if k in top:
            out[k] = top[k]
    return out


def rank_check(args, D, rank, world, what: str, local: int, units: int, full_pass):
    """world > 1, strong scaling: every rank's shard outputs against a 1-rank pass of the whole set.
    Each rank sends one (digest, units) pair (shard.digest: the units hashed with their global keys);
    rank 0 then runs the whole set by itself on its GPU (full_pass(world) -> (digest of everything,
    [digest of rank r's range for r in 0..world-1], units)) and compares: the gathered digests sum to the
    1-rank pass's and each rank's equals the 1-rank pass's over the same range. A mismatch fails the run
    on rank 0. The other ranks go on to the next leg's barrier meanwhile. Returns the check (rank 0)."""
    if world == 1 or args.scaling != "strong" or args.no_rank_check:
        return None
    from genomicsbench_palisade_amd import shard
    import torch.distributed as dist
    got = [None] * world
    dist.all_gather_object(got, (int(local), int(units)))
    if rank != 0:
        return None
    log(f"{what}: 1-rank pass of the whole set on rank 0 (gathered-output check)")
    t0 = time.perf_counter()
    full, per, nfull = full_pass(world)
    gathered = shard.digest_add(*[g[0] for g in got])
    match = [int(g[0]) == int(p) for g, p in zip(got, per)]
    out = {"world": world, "units": int(sum(g[1] for g in got)), "units_1rank": int(nfull),
           "bit_exact": bool(gathered == full and all(match) and sum(g[1] for g in got) == nfull),
           "per_rank_match": match, "digest": f"{full:016x}", "check_s": round(time.perf_counter() - t0, 2),
           "against": "a 1-rank pass of the whole set on rank 0's GPU; units hashed with their global keys "
                      "(shard.digest), gathered one digest per rank"}
    if not out["bit_exact"]:
        raise SystemExit(f"{what}: gathered {world}-rank outputs differ from the 1-rank pass: {out}")
    return out


def e2e_time(fn, reps: int = 2) -> float:
    """Mean wall seconds of fn() over `reps` calls after one warm call (host arrays in, host arrays out)."""
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def phmm_dropin_e2e(args, D, ta, cells, rank, world):
    """The reference's entry point itself, end to end: computelikelihoodsboth (the GKL C++ symbol of
    lib/libgkl_pairhmm_c.so, IntelPairHmmCSource.cpp:61-85) over the rank's testcases as host arrays --
    pack, H2D, f32 + f64 kernels, D2H, log10 -- and, on one GPU, bin/phmm (PairHMMUnitTest.cpp's CLI)
    parsing a large-shaped .in file of the same job."""
    lib = ctypes.CDLL(os.path.join(ROOT, "genomicsbench_palisade_amd", "lib", "libgkl_pairhmm_c.so"))
    both = getattr(lib, "_Z22computelikelihoodsbothP8testcasePdi")
    both.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    # initPairHMM prints a banner on stdout like the reference's (IntelPairHmmCSource.cpp:34); the
    # bench's stdout carries only its JSON line, so the banner goes to stderr
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        getattr(lib, "_Z11initPairHMMv")()
        ctypes.CDLL(None).fflush(None)
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    out = np.zeros(max(ta.n, 1))
    D.barrier()
    t = D.max(e2e_time(lambda: both(ctypes.addressof(ta.arr), out.ctypes.data, ta.n)))
    res = {"computelikelihoodsboth": {"value": D.sum(float(cells)) / t / 1e9, "unit": "GCUPS", "seconds": t,
                                      "note": "one call over the rank's whole job: host testcase[] in, double[] out "
                                              "(pack + H2D + kernels + D2H + log10)"}}
    return res


def phmm_dropin_per_batch(args, D, batches, rank, world, kernel_gcups, job_results=None):
    """computelikelihoodsboth called once per batch, as the reference's driver does
    (PairHMMUnitTest.cpp:549-593: one call per read_batch, batch_size = R x H <= MAX_BATCH_SIZE); the
    rank takes a contiguous range of whole batches balanced by cells. On one GPU the calls' results are
    checked bit for bit against the device job's results of the same testcases (job_results: the same
    kernels, so a difference is a host-side packing error)."""
    from genomicsbench_palisade_amd import shard
    from genomicsbench_palisade_amd._tc import TestcaseArray
    lib = ctypes.CDLL(os.path.join(ROOT, "genomicsbench_palisade_amd", "lib", "libgkl_pairhmm_c.so"))
    both = getattr(lib, "_Z22computelikelihoodsbothP8testcasePdi")
    both.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lo, hi = shard.rank_range([b.cells() for b in batches], rank, world)
    arrs = [TestcaseArray.from_batch(b) for b in batches[lo:hi]]  # testcase[] built outside the clock
    outs = [np.zeros(max(a.n, 1)) for a in arrs]
    cells = float(sum(a.cells() for a in arrs))

    def once():
        for a, o in zip(arrs, outs):
            both(ctypes.addressof(a.arr), o.ctypes.data, a.n)
    D.barrier()
    t = D.max(e2e_time(once))
    value = D.sum(cells) / t / 1e9
    check = None
    if job_results is not None and lo == 0 and hi == len(batches):
        got = np.concatenate([o[:a.n] for a, o in zip(arrs, outs)])
        bad = int((got.view(np.uint64) != np.asarray(job_results).view(np.uint64)).sum())
        check = {"testcases": int(len(got)), "mismatches": bad, "bit_exact": bad == 0,
                 "against": "the device job's results (themselves checked against the reference GKL)"}
        if bad:
            raise SystemExit(f"phmm per-batch drop-in parity FAILED: {check}")
    return {"value": value, "unit": "GCUPS", "seconds": t, "calls": hi - lo, "parity_check": check,
            "vs_kernel_rate": value / kernel_gcups if kernel_gcups else None,
            "note": f"computelikelihoodsboth once per batch ({hi - lo} calls of R x H testcases, batches {lo}..{hi}), "
                    f"as PairHMMUnitTest.cpp:549-593; testcase[] prepared outside the clock"}


def phmm_cli_e2e(batches, cells):
    """bin/phmm -f <large-shaped .in> -t 1 (whole job, one GPU): wall time incl. parsing and its own
    'Kernel runtime' line (pack + H2D + compute + D2H, no parsing)."""
    import subprocess
    import tempfile
    from genomicsbench_palisade_amd import gen
    exe = os.path.join(ROOT, "genomicsbench_palisade_amd", "bin", "phmm")
    with tempfile.TemporaryDirectory() as td:
        f = os.path.join(td, "large.in")
        gen.write_phmm_file(f, batches)
        t0 = time.perf_counter()
        r = subprocess.run([exe, "-f", f, "-t", "1"], capture_output=True, text=True, timeout=600)
        wall = time.perf_counter() - t0
    if r.returncode != 0:
        return {"error": r.stderr[-500:]}
    rt = [float(ln.split(":")[1].split()[0]) for ln in r.stdout.splitlines() if "Kernel runtime" in ln]
    kr = rt[0] if rt else float("nan")
    return {"value": cells / kr / 1e9 if kr > 0 else None, "unit": "GCUPS", "kernel_runtime_s": kr, "wall_s": wall,
            "wall_gcups": cells / wall / 1e9,
            "note": "bin/phmm on the job written as a .in file: 'Kernel runtime' (the reference's timed region, "
                    "PairHMMUnitTest.cpp:549-593: testcase construction, pack, H2D, kernels, D2H) and "
                    "process wall time (file parsing + runtime start-up included)"}


def bench_chain(args, D, rank, world, kind="large"):
    from genomicsbench_palisade_amd import chain, gen, shard
    log(f"chain {kind}: generating calls")
    full = gen.chain_dataset(kind, seed=set_seed(args, 5, rank))
    if args.scaling == "strong":
        calls, (lo, hi) = shard.shard_calls(full, rank, world)
    else:
        calls, (lo, hi) = full, (0, full.ncalls)
    b = chain.ChainBatch(calls)
    b.run()
    visited = b.results()[4]
    for _ in range(args.warmup):
        b.run()
        b.sync()

    def step():
        b.run()
        b.sync()
        return b.timing()
    elapsed, ms = timed_steps(D, args.steps, step)
    anchors_all = D.sum(float(calls.nanchors))
    visited_all = D.sum(float(visited))
    manch = anchors_all * args.steps / elapsed / 1e6
    ach = CHAIN_OPS_PER_PAIR * visited / (ms * 1e-3)
    out = {
        "value": round(manch, 3), "unit": "Manchors/s", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": f"chain {kind}: {full.ncalls} calls, {full.nanchors} anchors in the set (lognormal n, "
                               f"median 1500, max 87271), max_dist 5000, bw 500, n_segs 1; "
                               + shard_note(args, "calls", lo, hi, full.ncalls, world),
                   "anchors_all_ranks": int(anchors_all), "visited_pairs_all_ranks": int(visited_all),
                   "gpairs_per_s": visited_all * args.steps / elapsed / 1e9},
        "roofline": {"bound": "valu", "kernel": "chain_dp pipeline: chain_rows (dominant) + verify_lanes + pointer "
                                                  "jumping, timed as one step by the batch's events",
                     "achieved": ach / 1e12, "peak": PEAK_CHAIN_OPS / 1e12,
                     "unit": "T int32/fp64 op/s", "frac": ach / PEAK_CHAIN_OPS, "ops_per_visited_pair": CHAIN_OPS_PER_PAIR},
        "kernels_ms": {"chain_dp (all kernels of a step)": ms},
    }
    # the speculative segments' bookkeeping (chain_split.hip): a failed guess costs a sequential
    # fix-up and a re-mark of its call, so a nonzero count is worth seeing beside the time
    nsplit, rounds, fixups = b.split_stats()
    out["split_stats"] = {"split_calls": nsplit, "verify_rounds": rounds, "fixup_blocks": fixups}
    if fixups:
        log(f"chain {kind}: WARNING {fixups} speculative-segment fix-ups in the last step (window cap / warm-up "
            f"too short for these calls)")
    if world > 1:
        a0 = int(full.offsets[lo])
        r4 = b.results()[:4]
        keys = a0 + np.arange(len(r4[0]), dtype=np.int64)

        def full_pass(w):
            fb = chain.ChainBatch(full)
            fb.run()
            f4 = fb.results()[:4]
            fb.close()
            fk = np.arange(len(f4[0]), dtype=np.int64)
            per = []
            for r in range(w):
                c0, c1 = shard.call_range(full, r, w)
                s = slice(int(full.offsets[c0]), int(full.offsets[c1]))
                per.append(shard.digest(fk[s], *[x[s] for x in f4]))
            return shard.digest(fk, *f4), per, len(fk)
        out["rank_check"] = rank_check(args, D, rank, world, f"chain {kind}", shard.digest(keys, *r4), len(keys),
                                       full_pass)
    if proxy_on(args, world):
        log(f"chain {kind}: shard proxies of {args.shard_ns}")

        def t_rank(r, n):
            sub, _ = shard.shard_calls(full, r, n)
            sb = chain.ChainBatch(sub)
            proxy_warm(args, lambda: (sb.run(), sb.sync()))

            def st():
                sb.run()
                sb.sync()
                return 0.0
            el, _ = timed_steps(D, args.steps, st)
            sb.close()
            return el / args.steps * 1e3, sub.nanchors * args.steps / el / 1e6
        out["shard_proxy"] = shard_proxy(args, elapsed / args.steps * 1e3, manch, "Manchors/s", t_rank)
    if kind == "large":
        out["roofline"]["traffic"] = pmc_traffic("chain_rows")
        out["roofline"]["traffic_detail"] = pmc_traffic_detail("chain_rows")
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            log("chain: CPU baseline (+ reference run over every call, bit-exact check)")
            cpu = cpu_baseline_chain(calls, args.cpu_seconds, gpu=b.results()[:4])
        out["cpu_baseline"] = cpu
        out["backtrack"] = bench_chain_backtrack(args, D, rank, world, b, calls)
        if not args.no_e2e:
            log("chain: drop-in end to end")
            from genomicsbench_palisade_amd import check, lib
            L = lib()
            outs = [np.zeros(max(calls.nanchors, 1), np.int32) for _ in range(4)]
            t = D.max(e2e_time(lambda: check(L.gb_chain(
                ctypes.c_int64(calls.ncalls), calls.offsets.ctypes.data_as(ctypes.c_void_p),
                calls.avg_qspan.ctypes.data_as(ctypes.c_void_p), calls.params4.ctypes.data_as(ctypes.c_void_p),
                calls.x.ctypes.data_as(ctypes.c_void_p), calls.y.ctypes.data_as(ctypes.c_void_p),
                *[o.ctypes.data_as(ctypes.c_void_p) for o in outs]), "gb_chain")))
            out["dropin_e2e"] = {"gb_chain": {
                "value": anchors_all / t / 1e6, "unit": "Manchors/s", "seconds": t,
                "note": "host_chain_kernel's C ABI over the rank's calls in CSR: H2D + chain_dp + D2H of "
                        "score/parent/target/peak (the C++ drop-in adds the std::vector copies)"}}
            log("chain: host_chain_kernel over std::vector (the reference's call)")
            out["dropin_e2e"]["host_chain_kernel"] = chain_vector_e2e(D, calls, b, manch)
    b.close()
    return out


def dropin_bench_lib():
    """tests/_build/libdropin_bench.so: the C++ drop-ins called the way the reference drivers call them
    (tests/cpp/dropin_bench.cpp); None when not built."""
    path = os.path.join(ROOT, "tests", "_build", "libdropin_bench.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.bench_host_chain_kernel.argtypes = [i64, vp, vp, vp, vp, vp, ctypes.c_int, vp, vp, vp, vp]
    lib.bench_host_chain_kernel.restype = ctypes.c_double
    lib.bench_bsw_batches.argtypes = [vp, vp, i64, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]
    lib.bench_bsw_batches.restype = ctypes.c_double
    return lib


def chain_vector_e2e(D, calls, b, kernel_manch):
    """host_chain_kernel(std::vector<call_t>&, std::vector<return_t>&, int) of libgb_chain_dropin.so, one
    call over the rank's calls, timed around the call only as the reference's main.cpp:80-91 does; the
    outputs are compared with the device batch's (bit for bit)."""
    lib = dropin_bench_lib()
    if lib is None:
        return None
    outs = [np.zeros(max(calls.nanchors, 1), np.int32) for _ in range(4)]
    ts = []
    for _ in range(3):
        ts.append(lib.bench_host_chain_kernel(calls.ncalls, calls.offsets.ctypes.data, calls.avg_qspan.ctypes.data,
                                              calls.params4.ctypes.data, calls.x.ctypes.data, calls.y.ctypes.data,
                                              16, *[o.ctypes.data for o in outs]))
    t = D.max(float(np.mean(ts[1:])))
    exp = b.results()[:4]
    bad = sum(int((o[:calls.nanchors] != e).sum()) for o, e in zip(outs, exp))
    if bad:
        raise SystemExit(f"host_chain_kernel drop-in parity FAILED: {bad} mismatching outputs")
    value = D.sum(float(calls.nanchors)) / t / 1e6
    return {"value": value, "unit": "Manchors/s", "seconds": t, "vs_kernel_rate": value / kernel_manch,
            "parity_check": {"anchors": int(calls.nanchors), "bit_exact": True,
                             "against": "the device batch's score/parent/target/peak"},
            "note": "std::vector<call_t> in, std::vector<return_t> out (flatten, H2D, chain_dp, D2H, unflatten); "
                    "the vectors are built outside the clock, as the reference's read_call loop is"}


CHAIN_BT_MIN_CNT, CHAIN_BT_MIN_SC = 3, 40  # minimap2 defaults (-n 3, -m 40)
# algorithmic bytes per anchor of the backtrack: f, p, v read (12 B) + x, y of a chained anchor read
# and written (32 B)
CHAIN_BT_BYTES_PER_ANCHOR = 44


def bench_chain_backtrack(args, D, rank, world, b, calls):
    """Chain backtrack on the chain_dp outputs of the same batch: a step = one
    backtrack pass over every call (the DP outputs stay resident on the device)."""
    b.backtrack(CHAIN_BT_MIN_CNT, CHAIN_BT_MIN_SC)
    b.sync()
    nch, _, nan, _, _, tc, ta = b.chains()

    def step():
        b.backtrack(CHAIN_BT_MIN_CNT, CHAIN_BT_MIN_SC)
        b.sync()
        return b.backtrack_timing()
    elapsed, ms = timed_steps(D, args.steps, step)
    manch = D.sum(float(calls.nanchors)) * args.steps / elapsed / 1e6
    ach = CHAIN_BT_BYTES_PER_ANCHOR * calls.nanchors / (ms * 1e-3)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("chain backtrack: CPU baseline")
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        f, p, _, v, _ = b.results()
        threads = min(16, _cores())
        t1 = time.perf_counter()
        reps = 0
        while True:
            oracle_lib.chain_bt_oracle(calls, f, p, v, CHAIN_BT_MIN_CNT, CHAIN_BT_MIN_SC, threads)
            reps += 1
            if time.perf_counter() - t1 > min(args.cpu_seconds, 5.0):
                break
        dt = (time.perf_counter() - t1) / reps
        cpu = {"value": calls.nanchors / dt / 1e6, "unit": "Manchors/s", "cores": threads, "kind": "port",
               "sample": f"all {calls.ncalls} calls ({calls.nanchors} anchors) of the same set, C restatement of "
                         f"the testbed backtrack (oracle/chain_oracle.c, pinned to mm_chain_dp), {reps} pass(es), "
                         f"OpenMP {threads} threads"}
    return {
        "value": round(manch, 3), "unit": "Manchors/s", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": f"minimap2 chain backtrack (min_cnt {CHAIN_BT_MIN_CNT}, min_sc {CHAIN_BT_MIN_SC}) of "
                               f"the chain_dp outputs of the same calls", "chains": int(tc),
                   "chained_anchors": int(ta)},
        "roofline": {"bound": "hbm", "kernel": "chain backtrack pipeline (k_first sweep dominant)",
                     "achieved": ach / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": ach / PEAK_HBM,
                     "traffic": None, "bytes_per_anchor": CHAIN_BT_BYTES_PER_ANCHOR},
        "kernels_ms": {"backtrack (all kernels of a step)": ms},
        "cpu_baseline": cpu,
    }


def bench_bsw(args, D, rank, world, kind="large"):
    from genomicsbench_palisade_amd import bsw, gen, shard
    log(f"bsw {kind}: generating pairs")
    npairs = args.bsw_pairs if kind == "large" else gen.BSW_SMALL_PAIRS
    full = gen.bsw_dataset(npairs, seed=set_seed(args, 11, rank), threads=min(16, _cores()))
    if args.scaling == "strong":
        pairs, (lo, hi) = shard.shard_pairs(full, rank, world)
    else:
        pairs, (lo, hi) = full, (0, full.n)
    params = bsw.default_params()
    b = bsw.BswBatch(pairs, params)
    b.run()
    out6, _, cells = b.results(want_cells=False)
    for _ in range(args.warmup):
        b.run()
        b.sync()

    def step():
        b.run()
        b.sync()
        return b.timing()
    elapsed, ms = timed_steps(D, args.steps, step)
    cells_all = D.sum(float(cells))
    pairs_all = D.sum(float(pairs.n))
    gcups = cells_all * args.steps / elapsed / 1e9
    ach = BSW_OPS_PER_CELL * cells / (ms * 1e-3)
    out = {
        "value": round(gcups, 3), "unit": "GCUPS", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": f"bsw {kind}: {full.n} pairs in the set, query U[10,150], target = mutated query + "
                               f"U[0,100], h0 0 (20%) or U[10,70], w 100, zdrop 100; "
                               + shard_note(args, "pairs", lo, hi, full.n, world),
                   "cells_all_ranks": int(cells_all), "mpairs_per_s": pairs_all * args.steps / elapsed / 1e6},
        "roofline": {"bound": "valu", "kernel": "bsw_lane_kernel<NCH> (+ bsw_extend_kernel for long queries)",
                     "achieved": ach / 1e12, "peak": PEAK_INT_OPS / 1e12, "unit": "T int op/s",
                     "frac": ach / PEAK_INT_OPS, "ops_per_cell": BSW_OPS_PER_CELL},
        "kernels_ms": {"bsw (all launches of a step)": ms},
    }
    if world > 1:
        keys = lo + np.arange(pairs.n, dtype=np.int64)
        o6 = out6[:pairs.n]

        def full_pass(w):
            fb = bsw.BswBatch(full, params)
            fb.run()
            f6 = fb.results(want_cells=False)[0][:full.n]
            fb.close()
            fk = np.arange(full.n, dtype=np.int64)
            per = []
            for r in range(w):
                p0, p1 = shard.pair_range(full, r, w)
                per.append(shard.digest(fk[p0:p1], *f6[p0:p1].T))
            return shard.digest(fk, *f6.T), per, full.n
        out["rank_check"] = rank_check(args, D, rank, world, f"bsw {kind}", shard.digest(keys, *o6.T), pairs.n,
                                       full_pass)
    if proxy_on(args, world):
        log(f"bsw {kind}: shard proxies of {args.shard_ns}")

        def t_rank(r, n):
            sub, _ = shard.shard_pairs(full, r, n)
            sb = bsw.BswBatch(sub, params)
            proxy_warm(args, lambda: (sb.run(), sb.sync()))
            c = sb.results(want_cells=False)[2]

            def st():
                sb.run()
                sb.sync()
                return 0.0
            el, _ = timed_steps(D, args.steps, st)
            sb.close()
            return el / args.steps * 1e3, c * args.steps / el / 1e9
        out["shard_proxy"] = shard_proxy(args, elapsed / args.steps * 1e3, gcups, "GCUPS", t_rank)
    if kind == "large":
        out["roofline"]["traffic"] = pmc_traffic("bsw_lane_kernel")
        out["roofline"]["traffic_detail"] = pmc_traffic_detail("bsw_lane_kernel")
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            log("bsw: CPU baseline (+ bit-exact check of the sample)")
            cpu = cpu_baseline_bsw(pairs, params, args.cpu_seconds, gpu=out6)
        out["cpu_baseline"] = cpu
        if not args.no_e2e:
            log("bsw: drop-in end to end")
            b.close()
            sp = bsw.seqpairs(pairs)
            L = bsw._decl()
            t = D.max(e2e_time(lambda: bsw.check(L.gb_bsw_get_scores16(
                ctypes.byref(params), bsw._buf(sp), pairs.n, bsw._buf(pairs.tgt), len(pairs.tgt), bsw._buf(pairs.qry),
                len(pairs.qry)), "gb_bsw_get_scores16")))
            out["dropin_e2e"] = {"gb_bsw_get_scores16": {
                "value": cells_all / t / 1e9, "unit": "GCUPS", "seconds": t,
                "note": "BandedPairWiseSW::getScores16's C ABI over the rank's SeqPair[] and sequence buffers: "
                        "H2D + kernels + D2H into the SeqPair array"}}
            lib = dropin_bench_lib()
            if lib is not None:
                log("bsw: getScores16 per 512-pair batch from 16 threads (the reference's loop)")
                got = np.zeros((max(pairs.n, 1), 6), np.int32)
                par7, mat = params.as_array(), params.mat_array()  # kept alive across the calls
                ts = []
                for _ in range(2):
                    ts.append(lib.bench_bsw_batches(par7.ctypes.data, mat.ctypes.data,
                                                    pairs.n, sp.ctypes.data, pairs.tgt.ctypes.data,
                                                    pairs.qry.ctypes.data, 512, 16, got.ctypes.data))
                t = D.max(float(min(ts)))
                bad = int((got[:pairs.n] != out6[:pairs.n]).any(axis=1).sum())
                if bad:
                    raise SystemExit(f"getScores16 per-batch drop-in parity FAILED: {bad} pairs")
                v = cells_all / t / 1e9
                out["dropin_e2e"]["getScores16_per_batch"] = {
                    "value": v, "unit": "GCUPS", "seconds": t, "vs_kernel_rate": v / gcups,
                    "parity_check": {"pairs": int(pairs.n), "bit_exact": True, "against": "the device batch's out6"},
                    "note": "BandedPairWiseSW::getScores16 on 512-pair batches taken dynamically by 16 host "
                            "threads, one object each, as main_banded.cpp:896-924 (each batch's idr/idq index "
                            "its own buffers, as loadPairs lays them out)"}
    b.close()
    return out


def bench_phmm(args, D, rank, world, kind="large"):
    import genomicsbench_palisade_amd as gb  # noqa: F401
    from genomicsbench_palisade_amd import gen, phmm, shard
    from genomicsbench_palisade_amd._tc import TestcaseArray

    phmm.init_pairhmm()
    nb = args.batches if kind == "large" else args.small_batches
    log(f"phmm {kind}: generating + packing the job")
    batches = gen.phmm_dataset(kind, nb, seed=set_seed(args, 1, rank))
    full = TestcaseArray.from_batches(batches)
    if args.scaling == "strong":
        ta, tidx = shard.shard_testcases(full, rank, world)
    else:
        ta, tidx = full, np.arange(full.n)
    job = phmm.DeviceBatch(ta)
    ntc, cells, _ = job.stats()
    # one checked pass first (its results give the f64 share), then the warm-up steps run straight into
    # the timed ones so the GPU does not sit idle between them
    job.run()
    res, rf, rd, used, _ = job.results()
    rl = ta.np_arr["rslen"][:ta.n].astype(np.int64)
    hl = ta.np_arr["haplen"][:ta.n].astype(np.int64)
    cells_f64 = int((rl * hl)[used.astype(bool)].sum())
    for _ in range(args.warmup):
        job.run()

    k64 = []

    # the steps are enqueued back to back on the job's stream (no host round trip between them);
    # kernel times come from the last step's events
    def after():
        job.sync()
        a, b, _ = job.timing()
        k64.append(b)
        return a
    elapsed, ms32 = timed_steps(D, args.steps, job.run, after)
    ms64 = float(np.mean(k64)) if k64 else 0.0
    cells_all = D.sum(float(cells))
    gcups = cells_all * args.steps / elapsed / 1e9
    # the f32 pass's early exit drops testcases proven to fall back before their last rows: its
    # roofline counts the cells it computed (the step's GCUPS counts every cell of the job, as the
    # reference's does)
    dropped, skipped = job.exit_stats()
    cells32 = cells - skipped
    r32 = {"bound": "valu", "kernel": "phmm_forward<float> (with the f32 early exit)",
           "achieved": PHMM_FLOP_PER_CELL * cells32 / (ms32 * 1e-3) / 1e12, "peak": PEAK_F32_OPS / 1e12,
           "unit": "TFLOP/s (non-FMA FP ops)", "cells": cells32,
           "early_exit": {"testcases_dropped": dropped, "cells_skipped": skipped,
                          "cells_skipped_frac": skipped / max(cells, 1)}}
    r32["frac"] = r32["achieved"] / r32["peak"]
    r64 = {"bound": "valu", "kernel": "phmm_forward<double> (f64 fallback, its testcases only)",
           "achieved": PHMM_FLOP_PER_CELL * cells_f64 / max(ms64 * 1e-3, 1e-12) / 1e12, "peak": PEAK_F64_OPS / 1e12,
           "unit": "TFLOP/s (non-FMA FP64 ops)", "cells": cells_f64}
    r64["frac"] = r64["achieved"] / r64["peak"]
    out = {
        "value": gcups, "unit": "GCUPS", "elapsed": elapsed, "ntc": full.n, "cells": full.cells(), "cells_all_ranks": cells_all,
        "f64_frac": float(used.mean()) if ta.n else 0.0,
        "shard": (f"{len(tidx)} of {full.n} testcases: the rank-{rank} 1/{world} piece of every batch (stratified)"
                  if args.scaling == "strong" and world > 1 else shard_note(args, "testcases", 0, full.n, full.n, world)),
        "roofline": r32, "roofline_f64": r64,
        "kernels_ms": {"phmm_forward<float>": ms32, "phmm_forward<double>": ms64},
        # the job's cells over the f32 pass alone (the early exit skips part of the fallback
        # testcases' rows): what the step would be without the f64 fallback (its 36 % share of
        # testcases is a property of the synthetic generator)
        "f32_only_gcups": cells / max(ms32 * 1e-3, 1e-12) / 1e9,
    }
    if world > 1:
        def full_pass(w):
            fj = phmm.DeviceBatch(full)
            fj.run()
            fres, _, _, fused, _ = fj.results()
            fj.close()
            fk = np.arange(full.n, dtype=np.int64)
            per = []
            for r in range(w):
                ix = shard.testcase_index(full, r, w)
                per.append(shard.digest(ix, fres[ix], fused[ix]))
            return shard.digest(fk, fres[:full.n], fused[:full.n]), per, full.n
        out["rank_check"] = rank_check(args, D, rank, world, f"phmm {kind}",
                                       shard.digest(tidx, res[:ta.n], used[:ta.n]), ta.n, full_pass)
    if proxy_on(args, world):
        log(f"phmm {kind}: shard proxies of {args.shard_ns}")

        def t_rank(r, n):
            sub, _ = shard.shard_testcases(full, r, n)
            sj = phmm.DeviceBatch(sub)
            proxy_warm(args, lambda: (sj.run(), sj.sync()))
            el, _ = timed_steps(D, args.steps, sj.run, lambda: (sj.sync(), 0.0)[1])
            c = sj.stats()[1]
            sj.close()
            return el / args.steps * 1e3, c * args.steps / el / 1e9
        out["shard_proxy"] = shard_proxy(args, elapsed / args.steps * 1e3, gcups, "GCUPS", t_rank)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if kind == "large":
            log("phmm: CPU baseline (+ bit-exact check of the sample)")
            cpu = cpu_baseline_phmm(ta, args.cpu_seconds, gpu=(res, rf, rd))
        else:
            # BASELINE.json config 1: the reference on the 'small' job, single thread
            log("phmm small: single-thread CPU reference (+ bit-exact check of the sample)")
            cpu = cpu_baseline_phmm(ta, args.cpu_seconds, gpu=(res, rf, rd), threads=1)
    out["cpu_baseline"] = cpu
    if kind == "large":
        r32["traffic"] = pmc_traffic("phmm_forward<float>")
        r32["traffic_detail"] = pmc_traffic_detail("phmm_forward<float>")
        r64["traffic"] = pmc_traffic("phmm_forward<double>")
        if not args.no_e2e:
            log("phmm: drop-in end to end")
            job.close()
            e2e = phmm_dropin_e2e(args, D, ta, cells, rank, world)
            log("phmm: computelikelihoodsboth once per batch")
            e2e["computelikelihoodsboth_per_batch"] = phmm_dropin_per_batch(
                args, D, batches, rank, world, gcups, res if world == 1 else None)
            if world == 1:
                e2e["bin/phmm"] = phmm_cli_e2e(batches, full.cells())
            out["dropin_e2e"] = e2e
    job.close()
    return out


def bench_fmi(args, D, rank, world):
    from genomicsbench_palisade_amd import fmi, gen, shard

    t0 = time.perf_counter()
    log("fmi: reference + GPU index build")
    ref = gen.fmi_reference(int(args.fmi_ref_mbp * 1e6), seed=7)  # same reference on every rank
    idx = fmi.Index.build(ref)
    t_index = time.perf_counter() - t0
    log("fmi: generating reads")
    codes_all, lens_all = gen.fmi_reads(ref, args.fmi_reads, read_len=151, seed=set_seed(args, 8, rank))
    if args.scaling == "strong":
        lo, hi = shard.read_range(len(lens_all), rank, world)
    else:
        lo, hi = 0, len(lens_all)
    codes, lens = codes_all[lo:hi], lens_all[lo:hi]
    log("fmi: timed search")
    rs = fmi.Reads(idx, codes, lens)
    for _ in range(args.warmup):
        rs.search(19)
        rs.sync()
    _, total, _, phases = rs.results(batch_size=512, want_smems=False)
    calls = [0]

    def step():
        rs.search(19)
        rs.sync()
        a, _, calls[0] = rs.timing()
        return a
    elapsed, ms = timed_steps(D, args.steps, step)
    rcheck = fmi_rank_check(args, D, rank, world, "fmi large", fmi, shard, idx, rs, codes_all, lens_all, lo)
    calls = calls[0]
    reads_all = D.sum(float(len(lens)))
    mreads = reads_all * args.steps / elapsed / 1e6
    alg_bytes = calls * FMI_BYTES_PER_EXT + len(lens) * 151 + total * 40
    occ_bytes = calls * FMI_OCC_BYTES_PER_EXT + len(lens) * 151 + total * 40
    ach = alg_bytes / (ms * 1e-3)
    proxy = fmi_shard_proxy(args, D, fmi, shard, idx, codes_all, lens_all, elapsed / args.steps * 1e3, mreads) \
        if proxy_on(args, world) else None
    cpu = None
    n, _, _ = idx.info()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import fmi_util
        n_, c_, s_ = idx.info()
        oi = fmi_util.OracleIndex(adopt=(n_, c_, s_, idx.cp_occ()))  # same tables, no CPU SA build
        log("fmi: CPU baseline")
        cpu = cpu_baseline_fmi(oi, codes, lens, args.cpu_seconds, fmi, idx)
        oi.close()
    e2e = None
    if not args.no_e2e:
        log("fmi: drop-in end to end")

        def once():
            r2 = fmi.Reads(idx, codes, lens)
            r2.search(19)
            r2.results(batch_size=512)
            r2.close()
        t = D.max(e2e_time(once, reps=1))
        e2e = {"gb_fmi_search": {"value": reads_all / t / 1e6, "unit": "Mreads/s", "seconds": t,
                                 "note": "enc_qdb + lengths H2D, fmi.cpp batch pipeline, all SMEMs + per-batch "
                                         "counts D2H (index already resident)"}}
        if args.fmi_class_reads > 0:
            log("fmi: FMI_search class drop-in (fmi.cpp's per-batch loop, 16 threads)")
            e2e["FMI_search_class"] = fmi_class_e2e(args, D, fmi, ref, idx, codes, lens, mreads)
    sa = bench_sa(args, D, rank, world, fmi, idx, rs, codes, lens)
    rs.close()
    small = None if args.no_small else bench_fmi_small(args, D, rank, world, fmi, gen, shard, idx, ref)
    idx.close()
    return {
        "value": round(mreads, 3), "unit": "Mreads/s", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": f"fmi large: {args.fmi_ref_mbp:g} Mbp synthetic genome-like reference "
                               f"(BWT rows {n}), {len(lens_all)} reads x 151 bp in the set, minSeedLen 19, batch 512; "
                               + shard_note(args, "reads", lo, hi, len(lens_all), world),
                   "reads_all_ranks": int(reads_all),
                   "smems_per_read": total / max(len(lens), 1), "num_smem1_2_3": [int(x) for x in phases],
                   "backwardExt_per_read": calls / max(len(lens), 1), "index_build_s": round(t_index, 2)},
        "roofline": {"bound": "hbm", "kernel": "smem_search", "achieved": ach / 1e9, "peak": PEAK_HBM / 1e9,
                     "unit": "GB/s", "frac": ach / PEAK_HBM, "traffic": pmc_traffic("smem_search"),
                     "traffic_detail": pmc_traffic_detail("smem_search"),
                     "algorithmic_bytes": int(alg_bytes),
                     "note": "achieved uses the reference's 128 B (two 64-B CP_OCC lines) per backwardExt; "
                             "the kernel itself reads one Occ32 line (~35 B of it) per extension",
                     "occ32_bytes": int(occ_bytes), "achieved_occ32": occ_bytes / (ms * 1e-3) / 1e9},
        "kernels_ms": {"smem_search": ms},
        "cpu_baseline": cpu,
        "dropin_e2e": e2e,
        "sa_lookup": sa,
        "shard_proxy": proxy,
        "rank_check": rcheck,
        "small": small,
    }


def bench_fmi_human(args, D, rank, world):
    """fmi over a human-scale index: a 3.217 Gbp synthetic genome-like reference (+RC: n = 6.43 G BWT
    rows, the row count of the reference's human run, fmi_output:19-24; 3.2 GB of Occ32 and 6.4 GB of
    CP_OCC against the 'large' leg's 0.51 / 1.02 GB), built on the GPU, and --fmi-human-reads reads.
    Same step as the 'large' leg (the fmi.cpp batch pipeline over every read). The first reads are
    checked against the oracle run over the same CP_OCC tables, bit for bit (the run fails
    otherwise); the oracle's time on them is the CPU number (kind 'port', C restatement)."""
    from genomicsbench_palisade_amd import fmi, gen
    t0 = time.perf_counter()
    log(f"fmi human: {args.fmi_human_gbp:g} Gbp reference")
    ref = gen.fmi_reference(int(args.fmi_human_gbp * 1e9), seed=17)
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    idx = fmi.Index.build(ref)
    t_index = time.perf_counter() - t0
    n, _, _ = idx.info()
    log(f"fmi human: {n} BWT rows built in {t_index:.1f} s; generating reads")
    codes, lens = gen.fmi_reads(ref, args.fmi_human_reads, read_len=151, seed=18)
    del ref
    rs = fmi.Reads(idx, codes, lens)
    for _ in range(max(1, args.warmup)):
        rs.search(19)
        rs.sync()
    _, total, _, phases = rs.results(batch_size=512, want_smems=False)
    calls = [0]

    def step():
        rs.search(19)
        rs.sync()
        a, _, calls[0] = rs.timing()
        return a
    elapsed, ms = timed_steps(D, args.steps, step)
    rs.close()
    calls = calls[0]
    nr = len(lens)
    mreads = nr * args.steps / elapsed / 1e6
    alg_bytes = calls * FMI_BYTES_PER_EXT + nr * 151 + total * 40
    occ_bytes = calls * FMI_OCC_BYTES_PER_EXT + nr * 151 + total * 40
    check = cpu = None
    if not args.no_cpu_baseline:
        log("fmi human: oracle check + CPU time on the first reads")
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import fmi_util
        threads = max(1, min(16, _cores()))
        m = min(nr, args.fmi_human_check)
        n_, c_, s_ = idx.info()
        oi = fmi_util.OracleIndex(adopt=(n_, c_, s_, idx.cp_occ()))
        t1 = time.perf_counter()
        _, ocalls, parts = oi.run_threaded(codes[:m], lens[:m], threads, collect=True)
        t_cpu = time.perf_counter() - t1
        # reference kind: bwa v1's own mem_collect_intv (tools/bwa, compiled unmodified into oracle/_ref)
        # over a bwt_t rebuilt from the same CP_OCC tables, on the same reads
        ref_t = ref_tot = None
        blib = fmi_util.ref_bwa()
        if blib is not None:
            bwt = fmi_util.bwa_from_tables(blib, n_, s_, oi._occ)
            t1 = time.perf_counter()
            ref_tot = fmi_util.bwa_collect_threaded(blib, bwt, codes[:m], lens[:m], threads)
            ref_t = time.perf_counter() - t1
            blib.ref_bwa_free(bwt)
        oi.close()
        r2 = fmi.Reads(idx, codes[:m], lens[:m])
        r2.search(19)
        sm, tot, _, _ = r2.results(batch_size=512)
        _, _, gcalls = r2.timing()
        r2.close()
        exp = np.concatenate(parts) if parts else sm[:0]
        same = tot == len(exp) and all((sm[f] == exp[f]).all() for f in ("rid", "m", "n", "k", "l", "s"))
        check = {"reads": int(m), "smems": int(tot), "bit_exact": bool(same), "backwardExt_equal": bool(gcalls == ocalls)}
        if not (same and gcalls == ocalls):
            raise SystemExit(f"fmi human-scale parity FAILED on the first reads: {check}")
        cpu = {"value": m / t_cpu / 1e6, "unit": "Mreads/s", "cores": threads, "kind": "port",
               "sample": f"first {m} reads, C restatement of bwa-mem2 FMI_search over the same CP_OCC tables "
                         f"(batches of 512 over {threads} threads), {t_cpu:.1f} s"}
        if ref_t is not None:
            if ref_tot != tot:
                raise SystemExit(f"fmi human: bwa v1 interval count {ref_tot} != GPU SMEM count {tot}")
            cpu = {"value": m / ref_t / 1e6, "unit": "Mreads/s", "cores": threads, "kind": "reference",
                   "sample": f"first {m} reads, bwa v1 mem_collect_intv (tools/bwa bwt_smem1 + bwt_seed_strategy1, "
                             f"compiled unmodified) over a bwt_t rebuilt from the same CP_OCC tables, {threads} "
                             f"threads, {ref_t:.1f} s; {ref_tot} intervals == GPU SMEM count", "port": cpu}
    idx.close()
    return {
        "value": round(mreads, 3), "unit": "Mreads/s", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": f"fmi human-scale: {args.fmi_human_gbp:g} Gbp synthetic genome-like reference (seed 17, "
                               f"BWT rows {n}, as fmi_output:19-24's n = 6434693835), {nr} reads x 151 bp (seed 18), "
                               f"minSeedLen 19, batch 512; one GPU",
                   "smems_per_read": total / max(nr, 1), "num_smem1_2_3": [int(x) for x in phases],
                   "backwardExt_per_read": calls / max(nr, 1), "index_build_s": round(t_index, 2),
                   "reference_gen_s": round(t_gen, 2)},
        "roofline": {"bound": "hbm", "kernel": "smem_search", "achieved": alg_bytes / (ms * 1e-3) / 1e9,
                     "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": alg_bytes / (ms * 1e-3) / PEAK_HBM,
                     "traffic": pmc_traffic("smem_search", "human"),
                     "traffic_detail": pmc_traffic_detail("smem_search", "human"),
                     "algorithmic_bytes": int(alg_bytes),
                     "note": "achieved uses the reference's 128 B (two 64-B CP_OCC lines) per backwardExt; "
                             "achieved_occ32 the kernel's own ~35 B of one Occ32 block per extension",
                     "occ32_bytes": int(occ_bytes), "achieved_occ32": occ_bytes / (ms * 1e-3) / 1e9,
                     "frac_occ32": occ_bytes / (ms * 1e-3) / PEAK_HBM},
        "kernels_ms": {"smem_search (+ heavy pass, sort)": ms},
        "parity_check": check,
        "cpu_baseline": cpu,
    }


def _smem_digest(shard, sm, bc, first_batch, rid0=0):
    """rid0: the shard's first read (a shard's search numbers its reads from 0)."""
    keys = shard.smem_keys(sm["rid"], bc, first_batch)
    rid = sm["rid"].astype(np.int64) + rid0
    return shard.digest(keys, rid, *[sm[f] for f in ("m", "n", "k", "l", "s")])


def fmi_rank_check(args, D, rank, world, what, fmi, shard, idx, rs, codes_all, lens_all, lo):
    """rank_check for an fmi set: the rank's SMEMs (in fmi.cpp's per-batch order) keyed by (global
    batch, position in batch), against a 1-rank search of every read on rank 0."""
    if world == 1 or args.scaling != "strong" or args.no_rank_check:
        return None
    sm, tot, bc, _ = rs.results(batch_size=shard.FMI_BATCH)
    local = _smem_digest(shard, sm, bc, lo // shard.FMI_BATCH, lo)
    del sm

    def full_pass(w):
        fr = fmi.Reads(idx, codes_all, lens_all)
        fr.search(19)
        fsm, ftot, fbc, _ = fr.results(batch_size=shard.FMI_BATCH)
        fr.close()
        starts = np.concatenate([[0], np.cumsum(fbc)])
        per = []
        for r in range(w):
            r0, r1 = shard.read_range(len(lens_all), r, w)
            b0, b1 = r0 // shard.FMI_BATCH, (r1 + shard.FMI_BATCH - 1) // shard.FMI_BATCH
            per.append(_smem_digest(shard, fsm[starts[b0]:starts[b1]], fbc[b0:b1], b0))
        return _smem_digest(shard, fsm, fbc, 0), per, ftot
    return rank_check(args, D, rank, world, what, local, tot, full_pass)


def fmi_shard_proxy(args, D, fmi, shard, idx, codes_all, lens_all, full_ms, full_value):
    log(f"fmi: shard proxies of {args.shard_ns}")

    def t_rank(r, n):
        lo, hi = shard.read_range(len(lens_all), r, n)
        rs = fmi.Reads(idx, codes_all[lo:hi], lens_all[lo:hi])
        proxy_warm(args, lambda: (rs.search(19), rs.sync()))

        def st():
            rs.search(19)
            rs.sync()
            return 0.0
        el, _ = timed_steps(D, args.steps, st)
        rs.close()
        return el / args.steps * 1e3, (hi - lo) * args.steps / el / 1e6
    return shard_proxy(args, full_ms, full_value, "Mreads/s", t_rank)


def fmi_class_e2e(args, D, fmi, ref, idx, codes, lens, kernel_mreads):
    """The FMI_search class drop-in (lib/libgb_fmi_dropin.so) driven by fmi.cpp:253-348's batch loop
    (tests/cpp/fmi_class_driver.cpp: per 512-read batch getSMEMsAllPosOneThread, reseeding through
    getSMEMsOnePosOneThread, bwtSeedStrategyAllPosOneThread, sortSMEMs) from 16 host threads, over the
    first --fmi-class-reads reads of the rank's shard; the driver's own clock around the batch loop.
    Its sorted per-batch SMEMs are compared with the batched search's (bit for bit)."""
    import subprocess
    import tempfile
    drv = os.path.join(ROOT, "tests", "_build", "fmi_class_driver")
    if not os.path.exists(drv):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import fmi_util
    m = min(len(lens), args.fmi_class_reads) // 512 * 512
    if m == 0:
        return None
    with tempfile.TemporaryDirectory() as td:
        prefix = os.path.join(td, "ref")
        fmi.Index.build(ref, out_path=prefix + ".bwt.2bit.64").close()
        rb, ob = os.path.join(td, "reads.bin"), os.path.join(td, "out.bin")
        with open(rb, "wb") as f:
            f.write(np.array([m, codes.shape[1]], np.int32).tobytes() + lens[:m].astype(np.int32).tobytes()
                    + np.ascontiguousarray(codes[:m]).tobytes())
        r = subprocess.run([drv, prefix, rb, "512", "19", "16", ob], capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            raise SystemExit(f"fmi class driver failed: {r.stderr[-2000:]}")
        t = float([ln for ln in r.stderr.splitlines() if ln.startswith("SMEM phase:")][0].split()[2])
        raw = np.fromfile(ob, np.uint8)
    o = 8
    nb = int(raw[:8].view(np.int64)[0])
    parts = []
    for _ in range(nb):
        c = raw[o:o + 24].view(np.int64)
        o += 24
        k = int(c.sum())
        parts.append(raw[o:o + 40 * k].view(fmi_util.SMEM_DTYPE))
        o += 40 * k
    got = np.concatenate(parts)
    r2 = fmi.Reads(idx, codes[:m], lens[:m])
    r2.search(19)
    sm, tot, _, _ = r2.results(batch_size=512)
    r2.close()
    same = len(got) == tot and all((got[f] == sm[f]).all() for f in ("rid", "m", "n", "k", "l", "s"))
    if not same:
        raise SystemExit("FMI_search class drop-in parity FAILED against the batched search")
    t = D.max(t)
    value = D.sum(float(m)) / t / 1e6
    return {"value": value, "unit": "Mreads/s", "seconds": t, "reads": int(m), "vs_kernel_rate": value / kernel_mreads,
            "parity_check": {"reads": int(m), "smems": int(tot), "bit_exact": True,
                             "against": "the batched search (gb_fmi_search) on the same reads"},
            "note": "fmi.cpp's batch loop over the FMI_search class methods, 512-read batches from 16 host threads "
                    "(tests/cpp/fmi_class_driver.cpp), timed around the loop; index loaded before the clock"}


def bench_fmi_small(args, D, rank, world, fmi, gen, shard, idx, ref):
    """fmi 'small' (1 M reads, fmi_output:19) over the same index."""
    log("fmi small: timed search")
    codes_all, lens_all = gen.fmi_reads(ref, args.fmi_small_reads, read_len=151, seed=set_seed(args, 9, rank))
    lo, hi = shard.read_range(len(lens_all), rank, world) if args.scaling == "strong" else (0, len(lens_all))
    rs = fmi.Reads(idx, codes_all[lo:hi], lens_all[lo:hi])
    for _ in range(args.warmup):
        rs.search(19)
        rs.sync()
    calls = [0]

    def step():
        rs.search(19)
        rs.sync()
        a, _, calls[0] = rs.timing()
        return a
    elapsed, ms = timed_steps(D, args.steps, step)
    _, total, _, _ = rs.results(batch_size=512, want_smems=False)
    rcheck = fmi_rank_check(args, D, rank, world, "fmi small", fmi, shard, idx, rs, codes_all, lens_all, lo)
    rs.close()
    nr = hi - lo
    alg = calls[0] * FMI_BYTES_PER_EXT + nr * 151 + total * 40
    value = D.sum(float(nr)) * args.steps / elapsed / 1e6
    proxy = fmi_shard_proxy(args, D, fmi, shard, idx, codes_all, lens_all, elapsed / args.steps * 1e3, value) \
        if proxy_on(args, world) else None
    return {"value": round(value, 3), "unit": "Mreads/s", "shard_proxy": proxy, "rank_check": rcheck,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "config": {"workload": f"fmi small: {len(lens_all)} reads x 151 bp over the large index; "
                                   + shard_note(args, "reads", lo, hi, len(lens_all), world),
                       "smems_per_read": total / max(nr, 1)},
            "roofline": {"bound": "hbm", "kernel": "smem_search", "achieved": alg / (ms * 1e-3) / 1e9,
                         "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": alg / (ms * 1e-3) / PEAK_HBM},
            "kernels_ms": {"smem_search": ms}}


def bench_sa(args, D, rank, world, fmi, idx, rs, codes, lens):
    """SA coordinates of every SMEM of the last search (get_sa_entries_prefetch, max_occ 500, i.e.
    bwamem.cpp:737 over every read). A step = row expansion + all LF walks."""
    log("fmi: SA lookup")
    for _ in range(max(1, args.warmup)):
        rs.sa_run(fmi.MAX_OCC, fmi.SA_PREFETCH)
        rs.sync()
    st = [0, 0]

    def step():
        rs.sa_run(fmi.MAX_OCC, fmi.SA_PREFETCH)
        rs.sync()
        a, st[0], st[1] = rs.sa_timing()
        return a
    elapsed, ms = timed_steps(D, args.steps, step)
    steps, ncoords = st
    mcoords = D.sum(float(ncoords)) * args.steps / elapsed / 1e6
    # per coordinate: its row (8 B read), one sampled-SA entry (8 B), the coordinate (8 B written);
    # per LF step one 64-B Occ2 line
    alg_bytes = steps * SA_BYTES_PER_STEP + ncoords * SA_BYTES_PER_COORD
    ach = alg_bytes / (ms * 1e-3)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import fmi_util
        n_, c_, s_ = idx.info()
        oi = fmi_util.OracleIndex(adopt=(n_, c_, s_, idx.cp_occ(), idx.sampled_sa()))
        log("fmi: SA CPU baseline")
        cpu = cpu_baseline_sa(oi, codes, lens, args.cpu_seconds)
        oi.close()
    return {
        "value": round(mcoords, 3), "unit": "Mcoords/s", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": "SA coordinates of every SMEM of the fmi shard (get_sa_entries_prefetch, "
                               "max_occ 500, sampled SA every 8 rows)",
                   "coords_per_step": int(ncoords), "lf_steps_per_coord": steps / max(ncoords, 1)},
        "roofline": {"bound": "hbm", "kernel": "sa_walk", "achieved": ach / 1e9, "peak": PEAK_HBM / 1e9,
                     "unit": "GB/s", "frac": ach / PEAK_HBM, "traffic": pmc_traffic("sa_walk"),
                     "traffic_detail": pmc_traffic_detail("sa_walk"),
                     "algorithmic_bytes": int(alg_bytes)},
        "kernels_ms": {"sa_expand+sa_walk": ms},
        "cpu_baseline": cpu,
    }


def cpu_baseline_sa(oi, codes, lens, sample_seconds: float):
    """The C restatement of get_sa_entries_prefetch (oracle/fmi_oracle.c, kind 'port') over the SMEMs of
    the first reads of the same shard (found by the oracle's own search), threads over SMEM ranges."""
    threads = max(1, min(16, _cores()))
    m = min(len(lens), 20000)
    sm, _, _ = oi.run(codes[:m], lens[:m], batch_size=512)
    t0 = time.perf_counter()
    tot, _ = oi.sa_entries_threaded(sm, threads)
    t = time.perf_counter() - t0
    reps = 1
    if t < sample_seconds / 4 and t > 0:
        reps = max(1, int(sample_seconds / 2 / t))
        t0 = time.perf_counter()
        for _ in range(reps):
            oi.sa_entries_threaded(sm, threads)
        t = time.perf_counter() - t0
    return {"value": tot * reps / t / 1e6, "unit": "Mcoords/s", "cores": threads, "kind": "port",
            "sample": f"SA coordinates of the {len(sm)} SMEMs of the first {m} reads of the same shard "
                      f"(max_occ 500), {reps} pass(es) over {threads} threads, {t:.1f} s"}


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def child_envs(n: int, port: int, base=None):
    """The environments of the N ranks `bench.py --gpus N` starts when no launcher set WORLD_SIZE: one
    process per GPU, ranks 0..N-1 (LOCAL_RANK = RANK: one node), rendezvous on 127.0.0.1:port."""
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out.append(e)
    return out


def launch(n: int, argv, dry_run: bool = False, cmd=None, poll_s: float = 0.5) -> int:
    """`bench.py --gpus N` with WORLD_SIZE unset: start N fresh rank processes of this script (the
    same arguments, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, as torch.distributed.run would) and
    wait for them. This parent never imports torch or the package, so it never touches the GPU (the
    box forbids exec'ing after GPU initialisation; the ranks are children, not execs). Rank 0's stdout
    (the one JSON line) is this process's stdout; the other ranks' stdout goes to stderr. When a rank
    fails, the others are terminated and the first failing status is returned."""
    import subprocess
    port = _free_port()
    cmd = list(cmd) if cmd is not None else [sys.executable, "-u", os.path.abspath(__file__)] + list(argv)
    envs = child_envs(n, port)
    keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
    if dry_run:
        for e in envs:
            print(json.dumps({"cmd": cmd, "env": {k: e[k] for k in keys}}), flush=True)
        return 0
    log(f"launching {n} ranks on 127.0.0.1:{port}: {' '.join(cmd)}")
    sys.stdout.flush()
    procs = [subprocess.Popen(cmd, env=e, stdout=None if r == 0 else sys.stderr, start_new_session=False)
             for r, e in enumerate(envs)]
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad and status == 0:
                status = bad[0]
                log(f"a rank exited with status {status}; terminating the others")
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
            if all(c is not None for c in codes):
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        raise
    finally:
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    return status if status >= 0 else 128 - status


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (= ranks) of the run; without a launcher's WORLD_SIZE, bench.py starts the N rank "
                         "processes itself (one per GPU)")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="print the N rank processes' command and environment that --gpus N would start, then exit")
    ap.add_argument("--no-rank-check", action="store_true",
                    help="world > 1: skip the gathered-output check against a 1-rank pass on rank 0")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: one set sharded over the ranks (default); weak: a full set per rank")
    ap.add_argument("--batches", type=int, default=64, help="'large' phmm batches in the job")
    ap.add_argument("--small-batches", type=int, default=256, help="'small' phmm batches in the job")
    ap.add_argument("--fmi-reads", type=int, default=10_000_000, help="fmi 'large' reads in the set")
    ap.add_argument("--fmi-small-reads", type=int, default=1_000_000, help="fmi 'small' reads in the set")
    ap.add_argument("--fmi-ref-mbp", type=float, default=512.0)
    ap.add_argument("--fmi-human-gbp", type=float, default=3.217,
                    help="fmi human-scale leg: reference length in Gbp (one GPU only; 0 = off)")
    ap.add_argument("--fmi-human-reads", type=int, default=4_000_000)
    ap.add_argument("--fmi-human-check", type=int, default=20_000, help="human-scale reads checked vs the oracle")
    ap.add_argument("--fmi-class-reads", type=int, default=2_000_000,
                    help="reads of the FMI_search class drop-in leg (0 = off)")
    ap.add_argument("--bsw-pairs", type=int, default=10_606_460, help="bsw pairs in the 'large' set")
    ap.add_argument("--only", default=None, help="comma list of legs: phmm,fmi,chain,bsw,fmi_human (default all)")
    ap.add_argument("--no-small", action="store_true", help="skip the 'small'-set legs")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the drop-in end-to-end (host arrays) timings")
    ap.add_argument("--shard-of", default="2,4,8",
                    help="single-GPU proxy (world size 1, strong scaling): also time the shards an N-GPU run "
                         "would give its ranks, for each N of the comma list ('' or 0 = off)")
    ap.add_argument("--shard-rank", type=int, default=-1, help="proxy only this rank's shard (-1 = every rank)")
    ap.add_argument("--proxy-warm-ms", type=float, default=150.0,
                    help="proxy: each shard's warm-up runs at least this long (and at least 1 + --warmup steps)")
    ap.add_argument("--detail-out", default="gpurun_out/bench_detail.json",
                    help="where the full record goes (shard proxies, drop-ins, traffic detail, parity checks); "
                         "stdout carries only the compact headline line ('' = no file)")
    args = ap.parse_args()
    args.shard_ns = sorted({int(x) for x in str(args.shard_of).split(",") if x.strip() and int(x) > 1})
    args.shard_of = max(args.shard_ns) if args.shard_ns else 0
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            print(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} (from the launcher) does not match "
                  f"--gpus {args.gpus}", file=sys.stderr)
            raise SystemExit(2)
        if args.launch_dry_run:
            raise SystemExit("--launch-dry-run is for the self-launching form (WORLD_SIZE unset)")
    elif args.gpus > 1 or args.launch_dry_run:
        raise SystemExit(launch(args.gpus, sys.argv[1:], dry_run=args.launch_dry_run))

    # stdout carries exactly one line, the headline: everything else this process prints -- library
    # banners, torch.distributed's gloo connection messages under a launcher -- goes to stderr
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)
    world, rank, local = dist_env()
    D = Dist(world)
    import genomicsbench_palisade_amd as gb
    # one rank per GPU; more ranks than GPUs (a rehearsal of the multi-rank path on a smaller box)
    # share them round-robin. torch.cuda.device_count() does not initialise the GPU.
    import torch
    ndev = max(1, torch.cuda.device_count())
    gb.set_device(local % ndev)

    legs = set((args.only or "phmm,fmi,chain,bsw,fmi_human").split(","))
    ph = bench_phmm(args, D, rank, world) if "phmm" in legs else None
    fm = bench_fmi(args, D, rank, world) if "fmi" in legs else None
    ch = bench_chain(args, D, rank, world) if "chain" in legs else None
    bw = bench_bsw(args, D, rank, world) if "bsw" in legs else None
    small = None
    if not args.no_small:
        small = {}
        if "phmm" in legs:
            small["phmm"] = bench_phmm(args, D, rank, world, kind="small")
        if fm is not None:
            small["fmi"] = fm.pop("small")
        if "chain" in legs:
            small["chain"] = bench_chain(args, D, rank, world, kind="small")
        if "bsw" in legs:
            small["bsw"] = bench_bsw(args, D, rank, world, kind="small")
    elif fm is not None:
        fm.pop("small", None)
    if "fmi_human" in legs and world == 1 and args.fmi_human_gbp > 0:
        hu = bench_fmi_human(args, D, rank, world)
        fm = fm if fm is not None else {}
        fm["human"] = hu

    if rank == 0:
        seeds = "seed" if args.scaling == "strong" else "seed + rank"
        line = {
            "metric": "GCUPS (phmm) + Mreads/s (fmi) on 'large' set at 1/2/4/8 MI355X",
            "value": round(ph["value"], 3) if ph else None,
            "unit": "GCUPS (phmm)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ph["elapsed"] / args.steps * 1e3, 4) if ph else None,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32+f64 (phmm), int64 (fmi), int32/f64 (chain), int32 (bsw)",
            "data": f"synthetic, 'large'-shaped ({seeds}: phmm 1, fmi genome 7 + reads 8, chain 5, bsw 11)",
            "config": {"workload": ("phmm large: %d batches, %d testcases, %.3f G cells per step (whole job); "
                                    "%s; %.1f%% of rank 0's testcases on the f64 fallback" % (
                                        args.batches, ph["ntc"], ph["cells"] / 1e9, ph["shard"], 100 * ph["f64_frac"]))
                       if ph else None,
                       "parallelism": f"shard{world} ({args.scaling} scaling, no data-path collective)"},
            "roofline": ph["roofline"] if ph else None,
            "roofline_f64": ph["roofline_f64"] if ph else None,
            "kernels_ms": ph["kernels_ms"] if ph else None,
            "shard_proxy": ph.get("shard_proxy") if ph else None,
            "rank_check": ph.get("rank_check") if ph else None,
            "f32_only_gcups": ph.get("f32_only_gcups") if ph else None,
            "cpu_baseline": ph["cpu_baseline"] if ph else None,
            "dropin_e2e": ph.get("dropin_e2e") if ph else None,
            "fmi": fm,
            "chain": ch,
            "bsw": bw,
            "small": small,
            "cpu_host": cpu_host() if not args.no_cpu_baseline else None,
        }
        add_per_core(line)
        detail = args.detail_out
        if detail:
            d = detail if os.path.isabs(detail) else os.path.join(ROOT, detail)
            os.makedirs(os.path.dirname(d), exist_ok=True)
            with open(d, "w") as f:
                json.dump(line, f)
            log(f"full bench record: {detail} ({len(json.dumps(line))} bytes)")
        sys.stdout.flush()
        os.write(out_fd, (json.dumps(headline(line, detail)) + "\n").encode())
    D.close()


if __name__ == "__main__":
    main()
