#!/usr/bin/env python3
"""bench.py -- GenomicsBench hot kernels on MI355X (driver contract: one JSON line on rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batches B] [--no-cpu-baseline]

Metric (BASELINE.json): "GCUPS (phmm) + Mreads/s (fmi) on 'large' set at 1/2/4/8 MI355X".
phmm (the line's `value`): a step = one PairHMM forward pass (f32 kernel + f64 fallback kernel +
log10 epilogue) over one 'large'-shaped synthetic job of B batches (gen.phmm_dataset, seed 1 + rank)
already resident in HBM; value = total cells of all ranks x K / max-over-ranks wall time, in GCUPS.
chain / bsw (the "chain" / "bsw" objects): a step = chain_dp over every call of a 'large'-shaped
set (10k calls, 25 M anchors, seed 5 + rank; Manchors/s) / the banded SW extension of every pair of
a 'large'-shaped set (10 606 460 pairs, seed 11 + rank; GCUPS over the reference's inner-loop cells).
fmi (the line's "fmi" object): a step = the whole fmi.cpp per-batch pipeline (SMEMs, reseeding,
LAST seeds, per-read sort) over every read of the rank's shard (gen.fmi_reads, seed 8 + rank) against
a 512 Mbp genome-like synthetic reference (+RC: 1.024 G BWT rows, 1.02 GB CP_OCC) built on the GPU;
value = reads of all ranks x K / max-over-ranks wall time, in Mreads/s.
Weak scaling: every rank processes its own shard of the same shape (independent shards, no
data-path collective; torch.distributed only provides the barrier and the max-time reduction).
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
SA_BYTES_PER_STEP = 64               # one 64-B Occ2 line per LF step of an SA lookup
SA_BYTES_PER_COORD = 24              # row in, sampled-SA entry, coordinate out (8 B each)
CHAIN_OPS_PER_PAIR = 25              # ~25 int32/fp64 ops per visited (i, j) pair
PEAK_CHAIN_OPS = PEAK_F64_OPS        # INT32/FP64 VALU, 39.3e12 lane-op/s
BSW_OPS_PER_CELL = 13                # ~13 int ops per scalar inner-loop iteration
PEAK_INT_OPS = PEAK_F32_OPS          # 32-bit integer VALU lane-ops/s = 78.6e12


def pmc_traffic_detail(kernel: str):
    """Per-launch HBM bytes of `kernel` from the newest committed profiles/*_pmc.json (rocprofv3
    FETCH_SIZE and WRITE_SIZE passes of this same bench configuration, tools/gpu_prof.sh +
    tools/pmc_summary.py, fetch corrected by the calibrated factor of the kernel's read class);
    None when no profile covers it. PMC cannot run inside the timed process."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), key=os.path.getmtime)
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
                    "source": os.path.relpath(f, ROOT)}
    return None


def pmc_traffic(kernel: str):
    """roofline.traffic: corrected HBM bytes per launch (number), or None."""
    d = pmc_traffic_detail(kernel)
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


def cpu_baseline_phmm(ta, sample_seconds: float):
    """Reference GKL kernels (oracle/_ref, kind 'reference') -- or the C restatement when the
    reference build is absent (kind 'port') -- on a bounded random sample of the same job."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from genomicsbench_palisade_amd._tc import TestcaseArray  # noqa: F401
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores))  # the GPU box grants 16 CPUs per GPU
    ref = oracle_lib.ref_phmm()
    rng = np.random.default_rng(123)
    order = rng.permutation(ta.n)
    kind = "reference" if ref is not None else "port"
    engine = 512 if (ref is not None and ref.ref_phmm_has_avx512()) else 256

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
    return {"value": gcups, "unit": "GCUPS", "cores": threads, "kind": kind,
            "sample": f"{m} of {ta.n} testcases ({sub.cells() / 1e9:.2f} G cells, random) of the same "
                      f"job x {reps} passes, {eng} GKL kernels, OpenMP {threads} threads, {t:.1f} s"}


def cpu_baseline_fmi(oracle_index, codes, lens, sample_seconds: float):
    """The bwa-mem2 SMEM restatement (oracle/fmi_oracle.c, kind 'port': the reference FMI_search.cpp
    is not buildable here without Palisade) over a bounded sample of the same reads."""
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores))
    cal = min(len(lens), 4000 * threads)
    t0 = time.perf_counter()
    oracle_index.run_threaded(codes[:cal], lens[:cal], threads)
    rate = cal / max(time.perf_counter() - t0, 1e-6)
    m = int(min(len(lens), max(cal, rate * sample_seconds)))
    t0 = time.perf_counter()
    oracle_index.run_threaded(codes[:m], lens[:m], threads)
    t = time.perf_counter() - t0
    return {"value": m / t / 1e6, "unit": "Mreads/s", "cores": threads, "kind": "port",
            "sample": f"first {m} of {len(lens)} reads of the same shard, C restatement of bwa-mem2 "
                      f"FMI_search (batches of 512 over {threads} threads), {t:.1f} s"}


def _cores():
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def cpu_baseline_chain(calls, sample_seconds: float):
    """The reference's scalar chain_dp (tools/minimap2-acceleration/kernel/scalar, compiled from the
    reference tree into oracle/_ref, kind 'reference'; the C restatement when absent, kind 'port')
    over a bounded random sample of the same calls, OpenMP over calls like host_chain_kernel."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from genomicsbench_palisade_amd import gen
    threads = max(1, min(16, _cores()))
    ref = oracle_lib.ref_chain()
    rng = np.random.default_rng(321)
    order = rng.permutation(calls.ncalls)

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
                      f"OpenMP {threads} threads, {reps} pass(es) of {t:.2f} s"}


def cpu_baseline_bsw(pairs, params, sample_seconds: float):
    """bwa v1 ksw_extend2 compiled from the reference tree (oracle/_ref/libref_bwa.so) -- the function
    the benchmark's scalarBandedSWA (bandedSWA.cpp:130-251) restates; the benchmark's own SSE
    getScores16 needs Palisade and is not buildable here -- on a bounded random sample of the same
    pairs, one pair stream per thread (ctypes releases the GIL). Falls back to the C restatement."""
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
                list(ex.map(lambda q: oracle_lib.ref_bsw_run(ref, q, params), parts))
            else:
                list(ex.map(lambda q: oracle_lib.bsw_oracle(q, params, 1), parts))
        return time.perf_counter() - t0

    cal = pairs.subset(rng.choice(pairs.n, 4000 * threads, replace=False))
    rate = cal.n / max(run(cal), 1e-6)
    m = int(min(pairs.n, max(cal.n, rate * sample_seconds)))
    idx = np.sort(rng.choice(pairs.n, m, replace=False))
    sub = pairs.subset(idx)
    cells = oracle_lib.bsw_oracle(sub, params, threads)[2]
    t = run(sub)
    return {"value": cells / t / 1e9, "unit": "GCUPS", "cores": threads,
            "kind": "reference" if ref is not None else "port", "pairs_per_s": m / t,
            "sample": f"{m} of {pairs.n} pairs (random) of the same set, "
                      f"{'bwa ksw_extend2 (tools/bwa/ksw.c)' if ref is not None else 'C restatement'}, "
                      f"{threads} threads, {t:.1f} s"}


def bench_chain(args, D, rank, world):
    from genomicsbench_palisade_amd import chain, gen
    log("chain: generating calls")
    calls = gen.chain_dataset("large", seed=5 + rank)
    b = chain.ChainBatch(calls)
    for _ in range(args.warmup):
        b.run()
        b.sync()
    visited = b.results()[4]
    D.barrier()
    device_sync()
    t0 = time.perf_counter()
    ks = []
    for _ in range(args.steps):
        b.run()
        b.sync()
        ks.append(b.timing())
    device_sync()
    D.barrier()
    elapsed = D.max(time.perf_counter() - t0)
    manch = D.sum(float(calls.nanchors)) * args.steps / elapsed / 1e6
    ms = float(np.mean(ks))
    ach = CHAIN_OPS_PER_PAIR * visited / (ms * 1e-3)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("chain: CPU baseline")
        cpu = cpu_baseline_chain(calls, args.cpu_seconds)
    bt = bench_chain_backtrack(args, D, rank, world, b, calls)
    b.close()
    return {
        "backtrack": bt,
        "value": round(manch, 3), "unit": "Manchors/s", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": f"chain large: {calls.ncalls} calls, {calls.nanchors} anchors/rank (lognormal "
                               f"n, median 1500, max 87271), max_dist 5000, bw 500, n_segs 1",
                   "visited_pairs": int(visited), "gpairs_per_s": visited * args.steps * D.world / elapsed / 1e9},
        "roofline": {"bound": "valu", "kernel": "chain_kernel", "achieved": ach / 1e12, "peak": PEAK_CHAIN_OPS / 1e12,
                     "unit": "T int32/fp64 op/s", "frac": ach / PEAK_CHAIN_OPS, "traffic": pmc_traffic("chain_kernel"),
                     "traffic_detail": pmc_traffic_detail("chain_kernel"),
                     "ops_per_visited_pair": CHAIN_OPS_PER_PAIR},
        "kernels_ms": {"chain_kernel": ms},
        "cpu_baseline": cpu,
    }


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
    D.barrier()
    device_sync()
    t0 = time.perf_counter()
    ks = []
    for _ in range(args.steps):
        b.backtrack(CHAIN_BT_MIN_CNT, CHAIN_BT_MIN_SC)
        b.sync()
        ks.append(b.backtrack_timing())
    device_sync()
    D.barrier()
    elapsed = D.max(time.perf_counter() - t0)
    manch = D.sum(float(calls.nanchors)) * args.steps / elapsed / 1e6
    ms = float(np.mean(ks))
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


def bench_bsw(args, D, rank, world):
    from genomicsbench_palisade_amd import bsw, gen
    log("bsw: generating pairs")
    pairs = gen.bsw_dataset(args.bsw_pairs, seed=11 + rank, threads=min(16, _cores()))
    params = bsw.default_params()
    b = bsw.BswBatch(pairs, params)
    for _ in range(args.warmup):
        b.run()
        b.sync()
    _, _, cells = b.results(want_cells=False)
    D.barrier()
    device_sync()
    t0 = time.perf_counter()
    ks = []
    for _ in range(args.steps):
        b.run()
        b.sync()
        ks.append(b.timing())
    device_sync()
    D.barrier()
    elapsed = D.max(time.perf_counter() - t0)
    gcups = D.sum(float(cells)) * args.steps / elapsed / 1e9
    ms = float(np.mean(ks))
    ach = BSW_OPS_PER_CELL * cells / (ms * 1e-3)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("bsw: CPU baseline")
        cpu = cpu_baseline_bsw(pairs, params, args.cpu_seconds)
    b.close()
    return {
        "value": round(gcups, 3), "unit": "GCUPS", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": f"bsw large: {pairs.n} pairs/rank, query U[10,150], target = mutated query + "
                               f"U[0,100], h0 0 (20%) or U[10,70], w 100, zdrop 100",
                   "cells": int(cells), "mpairs_per_s": pairs.n * D.world * args.steps / elapsed / 1e6},
        "roofline": {"bound": "valu", "kernel": "bsw_lane_kernel<NCH> (+ bsw_extend_kernel for long queries)",
                     "achieved": ach / 1e12,
                     "peak": PEAK_INT_OPS / 1e12, "unit": "T int op/s", "frac": ach / PEAK_INT_OPS,
                     "traffic": pmc_traffic("bsw_lane_kernel"),
                     "traffic_detail": pmc_traffic_detail("bsw_lane_kernel"), "ops_per_cell": BSW_OPS_PER_CELL},
        "kernels_ms": {"bsw (all launches of a step)": ms},
        "cpu_baseline": cpu,
    }


def bench_phmm(args, D, rank, world):
    import genomicsbench_palisade_amd as gb  # noqa: F401
    from genomicsbench_palisade_amd import gen, phmm
    from genomicsbench_palisade_amd._tc import TestcaseArray

    phmm.init_pairhmm()
    log("phmm: generating + packing the job")
    batches = gen.phmm_dataset("large", args.batches, seed=1 + rank)
    ta = TestcaseArray.from_batches(batches)
    job = phmm.DeviceBatch(ta)
    ntc, cells, _ = job.stats()
    for _ in range(args.warmup):
        job.run()
        job.sync()
    _, rf, _, used, _ = job.results()
    rl = ta.np_arr["rslen"][:ta.n].astype(np.int64)
    hl = ta.np_arr["haplen"][:ta.n].astype(np.int64)
    cells_f64 = int((rl * hl)[used.astype(bool)].sum())

    D.barrier()
    device_sync()
    t0 = time.perf_counter()
    k32, k64 = [], []
    for _ in range(args.steps):
        job.run()
        job.sync()
        a, b, _ = job.timing()
        k32.append(a)
        k64.append(b)
    device_sync()
    D.barrier()
    elapsed = D.max(time.perf_counter() - t0)
    total_cells = D.sum(float(cells)) * args.steps
    gcups = total_cells / elapsed / 1e9
    ms32, ms64 = float(np.mean(k32)), float(np.mean(k64))
    if ms32 >= ms64:
        kern, ach, peak = "phmm_forward<float>", PHMM_FLOP_PER_CELL * cells / (ms32 * 1e-3), PEAK_F32_OPS
    else:
        kern, ach, peak = "phmm_forward<double>", PHMM_FLOP_PER_CELL * cells_f64 / (ms64 * 1e-3), PEAK_F64_OPS
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("phmm: CPU baseline")
        cpu = cpu_baseline_phmm(ta, args.cpu_seconds)
    job.close()
    return {
        "value": gcups, "elapsed": elapsed, "ntc": ntc, "cells": cells, "f64_frac": float(used.mean()),
        "roofline": {"bound": "valu", "kernel": kern, "achieved": ach / 1e12, "peak": peak / 1e12,
                     "unit": "TFLOP/s (non-FMA FP ops)", "frac": ach / peak, "traffic": pmc_traffic(kern),
                     "traffic_detail": pmc_traffic_detail(kern)},
        "kernels_ms": {"phmm_forward<float>": ms32, "phmm_forward<double>": ms64},
        "cpu_baseline": cpu,
    }


def bench_fmi(args, D, rank, world):
    from genomicsbench_palisade_amd import fmi, gen

    t0 = time.perf_counter()
    log("fmi: reference + GPU index build")
    ref = gen.fmi_reference(int(args.fmi_ref_mbp * 1e6), seed=7)  # same reference on every rank
    idx = fmi.Index.build(ref)
    t_index = time.perf_counter() - t0
    log("fmi: generating reads")
    codes, lens = gen.fmi_reads(ref, args.fmi_reads, read_len=151, seed=8 + rank)
    log("fmi: timed search")
    rs = fmi.Reads(idx, codes, lens)
    for _ in range(args.warmup):
        rs.search(19)
        rs.sync()
    _, total, _, phases = rs.results(batch_size=512, want_smems=False)
    D.barrier()
    device_sync()
    t0 = time.perf_counter()
    ks, kt, calls = [], [], 0
    for _ in range(args.steps):
        rs.search(19)
        rs.sync()
        a, b, calls = rs.timing()
        ks.append(a)
        kt.append(b)
    device_sync()
    D.barrier()
    elapsed = D.max(time.perf_counter() - t0)
    mreads = D.sum(float(len(lens))) * args.steps / elapsed / 1e6
    ms = float(np.mean(ks))
    alg_bytes = calls * FMI_BYTES_PER_EXT + len(lens) * 151 + total * 40
    ach = alg_bytes / (ms * 1e-3)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import fmi_util
        n_, c_, s_ = idx.info()
        oi = fmi_util.OracleIndex(adopt=(n_, c_, s_, idx.cp_occ()))  # same tables, no CPU SA build
        log("fmi: CPU baseline")
        cpu = cpu_baseline_fmi(oi, codes, lens, args.cpu_seconds)
        oi.close()
    n, _, _ = idx.info()
    sa = bench_sa(args, D, rank, world, fmi, idx, rs, codes, lens)
    rs.close()
    idx.close()
    return {
        "value": round(mreads, 3), "unit": "Mreads/s", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": f"fmi large: {args.fmi_ref_mbp:g} Mbp synthetic genome-like reference "
                               f"(BWT rows {n}), {len(lens)} reads x 151 bp/rank, minSeedLen 19, batch 512",
                   "smems_per_read": total / len(lens), "num_smem1_2_3": [int(x) for x in phases],
                   "backwardExt_per_read": calls / len(lens), "index_build_s": round(t_index, 2)},
        "roofline": {"bound": "hbm", "kernel": "smem_search", "achieved": ach / 1e9, "peak": PEAK_HBM / 1e9,
                     "unit": "GB/s", "frac": ach / PEAK_HBM, "traffic": pmc_traffic("smem_search"),
                     "traffic_detail": pmc_traffic_detail("smem_search"),
                     "algorithmic_bytes": int(alg_bytes)},
        "kernels_ms": {"smem_search": ms, "smem_search+scan": float(np.mean(kt))},
        "cpu_baseline": cpu,
        "sa_lookup": sa,
    }


def bench_sa(args, D, rank, world, fmi, idx, rs, codes, lens):
    """SA coordinates of every SMEM of the last search (get_sa_entries_prefetch, max_occ 500, i.e.
    bwamem.cpp:737 over every read). A step = row expansion + all LF walks."""
    log("fmi: SA lookup")
    for _ in range(max(1, args.warmup)):
        rs.sa_run(fmi.MAX_OCC, fmi.SA_PREFETCH)
        rs.sync()
    D.barrier()
    device_sync()
    t0 = time.perf_counter()
    kms = []
    steps = ncoords = 0
    for _ in range(args.steps):
        rs.sa_run(fmi.MAX_OCC, fmi.SA_PREFETCH)
        rs.sync()
        a, steps, ncoords = rs.sa_timing()
        kms.append(a)
    device_sync()
    D.barrier()
    elapsed = D.max(time.perf_counter() - t0)
    mcoords = D.sum(float(ncoords)) * args.steps / elapsed / 1e6
    ms = float(np.mean(kms))
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batches", type=int, default=16, help="'large' phmm batches per job (per rank)")
    ap.add_argument("--fmi-reads", type=int, default=10_000_000, help="fmi reads per rank")
    ap.add_argument("--fmi-ref-mbp", type=float, default=512.0)
    ap.add_argument("--bsw-pairs", type=int, default=10_606_460, help="bsw pairs per rank (large set)")
    ap.add_argument("--only", default=None, help="comma list of legs: phmm,fmi,chain,bsw (default all)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world, rank, local = dist_env()
    D = Dist(world)
    import genomicsbench_palisade_amd as gb
    gb.set_device(local)

    legs = set((args.only or "phmm,fmi,chain,bsw").split(","))
    ph = bench_phmm(args, D, rank, world) if "phmm" in legs else None
    fm = bench_fmi(args, D, rank, world) if "fmi" in legs else None
    ch = bench_chain(args, D, rank, world) if "chain" in legs else None
    bw = bench_bsw(args, D, rank, world) if "bsw" in legs else None

    if rank == 0:
        line = {
            "metric": "GCUPS (phmm) + Mreads/s (fmi) on 'large' set at 1/2/4/8 MI355X",
            "value": round(ph["value"], 3) if ph else None,
            "unit": "GCUPS (phmm)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ph["elapsed"] / args.steps * 1e3, 4) if ph else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32+f64 (phmm), int64 (fmi), int32/f64 (chain), int32 (bsw)",
            "data": "synthetic ('large'-shaped PairHMM batches seed 1+rank; genome-like reference seed 7 "
                    "+ 151 bp reads seed 8+rank for fmi; minimap2-shaped anchor calls seed 5+rank for chain; "
                    "extension pairs seed 11+rank for bsw)",
            "config": {"workload": ("phmm large: %d batches/rank, %d testcases, %.3f G cells/rank/step, "
                                    "%.1f%% testcases on the f64 fallback" % (
                                        args.batches, ph["ntc"], ph["cells"] / 1e9, 100 * ph["f64_frac"]))
                       if ph else None,
                       "parallelism": f"shard{world}"},
            "roofline": ph["roofline"] if ph else None,
            "kernels_ms": ph["kernels_ms"] if ph else None,
            "cpu_baseline": ph["cpu_baseline"] if ph else None,
            "fmi": fm,
            "chain": ch,
            "bsw": bw,
        }
        print(json.dumps(line))
    D.close()


if __name__ == "__main__":
    main()
