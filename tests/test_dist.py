"""Multi-process (N>1) path on CPU: world_size-2 gloo process groups exercise bench.py's Dist
(barrier, max-over-ranks time, sum-over-ranks work), its timed_steps bracket and set_seed, and the
strong-scaling shard -> compute -> concatenate flow bench.py uses for all four legs (shard.py:
testcases as a cell-balanced piece of every batch, whole 512-read batches, calls by anchors, pairs by cell estimate), with the C
oracles standing in for the per-GPU kernels (CPU-only container): the two ranks' outputs
concatenate to the 1-rank output exactly."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from genomicsbench_palisade_amd import shard

WORKER = r'''
import json, os, sys, types
sys.path.insert(0, os.environ["GB_ROOT"]); sys.path.insert(0, os.path.join(os.environ["GB_ROOT"], "tests"))
import numpy as np
import bench, oracle_lib, fmi_util
from genomicsbench_palisade_amd import gen, shard, bsw
from genomicsbench_palisade_amd._tc import TestcaseArray
world, rank, local = bench.dist_env()
D = bench.Dist(world)
args = types.SimpleNamespace(scaling="strong")
D.barrier()
mx = D.max(float(rank + 1))
sm = D.sum(float(10 * (rank + 1)))
el, ms = bench.timed_steps(D, 3, lambda: 1.5)
# each leg exactly as bench.py takes it: the same seeded set on every rank, then this rank's shard
calls = gen.chain_dataset("small", num_calls=60, seed=bench.set_seed(args, 3, rank), median_n=200, max_n=3000)
sub, (lo, hi) = shard.shard_calls(calls, rank, world)
sc = oracle_lib.chain_oracle(sub, 1)[0] if sub.ncalls else np.zeros(0, np.int32)
pairs = gen.bsw_pairs(500, seed=bench.set_seed(args, 4, rank))
psub, _ = shard.shard_pairs(pairs, rank, world)
out = oracle_lib.bsw_oracle(psub, bsw.default_params(), 1)[0]
ta = TestcaseArray.from_batches(gen.phmm_dataset("small", 3, seed=bench.set_seed(args, 1, rank)))
tsub, tidx = shard.shard_testcases(ta, rank, world)
pr = np.zeros(tsub.n); rf = np.zeros(tsub.n, np.float32); rd = np.zeros(tsub.n)
import ctypes
if tsub.n:
    oracle_lib.oracle().phmm_oracle_batch(ctypes.addressof(tsub.arr), tsub.n, pr.ctypes.data, rf.ctypes.data, rd.ctypes.data, None, 1)
ref = gen.fmi_reference(60_000, seed=5)
codes, lens = gen.fmi_reads(ref, int(os.environ.get("GB_NREADS", "1300")), seed=bench.set_seed(args, 8, rank))
rlo, rhi = shard.read_range(len(lens), rank, world)
oi = fmi_util.OracleIndex(ref)
fs, fbc, _ = oi.run(codes[rlo:rhi], lens[rlo:rhi], batch_size=512)
fs["rid"] += rlo
# bench.rank_check: one digest per rank gathered, rank 0 compares with a 1-rank pass (here the oracle
# over the whole set stands in for the GPU pass); a corrupted shard must fail the check
a0 = int(calls.offsets[lo])
r4 = oracle_lib.chain_oracle(sub, 1)[:4] if sub.ncalls else [np.zeros(0, np.int32)] * 4
keys = a0 + np.arange(sub.nanchors, dtype=np.int64)
def full_pass(w):
    f4 = [x[:calls.nanchors] for x in oracle_lib.chain_oracle(calls, 1)[:4]]
    fk = np.arange(calls.nanchors, dtype=np.int64)
    per = []
    for r in range(w):
        c0, c1 = shard.call_range(calls, r, w)
        s = slice(int(calls.offsets[c0]), int(calls.offsets[c1]))
        per.append(shard.digest(fk[s], *[x[s] for x in f4]))
    return shard.digest(fk, *f4), per, len(fk)
rargs = types.SimpleNamespace(scaling="strong", no_rank_check=False)
rc = bench.rank_check(rargs, D, rank, world, "chain test", shard.digest(keys, *[x[:sub.nanchors] for x in r4]),
                      sub.nanchors, full_pass)
bad = [x[:sub.nanchors].copy() for x in r4]
if rank == 1 and sub.nanchors:
    bad[0][sub.nanchors // 2] += 1
try:
    bench.rank_check(rargs, D, rank, world, "chain test", shard.digest(keys, *bad), sub.nanchors, full_pass)
    caught = False
except SystemExit:
    caught = True
import torch.distributed as dist
got = [None] * world
dist.all_gather_object(got, {"chain": sc.tolist(), "bsw": out.tolist(), "phmm": pr.tolist(), "tidx": [int(x) for x in tidx],
                             "fmi": [list(map(int, t)) for t in zip(fs["rid"], fs["m"], fs["n"], fs["k"], fs["l"], fs["s"])],
                             "fmi_bc": fbc.tolist(), "rrange": [rlo, rhi],
                             "max": mx, "sum": sm, "range": [lo, hi], "timed_steps_ms": ms,
                             "rank_check": rc, "caught": caught})
if rank == 0:
    json.dump(got, open(os.environ["GB_OUT"], "w"))
D.close()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_balanced_ranges_properties():
    rng = np.random.default_rng(0)
    w = rng.integers(1, 100, 1000)
    for parts in (1, 2, 3, 8):
        r = shard.balanced_ranges(w, parts)
        assert r[0][0] == 0 and r[-1][1] == len(w)
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        sums = [w[lo:hi].sum() for lo, hi in r]
        assert max(sums) - w.sum() / parts <= w.max()
    assert shard.balanced_ranges([], 2) == [(0, 0), (0, 0)]
    r = shard.balanced_ranges([5], 3)
    assert r[0][0] == 0 and r[-1][1] == 1 and sum(hi - lo for lo, hi in r) == 1


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_shards_concatenate_to_the_full_result(tmp_path, world):
    """world 2 and 4 (the driver's 8-GPU scaling run also takes N = 2 / 4 / 8): every rank's shard
    of every leg, gathered, equals the 1-rank result, and rank_check catches a corrupted shard."""
    import oracle_lib
    from genomicsbench_palisade_amd import bsw, gen
    out = tmp_path / "gathered.json"
    wf = tmp_path / "worker.py"
    wf.write_text(WORKER)
    port = _free_port()
    procs = []
    nreads = 1300 if world == 2 else 2100  # whole 512-read batches for every rank
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GB_ROOT=ROOT, GB_OUT=str(out), OMP_NUM_THREADS="1", GB_NREADS=str(nreads))
        procs.append(subprocess.Popen([sys.executable, str(wf)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    for p in procs:
        try:
            o, e = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            p.kill()
            pytest.fail("gloo worker timed out")
        assert p.returncode == 0, e[-3000:]
    got = json.load(open(out))
    cat = lambda key: sum((g[key] for g in got), [])  # noqa: E731
    assert [g["max"] for g in got] == [float(world)] * world
    assert [g["sum"] for g in got] == [10.0 * world * (world + 1) / 2] * world
    calls = gen.chain_dataset("small", num_calls=60, seed=3, median_n=200, max_n=3000)
    full = oracle_lib.chain_oracle(calls, 1)[0]
    rngs = [g["range"] for g in got]
    assert rngs[0][0] == 0 and rngs[-1][1] == calls.ncalls and all(a[1] == b[0] for a, b in zip(rngs, rngs[1:]))
    assert (np.array(cat("chain"), np.int32) == full).all()
    pairs = gen.bsw_pairs(500, seed=4)
    fb = oracle_lib.bsw_oracle(pairs, bsw.default_params(), 1)[0]
    assert (np.array(cat("bsw"), np.int32).reshape(-1, 6) == fb).all()
    assert [g["timed_steps_ms"] for g in got] == [1.5] * world
    # bench.rank_check: rank 0 holds the check; the corrupted rank-1 shard was caught on rank 0 only
    rc = got[0]["rank_check"]
    assert rc["bit_exact"] and rc["per_rank_match"] == [True] * world and rc["units"] == calls.nanchors
    assert all(g["rank_check"] is None for g in got[1:])
    assert [g["caught"] for g in got] == [True] + [False] * (world - 1)
    # phmm: testcase shards balanced by cells concatenate to the 1-rank results
    import ctypes
    from genomicsbench_palisade_amd._tc import TestcaseArray
    ta = TestcaseArray.from_batches(gen.phmm_dataset("small", 3, seed=1))
    pr, rf, rd = np.zeros(ta.n), np.zeros(ta.n, np.float32), np.zeros(ta.n)
    oracle_lib.oracle().phmm_oracle_batch(ctypes.addressof(ta.arr), ta.n, pr.ctypes.data, rf.ctypes.data,
                                          rd.ctypes.data, None, 1)
    # phmm: the ranks' stratified pieces (1/2 of every batch) partition the job and gather back
    idx = np.array(cat("tidx"))
    assert (np.sort(idx) == np.arange(ta.n)).all()
    gathered = np.zeros(ta.n)
    gathered[idx] = np.array(cat("phmm"))
    assert (gathered.view(np.uint64) == pr.view(np.uint64)).all()
    # fmi: whole 512-read batches per rank; SMEM lists and per-batch counts concatenate
    import fmi_util
    ref = gen.fmi_reference(60_000, seed=5)
    codes, lens = gen.fmi_reads(ref, nreads, seed=8)
    fs, fbc, _ = fmi_util.OracleIndex(ref).run(codes, lens, batch_size=512)
    rr = [g["rrange"] for g in got]
    assert rr[0][0] == 0 and rr[-1][1] == nreads and all(a[1] == b[0] and a[1] % 512 == 0 for a, b in zip(rr, rr[1:]))
    if world == 2:
        assert rr == [[0, 1024], [1024, 1300]]
    exp = [list(map(int, t)) for t in zip(fs["rid"], fs["m"], fs["n"], fs["k"], fs["l"], fs["s"])]
    assert cat("fmi") == exp
    assert cat("fmi_bc") == fbc.tolist()
