"""Multi-process (N>1) path on CPU: world_size-2 gloo process groups exercise bench.py's Dist
(barrier, max-over-ranks time, sum-over-ranks work) and the shard -> compute -> concatenate flow
of shard.py, with the C oracles standing in for the per-GPU kernels (CPU-only container)."""
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
import json, os, sys
sys.path.insert(0, os.environ["GB_ROOT"]); sys.path.insert(0, os.path.join(os.environ["GB_ROOT"], "tests"))
import numpy as np
import bench, oracle_lib
from genomicsbench_palisade_amd import gen, shard, bsw
world, rank, local = bench.dist_env()
D = bench.Dist(world)
D.barrier()
mx = D.max(float(rank + 1))
sm = D.sum(float(10 * (rank + 1)))
# chain: shard calls by anchor count
calls = gen.chain_dataset("small", num_calls=60, seed=3, median_n=200, max_n=3000)
lo, hi = shard.rank_range(np.diff(calls.offsets), rank, world)
o0, o1 = calls.offsets[lo], calls.offsets[hi]
sub = gen.ChainCalls(calls.offsets[lo:hi + 1] - o0, calls.x[o0:o1], calls.y[o0:o1], calls.avg_qspan[lo:hi], calls.params4[lo:hi])
sc = oracle_lib.chain_oracle(sub, 1)[0] if sub.ncalls else np.zeros(0, np.int32)
# bsw: shard pairs by cell estimate
pairs = gen.bsw_pairs(500, seed=4)
blo, bhi = shard.rank_range(pairs.qlen.astype(np.int64) * pairs.tlen, rank, world)
out = oracle_lib.bsw_oracle(pairs.subset(np.arange(blo, bhi)), bsw.default_params(), 1)[0]
import torch.distributed as dist
got = [None] * world
dist.all_gather_object(got, {"chain": sc.tolist(), "bsw": out.tolist(), "max": mx, "sum": sm, "range": [lo, hi]})
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


def test_gloo_world2_shards_concatenate_to_the_full_result(tmp_path):
    import oracle_lib
    from genomicsbench_palisade_amd import bsw, gen
    out = tmp_path / "gathered.json"
    wf = tmp_path / "worker.py"
    wf.write_text(WORKER)
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GB_ROOT=ROOT, GB_OUT=str(out), OMP_NUM_THREADS="1")
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
    assert [g["max"] for g in got] == [2.0, 2.0] and [g["sum"] for g in got] == [30.0, 30.0]
    calls = gen.chain_dataset("small", num_calls=60, seed=3, median_n=200, max_n=3000)
    full = oracle_lib.chain_oracle(calls, 1)[0]
    assert got[0]["range"][0] == 0 and got[0]["range"][1] == got[1]["range"][0] and got[1]["range"][1] == calls.ncalls
    assert (np.array(got[0]["chain"] + got[1]["chain"], np.int32) == full).all()
    pairs = gen.bsw_pairs(500, seed=4)
    fb = oracle_lib.bsw_oracle(pairs, bsw.default_params(), 1)[0]
    assert (np.array(got[0]["bsw"] + got[1]["bsw"], np.int32).reshape(-1, 6) == fb).all()
