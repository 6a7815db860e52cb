"""bench.py --gpus N (CPU): the self-launcher that starts N rank processes when no launcher set
WORLD_SIZE, its refusal of a WORLD_SIZE / --gpus mismatch, and the output digests the N-rank run
gathers to compare its shards with a 1-rank pass (shard.digest)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from genomicsbench_palisade_amd import shard

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(kw)
    return e


def test_launch_dry_run_prints_the_rank_environments():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "3", "--launch-dry-run"],
                       capture_output=True, text=True, timeout=120, env=_env())
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines()]
    assert len(lines) == 4
    assert [ln["env"]["RANK"] for ln in lines] == ["0", "1", "2", "3"]
    assert [ln["env"]["LOCAL_RANK"] for ln in lines] == ["0", "1", "2", "3"]
    assert {ln["env"]["WORLD_SIZE"] for ln in lines} == {"4"}
    assert {ln["env"]["MASTER_ADDR"] for ln in lines} == {"127.0.0.1"}
    assert len({ln["env"]["MASTER_PORT"] for ln in lines}) == 1
    cmd = lines[0]["cmd"]
    assert cmd[0] == sys.executable and cmd[3:] == ["--gpus", "4", "--steps", "3", "--launch-dry-run"]
    assert os.path.samefile(cmd[2], BENCH)


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8"], capture_output=True, text=True, timeout=120,
                       env=_env(WORLD_SIZE="2", RANK="0"))
    assert r.returncode == 2
    assert "does not match --gpus 8" in r.stderr


def test_launch_forwards_rank0_stdout_only_and_propagates_failure(tmp_path, capfd):
    sys.path.insert(0, ROOT)
    import bench
    child = tmp_path / "child.py"
    child.write_text(
        "import os, sys\n"
        "r = int(os.environ['RANK'])\n"
        "print('line from rank', r, os.environ['WORLD_SIZE'], os.environ['MASTER_ADDR'], flush=True)\n"
        "sys.exit(int(os.environ.get('FAIL_RANK', '-1')) == r and 3 or 0)\n")
    assert bench.launch(3, [], cmd=[sys.executable, str(child)], poll_s=0.05) == 0
    out, err = capfd.readouterr()
    assert out.splitlines() == ["line from rank 0 3 127.0.0.1"]
    assert "line from rank 1 3" in err and "line from rank 2 3" in err
    os.environ["FAIL_RANK"] = "1"
    try:
        assert bench.launch(2, [], cmd=[sys.executable, str(child)], poll_s=0.05) == 3
    finally:
        del os.environ["FAIL_RANK"]


def test_digest_is_split_invariant_and_order_sensitive():
    rng = np.random.default_rng(3)
    n = 10_000
    keys = np.arange(n, dtype=np.int64)
    a = rng.integers(-2**31, 2**31, n).astype(np.int32)
    f = rng.standard_normal(n)
    full = shard.digest(keys, a, f)
    for parts in (2, 3, 8):
        cuts = shard.balanced_ranges(rng.integers(1, 50, n), parts)
        assert shard.digest_add(*[shard.digest(keys[lo:hi], a[lo:hi], f[lo:hi]) for lo, hi in cuts]) == full
    # a unit at another place, a changed value, a flipped float bit or a missing unit all change it
    b = a.copy()
    b[[5, 6]] = b[[6, 5]]
    assert a[5] == a[6] or shard.digest(keys, b, f) != full
    b = a.copy()
    b[123] ^= 1
    assert shard.digest(keys, b, f) != full
    g = f.copy()
    g.view(np.uint64)[77] ^= np.uint64(1)
    assert shard.digest(keys, a, g) != full
    assert shard.digest(keys[1:], a[1:], f[1:]) != full
    assert shard.digest(keys[:0], a[:0]) == 0


def test_smem_keys_follow_the_batches():
    bc = np.array([3, 0, 2], np.int64)
    k = shard.smem_keys(np.zeros(5), bc, 10)
    assert [(int(x) >> 32, int(x) & 0xFFFFFFFF) for x in k] == [(10, 0), (10, 1), (10, 2), (12, 0), (12, 1)]
    # a shard's keys are the whole set's keys over the same batches
    full_bc = np.array([4, 3, 0, 2, 5], np.int64)
    fk = shard.smem_keys(np.zeros(14), full_bc, 0)
    part = shard.smem_keys(np.zeros(7), full_bc[2:], 2)
    assert (fk[7:] == part).all()


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", ["1", "2"])
def test_stdout_is_one_json_line(gpus, tmp_path):
    """The driver reads one JSON line from stdout: at N=1 and under the self-launcher at N=2 (two
    ranks sharing the GPU, gloo connection messages and library banners included) nothing else may
    reach it."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", gpus, "--only", "phmm", "--batches", "8", "--no-small",
                        "--no-e2e", "--no-cpu-baseline", "--steps", "2", "--warmup", "1", "--shard-of", "0",
                        "--detail-out", str(tmp_path / "d.json")],
                       capture_output=True, text=True, timeout=280, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, lines[:3]
    line = json.loads(lines[0])
    assert line["n_gpus"] == int(gpus) and line["value"] > 0
