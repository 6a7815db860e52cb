"""scripts/run-cpu.sh -- the reference's harness (scripts/run-cpu.sh:24-86) over bin/{fmi,bsw,phmm,chain}
on the reference's <INPUTS_DIR> layout, fed by scripts/make-inputs.py. The GPU test builds a scaled
synthetic 'small' layout, runs the harness, and checks each benchmark's output against the oracle."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

RUN = os.path.join(ROOT, "scripts", "run-cpu.sh")
MAKE = os.path.join(ROOT, "scripts", "make-inputs.py")


def test_usage_and_out_of_scope_benchmarks(tmp_path):
    r = subprocess.run(["bash", RUN], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stdout
    r = subprocess.run(["bash", RUN, str(tmp_path), "small", "dbg", "poa", "kmer-cnt", "pileup", "grm"],
                       capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.count("Skipping") == 5
    r = subprocess.run(["bash", RUN, str(tmp_path), "large", "nope"], capture_output=True, text=True)
    assert r.returncode == 1 and "unknown benchmark" in r.stderr


def test_make_inputs_layout_cpu_legs(tmp_path):
    """The CPU-only writers (bsw, phmm, chain) produce the file names run-cpu.sh reads."""
    r = subprocess.run([sys.executable, MAKE, str(tmp_path), "small", "--scale", "0.001", "--only", "bsw,phmm,chain"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    for p in ("bsw/small/bandedSWA_SRR7733443_100k_input.txt", "phmm/small/5m.in", "chain/small/in-1k.txt"):
        assert os.path.getsize(tmp_path / p) > 0, p


@pytest.mark.gpu
def test_run_cpu_small_layout_end_to_end(tmp_path):
    import fmi_util
    import oracle_lib
    from genomicsbench_palisade_amd import gen
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, MAKE, str(tmp_path), "small", "--scale", "0.002"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    bsw_out = tmp_path / "bsw.out"
    r = subprocess.run(["bash", RUN, str(tmp_path), "small"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, GB_BSW_OUT=str(bsw_out), GB_PHMM_PRINT="1"))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    out = r.stdout
    for b in ("fmi", "bsw", "phmm", "chain"):
        assert f"Running {b}" in out
    # fmi: totalSmems equals the oracle over the same index file and reads
    oi = fmi_util.OracleIndex(load_path=str(tmp_path / "fmi" / "broad.bwt.2bit.64"))
    codes, lens = gen.fmi_reads(gen.fmi_reference(1_024_000, seed=7), 2000, read_len=151, seed=9)
    exp, _, _ = oi.run(codes, lens, batch_size=512)
    tot = [int(ln.split("=")[1]) for ln in out.splitlines() if ln.startswith("totalSmems =")]
    assert tot == [len(exp)]
    # bsw: every pair processed, and each pair's six outputs equal the oracle's (pinned to ksw_extend2)
    assert "Total Pairs processed: 200" in out
    from genomicsbench_palisade_amd import bsw
    pairs = gen.bsw_dataset(200, seed=11)
    exp6 = oracle_lib.bsw_oracle(pairs, bsw.default_params())[0]
    got6 = np.loadtxt(bsw_out, dtype=np.int64, ndmin=2)
    assert got6.shape == (200, 6) and (got6 == exp6).all()
    # chain: one score/parent line per anchor, bit-exact against the oracle
    calls = gen.chain_dataset("small", num_calls=2, seed=5, max_n=1745)
    sc, par = oracle_lib.chain_oracle(calls, 1)[:2]
    rows = [ln for ln in open(tmp_path / "chain" / "small" / "out-1k.txt").read().splitlines()
            if ln and ln != "EOR" and "\t" in ln]
    got = np.array([[int(v) for v in ln.split("\t")] for ln in rows])
    assert (got[:, 0] == sc).all() and (got[:, 1] == par).all()
    assert "PairHMM completed" in out
    # phmm: every printed result ("%lf", PairHMMUnitTest.cpp's PRINT_OUTPUT) equals the oracle's, text
    # for text, in the file's testcase order
    from genomicsbench_palisade_amd._tc import TestcaseArray
    ta = TestcaseArray.from_batches(gen.phmm_dataset("small", 1, seed=1))
    import ctypes
    o = oracle_lib.oracle()
    res, rf, rd = np.zeros(ta.n), np.zeros(ta.n, np.float32), np.zeros(ta.n)
    o.phmm_oracle_batch(ctypes.addressof(ta.arr), ta.n, res.ctypes.data, rf.ctypes.data, rd.ctypes.data, None, 4)
    seg = out[out.index("Running phmm"):out.index("PairHMM completed")].splitlines()
    printed = [ln.strip() for ln in seg if ln.strip().lstrip("-").replace(".", "", 1).isdigit()]
    assert printed == ["%f" % v for v in res]
