"""Drop-in call-granularity probe: getScores16 per 512-pair batch from 16 threads (DROPIN_BSW_PAIRS
pairs of the 'large' set) and host_chain_kernel over std::vector (the 'large' chain set), through
tests/_build/libdropin_bench.so; prints seconds and rates. DROPIN_LEGS selects (bsw,chain)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from genomicsbench_palisade_amd import bsw, chain, gen, set_device  # noqa: E402

set_device(0)
lib = bench.dropin_bench_lib()
legs = os.environ.get("DROPIN_LEGS", "bsw,chain").split(",")
if "bsw" in legs:
    n = int(os.environ.get("DROPIN_BSW_PAIRS", "2000000"))
    p = gen.bsw_dataset(n, seed=11, threads=16)
    P = bsw.default_params()
    b = bsw.BswBatch(p, P)
    b.run()
    out6, _, cells = b.results(want_cells=False)
    b.run()
    b.sync()
    k = b.timing()
    b.close()
    sp = bsw.seqpairs(p)
    par7, mat = P.as_array(), P.mat_array()
    got = np.zeros((p.n, 6), np.int32)
    for th in (16, 8):
        t = min(lib.bench_bsw_batches(par7.ctypes.data, mat.ctypes.data, p.n, sp.ctypes.data, p.tgt.ctypes.data,
                                      p.qry.ctypes.data, 512, th, got.ctypes.data) for _ in range(2))
        ok = (got == out6[:p.n]).all()
        print(f"bsw: {p.n} pairs, kernel {cells / k / 1e6:.1f} GCUPS; getScores16 x 512 from {th} threads: "
              f"{t:.3f} s = {cells / t / 1e9:.1f} GCUPS ({cells / t / 1e9 / (cells / k / 1e6):.3f} of kernel), "
              f"exact {ok}", flush=True)
if "chain" in legs:
    calls = gen.chain_dataset("large", seed=5)
    b = chain.ChainBatch(calls)
    b.run()
    b.sync()
    t0 = time.perf_counter()
    for _ in range(5):
        b.run()
        b.sync()
    kt = (time.perf_counter() - t0) / 5
    r = bench.chain_vector_e2e(bench.Dist(1), calls, b, calls.nanchors / kt / 1e6)
    print(f"chain: kernel {calls.nanchors / kt / 1e6:.0f} Manchors/s; host_chain_kernel {r['value']:.0f} Manchors/s "
          f"({r['seconds'] * 1e3:.1f} ms, {r['vs_kernel_rate']:.3f} of kernel)", flush=True)
    b.close()
