"""fmi tail probe: per-read trace (GB_FMI_FLAGS=8) of smem_search on the bench's index and read
set -- for each read the wall clock (100 MHz) at which a lane took it and finished it, and its
backwardExt calls -- for the strong-scaling shards of FMI_TAIL_OF (default 8) and the full set.
Writes gpurun_out/fmi_tail_<tag>.npz (times relative to the first take, int32 ticks) and prints a
summary: step time, the time with >= 90 % / 50 % of reads in flight, the slowest read."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import fmi, gen, lib, set_device, shard  # noqa: E402

set_device(0)
mbp = float(os.environ.get("FMI_PROBE_MBP", "512"))
nreads = int(os.environ.get("FMI_PROBE_READS", "10000000"))
of = int(os.environ.get("FMI_TAIL_OF", "8"))
tag = os.environ.get("FMI_TAIL_TAG", "x")
ref = gen.fmi_reference(int(mbp * 1e6), seed=7)
idx = fmi.Index.build(ref)
codes, lens = gen.fmi_reads(ref, nreads, read_len=151, seed=8)
L = lib()
L.gb_fmi_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
L.gb_fmi_debug_trace_rows.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
out = {}
for name, (lo, hi) in [("shard0", shard.read_range(nreads, 0, of)), ("full", (0, nreads))]:
    rs = fmi.Reads(idx, codes[lo:hi], lens[lo:hi])
    os.environ["GB_FMI_FLAGS"] = "0"
    for _ in range(2):
        rs.search(19)
        rs.sync()
    t0 = time.perf_counter()
    rs.search(19)
    rs.sync()
    wall = time.perf_counter() - t0
    a, _, calls = rs.timing()
    os.environ["GB_FMI_FLAGS"] = "8"
    rs.search(19)
    rs.sync()
    at, _, _ = rs.timing()
    rows = ctypes.c_int64()
    L.gb_fmi_debug_trace_rows(rs.h, ctypes.byref(rows))
    tr = np.zeros(3 * rows.value, np.int64)
    L.gb_fmi_debug_trace(rs.h, tr.ctypes.data)
    tr = tr.reshape(-1, 3)  # one row per task: reads, then (split search) their LAST tasks
    rs.close()
    hv = tr[:, 2] < 0  # reads redone by smem_heavy (calls negated)
    tr[:, 2] = np.abs(tr[:, 2])
    t_lo = tr[:, 0].min()
    st, en, c = tr[:, 0] - t_lo, tr[:, 1] - t_lo, tr[:, 2]
    if hv.any():
        print(f"  {int(hv.sum())} reads handed to smem_heavy: start {st[hv].min() * 1e-5:.2f} ms, end "
              f"{en[hv].max() * 1e-5:.2f} ms, ext p50 {np.percentile(c[hv], 50):.0f} max {c[hv].max()}, "
              f"read ms max {(en[hv] - st[hv]).max() * 1e-5:.2f}; lane-kernel reads end by "
              f"{en[~hv].max() * 1e-5:.2f} ms", flush=True)
    span = en.max()
    # reads in flight over time (10 us bins)
    nb = int(span // 1000) + 1
    inflight = np.zeros(nb + 1, np.int64)
    np.add.at(inflight, (st // 1000).astype(np.int64), 1)
    np.add.at(inflight, (en // 1000).astype(np.int64), -1)
    inflight = np.cumsum(inflight)[:nb]
    peak = inflight.max()
    t90 = (inflight >= 0.9 * peak).sum() * 10e-3
    t50 = (inflight >= 0.5 * peak).sum() * 10e-3
    dur = (en - st) * 1e-5  # ms
    last_start = st.max() * 1e-5
    k = int(np.argmax(en))
    print(f"{name}: {hi - lo} reads, search {a:.2f} ms (traced {at:.2f}), {calls / (hi - lo):.1f} ext/read; "
          f"trace span {span * 1e-5:.2f} ms, peak in flight {peak}, >=90% {t90:.2f} ms, >=50% {t50:.2f} ms, "
          f"last take {last_start:.2f} ms; read ms p50 {np.percentile(dur, 50):.2f} p99 {np.percentile(dur, 99):.2f} "
          f"max {dur.max():.2f}; ext p50 {np.percentile(c, 50):.0f} p99 {np.percentile(c, 99):.0f} max {c.max()}; "
          f"slowest-ending read: start {st[k] * 1e-5:.2f} ms, {dur[k]:.2f} ms, {c[k]} ext", flush=True)
    if len(tr) > hi - lo:  # split search: the LAST tasks
        lt = slice(hi - lo, None)
        print(f"  split: LAST tasks take {st[lt].min() * 1e-5:.2f}..{st[lt].max() * 1e-5:.2f} ms, end by "
              f"{en[lt].max() * 1e-5:.2f} ms, ms p50 {np.percentile(dur[lt], 50):.2f} max {dur[lt].max():.2f}; "
              f"search tasks end by {en[:hi - lo].max() * 1e-5:.2f} ms", flush=True)
    if name == "shard0":
        out = dict(st=st.astype(np.int32), en=en.astype(np.int32), calls=c.astype(np.int32), heavy=hv)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"fmi_tail_{tag}.npz"), **out)
import resource  # noqa: E402
print(f"max RSS {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6:.1f} GB", flush=True)
