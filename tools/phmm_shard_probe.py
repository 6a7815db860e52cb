"""phmm strong-scaling shard probe: the 'large' job (64 batches, seed 1) and its shard PHMM_RANK (default
0) of PHMM_OF (default 8): per step the f32 kernel, f64 fallback and whole-step times (HIP events) and
the sync'd wall time, with the stack count and the GB_PHMM_STACK_ROWS setting in use."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import genomicsbench_palisade_amd as g  # noqa: E402
if os.environ.get("PHMM_LIB"):  # another build of libgb.so, to time two builds on one box
    g.LIBGB = os.path.abspath(os.environ["PHMM_LIB"])
from genomicsbench_palisade_amd import gen, phmm, set_device, shard  # noqa: E402
from genomicsbench_palisade_amd._tc import TestcaseArray  # noqa: E402

set_device(0)
phmm.init_pairhmm()
# PHMM_KIND=small: the 'small'-shaped job
full = TestcaseArray.from_batches(gen.phmm_dataset(os.environ.get("PHMM_KIND", "large"),
                                                   int(os.environ.get("PHMM_BATCHES", "64")), seed=1))
of, r = int(os.environ.get("PHMM_OF", "8")), int(os.environ.get("PHMM_RANK", "0"))
jobs = [("full", full), (f"shard {r}/{of}", shard.shard_testcases(full, r, of)[0])]
if os.environ.get("PHMM_SHARD_ONLY"):  # e.g. under a kernel trace
    jobs = jobs[1:]
for name, ta in jobs:
    for rows in os.environ.get("PHMM_ROWS", "default").split(";"):
        # a setting: "default", a GB_PHMM_STACK_ROWS value, or env assignments "K=V,K=V"
        for k in ("GB_PHMM_STACK_ROWS", "GB_PHMM_F64_ROWS", "GB_PHMM_RPL", "GB_PHMM_W2", "GB_PHMM_PIPE", "GB_PHMM_TAIL",
                  "GB_PHMM_F64_REGROUP", "GB_PHMM_F64_PARTS", "GB_PHMM_F64_GRID",
                  "GB_PHMM_EXIT", "GB_PHMM_F64_PLAN"):
            os.environ.pop(k, None)
        if "=" in rows:
            for kv in rows.split(","):
                k, v = kv.split("=")
                os.environ[k] = v
        elif rows != "default":
            os.environ["GB_PHMM_STACK_ROWS"] = rows
        job = phmm.DeviceBatch(ta)
        t0, k = time.perf_counter(), 0
        while k < 3 or time.perf_counter() - t0 < 0.15:  # past the GPU's clock ramp (bench.py proxy_warm)
            job.run()
            job.sync()
            k += 1
        steps = 10
        t0 = time.perf_counter()
        for _ in range(steps):
            job.run()
        job.sync()
        wall = (time.perf_counter() - t0) / steps * 1e3
        a, b, c = job.timing()
        ntc, cells, nf64 = job.stats()
        job.close()
        print(f"{name:12s} {rows:24s}: {ntc} testcases, {cells / 1e9:.2f} G cells, f64 {nf64}; wall {wall:.3f} ms "
              f"({cells / wall / 1e6:.1f} GCUPS); f32 {a:.3f} ms, f64 {b:.3f} ms, step {c:.3f} ms", flush=True)
