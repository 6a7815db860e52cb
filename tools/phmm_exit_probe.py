"""phmm f32 early exit (GB_PHMM_EXIT=1, the knob of profiles/r05zzi_phmm_exit.patch -- apply it to
build the exit kernel) against the default, on the 'large' job (64 batches, seed 1)
and its 1/8 shard: per setting the f32 / f64 / step times (HIP events, best of 3 rounds of 10 steps),
the testcases the exit dropped from the f32 pass, and the outputs against the first setting's --
final log10 likelihoods and raw f64 results bit for bit, raw f32 results bit for bit wherever the
first setting's passed MIN_ACCEPTED (a dropped testcase's f32 result is 0 by design).
PHMM_LIB: another build of libgb.so (time two builds on one box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import genomicsbench_palisade_amd as g  # noqa: E402
if os.environ.get("PHMM_LIB"):
    g.LIBGB = os.path.abspath(os.environ["PHMM_LIB"])
from genomicsbench_palisade_amd import gen, phmm, set_device, shard  # noqa: E402
from genomicsbench_palisade_amd._tc import TestcaseArray  # noqa: E402

set_device(0)
phmm.init_pairhmm()
full = TestcaseArray.from_batches(gen.phmm_dataset("large", 64, seed=1))
configs = os.environ.get("PHMM_CONFIGS", ";GB_PHMM_EXIT=1").split(";")
for name, ta in [("full", full), ("shard0/8", shard.shard_testcases(full, 0, 8)[0])]:
    ref = None
    for cfg in configs:
        os.environ.pop("GB_PHMM_EXIT", None)
        for kv in [c for c in cfg.split("+") if c]:
            k, v = kv.split("=")
            os.environ[k] = v
        job = phmm.DeviceBatch(ta)
        for _ in range(3):
            job.run()
        job.sync()
        best = None
        for _ in range(3):
            f32 = f64 = step = 0.0
            for _ in range(10):
                job.run()
                a, b, c = job.timing()
                f32, f64, step = f32 + a, f64 + b, step + c
            t = (f32 / 10, f64 / 10, step / 10)
            best = t if best is None or t[2] < best[2] else best
        out = job.results()
        ntc, cells, nf64 = job.stats()
        job.close()
        res, rf, rd, ud = out[0], out[1], out[2], out[3]
        note = ""
        if ref is None:
            ref = (res, rf, rd, ud)
        else:
            same_final = (res.view(np.uint64) == ref[0].view(np.uint64)).all()
            same_rd = (rd.view(np.uint64)[ref[3] != 0] == ref[2].view(np.uint64)[ref[3] != 0]).all()
            passed = ref[1] >= np.float32(1e-28)
            same_rf = (rf.view(np.uint32)[passed] == ref[1].view(np.uint32)[passed]).all()
            same_ud = (ud == ref[3]).all()
            dropped = int(((rf == 0) & (ref[1] > 0)).sum())
            note = (f" dropped {dropped} of {int((~passed).sum())} failing; final same={same_final} rd same={same_rd}"
                    f" rf(passing) same={same_rf} used_double same={same_ud}")
        print(f"{os.path.basename(g.LIBGB)} {name:9s} [{cfg or 'default':16s}] f32 {best[0]:.3f} ms f64 {best[1]:.3f} ms "
              f"step {best[2]:.3f} ms ({cells / best[2] / 1e6:.1f} GCUPS) f64 testcases {nf64}{note}", flush=True)
