"""phmm probe: f32 / f64 pass times on the bench's 'large' job for kernel variants selected by
environment variables (read when a batch runs): PROBE_VARIANTS="NAME:VAR=VAL,VAR=VAL;NAME2:...".
'large'-shaped jobs with other haplotype caps via PHMM_HAPMAX (default 473 only)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import genomicsbench_palisade_amd as g  # noqa: E402
if os.environ.get("PHMM_LIB"):  # another build of libgb.so, to time two builds on one box
    g.LIBGB = os.path.abspath(os.environ["PHMM_LIB"])
from genomicsbench_palisade_amd import gen, phmm, set_device
from genomicsbench_palisade_amd._tc import TestcaseArray
set_device(0)
phmm.init_pairhmm()


def job_for(hap_max, nb=16):
    if hap_max == 473:
        return TestcaseArray.from_batches(gen.phmm_dataset("large", nb, seed=1))
    rng = np.random.default_rng(1)
    out = []
    for _ in range(nb):
        R = max(1, int(1193 * rng.random() ** 2))
        H = max(1, int(128 * rng.random() ** 1.5))
        while R * H > 50000:
            R = max(1, R // 2)
        out.append(gen.phmm_batch(rng, R, H, read_len=(min(100, hap_max), min(250, hap_max)), hap_max=hap_max))
    return TestcaseArray.from_batches(out)


variants = []
for v in os.environ.get("PROBE_VARIANTS", "base:").split(";"):
    name, _, kv = v.partition(":")
    variants.append((name, dict(x.split("=") for x in kv.split(",") if x)))
for hm in [int(x) for x in os.environ.get("PHMM_HAPMAX", "473").split(",")]:
    ta = job_for(hm)
    job = phmm.DeviceBatch(ta)
    ntc, cells, _ = job.stats()
    for rep in range(2):
        for name, env in variants:
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            ts = []
            for _ in range(4):
                job.run(); job.sync()
                ts.append(job.timing())
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v
            a = min(x[0] for x in ts[1:]); b = min(x[1] for x in ts[1:]); t = min(x[2] for x in ts[1:])
            print(f"{os.path.basename(g.LIBGB)} hap_max {hm} {name:10s}: f32 {a:.3f} ms ({cells / a / 1e6:.0f} GCUPS f32)  f64 {b:.3f} ms  total {t:.3f} ms -> {cells / t / 1e6:.0f} GCUPS", flush=True)
    job.close()
