"""phmm probe: the bench's 'large' job (16 batches, seed 1), two timed runs of the device batch."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genomicsbench_palisade_amd import gen, phmm, set_device
from genomicsbench_palisade_amd._tc import TestcaseArray
set_device(0)
phmm.init_pairhmm()
ta = TestcaseArray.from_batches(gen.phmm_dataset("large", int(os.environ.get("PHMM_BATCHES", "16")), seed=1))
job = phmm.DeviceBatch(ta)
ntc, cells, nf64 = job.stats()
for _ in range(3):
    job.run(); job.sync()
    a, b, t = job.timing()
    print(f"f32 {a:.3f} ms f64 {b:.3f} ms total {t:.3f} ms -> {cells / t / 1e6:.1f} GCUPS ({nf64} f64 testcases)", flush=True)
