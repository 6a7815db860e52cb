"""phmm co-residency probe: does a second PairHMM job on another stream add throughput to the first?
The 'large' job is packed twice (two device batches, two streams). K steps on one batch back to back,
then K steps on each batch enqueued alternately (the two streams' f32 and f64 kernels then overlap on
the CUs). If the two-stream run takes ~2x the one-stream run, the SIMDs' issue slots are already
full and overlapping the f64 fallback with the f32 pass (or any other co-scheduling) cannot shorten
the step. Prints ms per job for both and the ratio."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import gen, phmm, set_device  # noqa: E402
from genomicsbench_palisade_amd._tc import TestcaseArray  # noqa: E402

set_device(0)
phmm.init_pairhmm()
ta = TestcaseArray.from_batches(gen.phmm_dataset("large", int(os.environ.get("PHMM_BATCHES", "64")), seed=1))
a, b = phmm.DeviceBatch(ta), phmm.DeviceBatch(ta)
K = int(os.environ.get("PHMM_STEPS", "10"))
for x in (a, b):
    x.run()
    x.sync()


def one():
    t0 = time.perf_counter()
    for _ in range(K):
        a.run()
    a.sync()
    return (time.perf_counter() - t0) / K * 1e3


def two():
    t0 = time.perf_counter()
    for _ in range(K):
        a.run()
        b.run()
    a.sync()
    b.sync()
    return (time.perf_counter() - t0) / (2 * K) * 1e3


t1 = min(one() for _ in range(3))
t2 = min(two() for _ in range(3))
f32, f64, tot = a.timing()
print(f"one stream: {t1:.2f} ms per job (f32 {f32:.2f} + f64 {f64:.2f} ms); two streams: {t2:.2f} ms per job; "
      f"ratio {t2 / t1:.3f} (1.0 = no gain from co-residency)", flush=True)
a.close()
b.close()
