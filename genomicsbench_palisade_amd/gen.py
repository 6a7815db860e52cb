"""Seeded synthetic inputs shaped like the reference's 'small'/'large' datasets.

The real input-datasets tarball (README.md:26 of the reference) is not available, so every benchmark
and parity test runs on these generators. Shapes follow the comments/logs recovered in SURVEY.md:
  phmm  small: batches <=110 reads x <=37 haps, reads <=250 bp, haps <=302 bp
        large: batches <=1193 reads x <=128 haps, reads <=250 bp, haps <=473 bp
        (PairHMMUnitTest.cpp:1,9-10,30; <=50000 testcases per batch, :69,558)
"""
from __future__ import annotations

import numpy as np

BASES = np.frombuffer(b"ACGT", dtype=np.uint8)


class PhmmBatch:
    """One read_batch() worth of data (PairHMMUnitTest.cpp:118-210,461-474): R reads x H haps.

    reads[r] = (bases, q, i, d, c) as bytes, already normalized (phred-33, q>=6) like normalize()
    (PairHMMUnitTest.cpp:107-113); haps[h] = bases. Testcases are r-major: tc[r*H+h].
    """

    def __init__(self, reads, haps):
        self.reads = reads
        self.haps = haps

    @property
    def num_testcases(self):
        return len(self.reads) * len(self.haps)

    def cells(self):
        return sum(len(r[0]) for r in self.reads) * sum(len(h) for h in self.haps)


def _mutate(rng, seq: np.ndarray, sub_rate: float, n_rate: float) -> np.ndarray:
    out = seq.copy()
    m = rng.random(len(out)) < sub_rate
    out[m] = BASES[rng.integers(0, 4, m.sum())]
    nm = rng.random(len(out)) < n_rate
    out[nm] = ord("N")
    return out


def phmm_batch(rng, num_reads, num_haps, read_len=(100, 250), hap_max=473, sub_rate=0.10,
               n_rate=0.01, q_range=(6, 40)):
    """Reads ~ U[read_len], haps ~ U[rl, hap_max] built around a common source; reads are sampled
    from the first haplotype with sub_rate substitutions and n_rate N's."""
    hap_lens = []
    rl_lo, rl_hi = read_len
    max_rl = rl_hi
    src = BASES[rng.integers(0, 4, hap_max + 64)]
    haps = []
    for _ in range(num_haps):
        hl = int(rng.integers(min(max_rl, hap_max), hap_max + 1)) if hap_max > max_rl else hap_max
        off = int(rng.integers(0, 32))
        h = _mutate(rng, src[off:off + hl], 0.02, 0.002)
        haps.append(h.tobytes())
        hap_lens.append(hl)
    reads = []
    for _ in range(num_reads):
        rl = int(rng.integers(rl_lo, rl_hi + 1))
        hl = len(haps[0])
        st = int(rng.integers(0, max(1, hl - rl + 1)))
        b = _mutate(rng, np.frombuffer(haps[0], dtype=np.uint8)[st:st + rl], sub_rate, n_rate)
        if len(b) < rl:
            b = np.concatenate([b, BASES[rng.integers(0, 4, rl - len(b))]])
        q = rng.integers(q_range[0], q_range[1] + 1, rl).astype(np.uint8)
        i = rng.integers(40, 46, rl).astype(np.uint8)
        d = rng.integers(40, 46, rl).astype(np.uint8)
        c = np.full(rl, 10, dtype=np.uint8)
        reads.append((b.tobytes(), q.tobytes(), i.tobytes(), d.tobytes(), c.tobytes()))
    return PhmmBatch(reads, haps)


def phmm_dataset(kind: str, num_batches: int, seed: int = 1):
    """'small' / 'large' shaped batches (seed 1 by default)."""
    rng = np.random.default_rng(seed)
    if kind == "large":
        max_r, max_h, hap_max = 1193, 128, 473
    elif kind == "small":
        max_r, max_h, hap_max = 110, 37, 302
    else:
        raise ValueError(kind)
    out = []
    for _ in range(num_batches):
        # skewed batch sizes: most batches small, a few near the maximum
        R = max(1, int(max_r * rng.random() ** 2))
        H = max(1, int(max_h * rng.random() ** 1.5))
        while R * H > 50000:  # MAX_BATCH_SIZE, PairHMMUnitTest.cpp:69,558
            R = max(1, R // 2)
        out.append(phmm_batch(rng, R, H, hap_max=hap_max))
    return out


def write_phmm_file(path, batches):
    """Write the reference's .in text format (read_batch, PairHMMUnitTest.cpp:137,157,464):
    'R H' then R lines 'bases q i d c' (quals stored +33 raw) then H lines 'bases'."""
    with open(path, "w") as f:
        for b in batches:
            f.write(f"{len(b.reads)} {len(b.haps)}\n")
            for bases, q, i, d, c in b.reads:
                enc = lambda s: bytes(x + 33 for x in s).decode("latin-1")
                f.write(f"{bases.decode()} {enc(q)} {enc(i)} {enc(d)} {enc(c)}\n")
            for h in b.haps:
                f.write(h.decode() + "\n")
