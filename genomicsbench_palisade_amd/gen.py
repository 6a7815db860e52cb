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


# ---------------------------------------------------------------------------------------------
# fmi: synthetic reference + reads ('large' = 10 M x 151 bp reads over a 512 Mbp
# reference (+RC); 1% substitutions, 0.1% indels, 0.05% N; seed 7)
# ---------------------------------------------------------------------------------------------
def fmi_reference(length: int, seed: int = 7, repeat_frac: float = 0.08):
    """Random A/C/G/T codes (0..3) with genome-like structure: ~repeat_frac of the sequence is
    overwritten by mutated copies of earlier segments (interspersed repeats) and short tandem
    repeats, so the SMEM search sees multi-copy intervals and reseeding, not only unique hits."""
    rng = np.random.default_rng(seed)
    ref = rng.integers(0, 4, length, dtype=np.uint8)
    budget = int(length * repeat_frac)
    while budget > 0 and length > 1000:
        if rng.random() < 0.85:  # interspersed copy, 1-15% divergence
            L = int(min(length // 4, max(50, rng.geometric(1 / 800))))
            src = int(rng.integers(0, length - L))
            dst = int(rng.integers(0, length - L))
            seg = ref[src:src + L].copy()
            mut = rng.random(L) < rng.uniform(0.0, 0.15)
            seg[mut] = rng.integers(0, 4, int(mut.sum()), dtype=np.uint8)
            if rng.random() < 0.5:
                seg = (3 - seg[::-1]).astype(np.uint8)
        else:  # tandem repeat of a short unit
            unit = rng.integers(0, 4, int(rng.integers(1, 7)), dtype=np.uint8)
            L = int(rng.integers(20, 300))
            seg = np.resize(unit, L)
            dst = int(rng.integers(0, length - L))
        ref[dst:dst + len(seg)] = seg
        budget -= len(seg)
    return ref


def fmi_reads(ref: np.ndarray, num_reads: int, read_len: int = 151, seed: int = 7, sub_rate=0.01,
              indel_rate=0.001, n_rate=0.0005, chunk: int = 250_000):
    """Reads sampled uniformly from both strands; returns (codes[num_reads, read_len] uint8 with
    4 = N, lens int32). Codes follow fmi.cpp:141-177 (A0 C1 G2 T3, anything else 4). Generated in
    chunks so 10 M-read sets stay within a few GB of host memory."""
    rng = np.random.default_rng(seed)
    G = len(ref)
    out = np.empty((num_reads, read_len), np.uint8)
    span = read_len + 8
    for c0 in range(0, num_reads, chunk):
        nr = min(chunk, num_reads - c0)
        starts = rng.integers(0, G - span, nr)
        strand = rng.random(nr) < 0.5
        frag = ref[starts[:, None] + np.arange(span)[None, :]]
        # indels: at most one per read, applied on the fragment before trimming (vectorized)
        R = np.nonzero(rng.random(nr) < indel_rate * read_len)[0]
        if len(R):
            p = rng.integers(1, read_len - 1, len(R))[:, None]
            dele = (rng.random(len(R)) < 0.5)[:, None]
            col = np.arange(span)[None, :]
            src = np.where(dele, np.minimum(col + (col >= p), span - 1), col - (col > p))
            sub_frag = np.take_along_axis(frag[R], src, axis=1)
            ins_rows = np.nonzero(~dele[:, 0])[0]
            sub_frag[ins_rows, p[ins_rows, 0]] = rng.integers(0, 4, len(ins_rows))
            frag[R] = sub_frag
        frag = np.ascontiguousarray(frag[:, :read_len])
        frag[strand] = (3 - frag[strand, ::-1])
        flat = frag.reshape(-1)
        si = rng.integers(0, flat.size, rng.binomial(flat.size, sub_rate))
        flat[si] = (flat[si] + rng.integers(1, 4, len(si))) % 4
        flat[rng.integers(0, flat.size, rng.binomial(flat.size, n_rate))] = 4
        out[c0:c0 + nr] = frag
    return out, np.full(num_reads, read_len, np.int32)


def write_fasta(path, ref: np.ndarray, name="chr1", width=80):
    s = np.frombuffer(b"ACGT", np.uint8)[ref].tobytes()
    with open(path, "wb") as f:
        f.write(b">" + name.encode() + b"\n")
        for i in range(0, len(s), width):
            f.write(s[i:i + width] + b"\n")


def write_fastq(path, codes: np.ndarray, lens: np.ndarray):
    lut = np.frombuffer(b"ACGTN", np.uint8)
    with open(path, "wb") as f:
        for r in range(len(lens)):
            s = lut[codes[r, :lens[r]]].tobytes()
            f.write(b"@r%d\n%s\n+\n%s\n" % (r, s, b"I" * len(s)))


def read_pac(path):
    """pac2nt (FMI_search.cpp:93-169): forward-strand codes from a bwa .pac file."""
    raw = np.fromfile(path, np.uint8)
    seq_len = (len(raw) - 2) * 4 + int(raw[-1])  # pac_seq_len: (ftell(-1) - 1) * 4 + last byte
    b = raw[: (seq_len + 3) // 4]
    codes = np.stack([(b >> 6) & 3, (b >> 4) & 3, (b >> 2) & 3, b & 3], axis=1).reshape(-1)
    return codes[:seq_len].astype(np.uint8)
