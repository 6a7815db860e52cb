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


# ---------------------------------------------------------------------------------------------
# chain: minimap2-style anchor sets (n ~ lognormal, max 87 271 anchors per call,
# anchors sorted by x, ~85% forward strand, spans {15,19,28}, max_dist 5000, bw 500, n_segs 1;
# 'large' = 10 000 calls, 'small' = 1 000; seed 5)
# ---------------------------------------------------------------------------------------------
class ChainCalls:
    """CSR anchor sets: anchors of call c are x[offsets[c]:offsets[c+1]] (call_t, host_data.h:19-39)."""

    def __init__(self, offsets, x, y, avg_qspan, params4):
        self.offsets = np.asarray(offsets, np.int64)
        self.x = np.asarray(x, np.uint64)
        self.y = np.asarray(y, np.uint64)
        self.avg_qspan = np.asarray(avg_qspan, np.float32)
        self.params4 = np.asarray(params4, np.int32).reshape(-1, 4)  # max_dist_x, max_dist_y, bw, n_segs

    @property
    def ncalls(self):
        return len(self.offsets) - 1

    @property
    def nanchors(self):
        return int(self.offsets[-1])

    def slice(self, lo: int, hi: int) -> "ChainCalls":
        """Calls lo..hi-1 as their own CSR set (anchors copied, offsets rebased)."""
        o0, o1 = int(self.offsets[lo]), int(self.offsets[hi])
        return ChainCalls(self.offsets[lo:hi + 1] - o0, self.x[o0:o1].copy(), self.y[o0:o1].copy(),
                          self.avg_qspan[lo:hi].copy(), self.params4[lo:hi].copy())


def chain_call(rng, n: int):
    """One read's anchors: a collinear true locus (~85% of anchors, with small indel drift) plus
    spurious hits at other loci (repeats), mixed strands, sorted by x like minimap2's dumps."""
    n_true = max(1, int(n * rng.uniform(0.75, 0.95)))
    n_sp = n - n_true
    spans = rng.choice(np.array([15, 19, 28]), size=n)
    Lq = int(n_true * rng.uniform(6, 14)) + 100
    rid0, rev0 = int(rng.integers(0, 24)), int(rng.random() < 0.15)
    r0 = int(rng.integers(1_000_000, 200_000_000))
    qpos = np.sort(rng.integers(0, Lq, n_true))
    drift = np.cumsum(rng.choice(np.array([-2, -1, 0, 0, 0, 0, 1, 2]), size=n_true) *
                      (rng.random(n_true) < 0.1))
    rpos = r0 + qpos + drift
    xs = [(rev0 << 63) | (rid0 << 32) | rpos.astype(np.uint64)]
    ys = [qpos]
    if n_sp:
        nl = max(1, n_sp // int(rng.integers(5, 60)))
        loc = rng.integers(0, nl, n_sp)
        lrid = rng.integers(0, 24, nl)
        lrev = (rng.random(nl) < 0.3).astype(np.uint64)
        lr0 = rng.integers(1_000_000, 200_000_000, nl)
        q = rng.integers(0, Lq, n_sp)
        rp = lr0[loc] + q + rng.integers(-50, 50, n_sp)
        xs.append((lrev[loc] << np.uint64(63)) | (lrid[loc].astype(np.uint64) << np.uint64(32)) | rp.astype(np.uint64))
        ys.append(q)
    x = np.concatenate([np.asarray(a, np.uint64) for a in xs])
    q = np.concatenate(ys).astype(np.uint64)
    y = (spans.astype(np.uint64) << np.uint64(32)) | q  # seg id 0
    order = np.lexsort((y, x))
    return x[order], y[order], float(spans.mean())


def chain_dataset(kind: str = "large", num_calls: int | None = None, seed: int = 5,
                  median_n: int = 1500, max_n: int = 87271):
    rng = np.random.default_rng(seed)
    if num_calls is None:
        num_calls = 10_000 if kind == "large" else 1_000
    ns = np.minimum(max_n, np.maximum(2, rng.lognormal(np.log(median_n), 1.0, num_calls).astype(np.int64)))
    ns[int(rng.integers(0, num_calls))] = max_n  # the logged maximum (scripts/chain_small_outt:3938)
    offs = np.zeros(num_calls + 1, np.int64)
    xs, ys, aq = [], [], []
    for c in range(num_calls):
        x, y, a = chain_call(rng, int(ns[c]))
        xs.append(x)
        ys.append(y)
        aq.append(a)
        offs[c + 1] = offs[c] + len(x)
    params = np.tile(np.array([5000, 5000, 500, 1], np.int32), (num_calls, 1))
    return ChainCalls(offs, np.concatenate(xs), np.concatenate(ys), np.array(aq, np.float32), params)


def write_chain_file(path, calls: ChainCalls):
    """read_call format (benchmarks/chain/src/host_data_io.cpp:40-80)."""
    with open(path, "w") as f:
        for c in range(calls.ncalls):
            o0, o1 = calls.offsets[c], calls.offsets[c + 1]
            p = calls.params4[c]
            f.write(f"{o1 - o0}\t{calls.avg_qspan[c]:f}\t{p[0]}\t{p[1]}\t{p[2]}\t{p[3]}\n")
            for xx, yy in zip(calls.x[o0:o1].tolist(), calls.y[o0:o1].tolist()):
                f.write(f"{xx}\t{yy}\n")
            f.write("EOR\n")


class BswPairs:
    """Flattened bsw pairs: pair p has target (ref) tgt[toff[p]:toff[p]+tlen[p]] and query
    qry[qoff[p]:qoff[p]+qlen[p]], codes 0..4 (loadPairs subtracts '0', main_banded.cpp:190-195)."""

    def __init__(self, tgt, toff, tlen, qry, qoff, qlen, h0):
        self.tgt, self.toff, self.tlen = tgt, toff, tlen
        self.qry, self.qoff, self.qlen = qry, qoff, qlen
        self.h0 = h0

    @property
    def n(self):
        return len(self.h0)

    def subset(self, idx):
        idx = np.asarray(idx, np.int64)
        tl, ql = self.tlen[idx], self.qlen[idx]
        toff = np.zeros(len(idx), np.int64)
        qoff = np.zeros(len(idx), np.int64)
        toff[1:] = np.cumsum(tl)[:-1]
        qoff[1:] = np.cumsum(ql)[:-1]
        tgt = np.concatenate([self.tgt[self.toff[p]:self.toff[p] + self.tlen[p]] for p in idx.tolist()]) \
            if len(idx) else np.zeros(0, np.uint8)
        qry = np.concatenate([self.qry[self.qoff[p]:self.qoff[p] + self.qlen[p]] for p in idx.tolist()]) \
            if len(idx) else np.zeros(0, np.uint8)
        return BswPairs(tgt, toff, tl.copy(), qry, qoff, ql.copy(), self.h0[idx].copy())

    def slice(self, lo: int, hi: int) -> "BswPairs":
        """Pairs lo..hi-1 (contiguous, so the sequence pools are sliced, not gathered)."""
        if hi <= lo:
            return self.subset(np.zeros(0, np.int64))
        t0, t1 = int(self.toff[lo]), int(self.toff[hi - 1] + self.tlen[hi - 1])
        q0, q1 = int(self.qoff[lo]), int(self.qoff[hi - 1] + self.qlen[hi - 1])
        return BswPairs(self.tgt[t0:t1].copy(), (self.toff[lo:hi] - t0).astype(np.int64), self.tlen[lo:hi].copy(),
                        self.qry[q0:q1].copy(), (self.qoff[lo:hi] - q0).astype(np.int64), self.qlen[lo:hi].copy(),
                        self.h0[lo:hi].copy())


def _ragged_local(lens):
    """(pair index, position within pair) for every element of a ragged concatenation."""
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens)[:-1]
    tot = int(np.sum(lens))
    pid = np.repeat(np.arange(len(lens), dtype=np.int64), lens)
    return offs, pid, np.arange(tot, dtype=np.int64) - offs[pid]


def bsw_pairs(num_pairs: int, seed: int = 11, qlen=(10, 150), extra=(0, 100), n_rate=0.002):
    """bwa-mem-like extension pairs: query ~ U[10,150], target = query
    mutated (per-pair substitution rate 0-12 %, one indel of +-1..6 bp in 30 % of pairs, 8 % of
    targets unrelated) followed by U[0,100] extra bases; h0 = 0 for 20 %, else U[10,70]."""
    rng = np.random.default_rng(seed)
    n = int(num_pairs)
    ql = rng.integers(qlen[0], qlen[1] + 1, n).astype(np.int32)
    tl = (ql + rng.integers(extra[0], extra[1] + 1, n)).astype(np.int32)
    h0 = np.where(rng.random(n) < 0.2, 0, rng.integers(10, 71, n)).astype(np.int32)
    qoff, qpid, _ = _ragged_local(ql)
    qry = rng.integers(0, 4, int(ql.sum())).astype(np.uint8)
    qry[rng.random(len(qry)) < n_rate] = 4
    toff, tpid, k = _ragged_local(tl)
    brk = (rng.random(n) * ql).astype(np.int64)
    dlt = rng.integers(1, 7, n) * np.where(rng.random(n) < 0.5, -1, 1)
    dlt[rng.random(n) >= 0.3] = 0
    src = k + np.where(k >= brk[tpid], dlt[tpid], 0)
    ok = (src >= 0) & (src < ql[tpid]) & (rng.random(n) >= 0.08)[tpid]
    tgt = rng.integers(0, 4, len(k)).astype(np.uint8)
    tgt[ok] = qry[qoff[tpid[ok]] + src[ok]]
    sub = rng.random(n) * 0.12
    m = rng.random(len(tgt)) < sub[tpid]
    tgt[m] = rng.integers(0, 4, int(m.sum())).astype(np.uint8)
    tgt[rng.random(len(tgt)) < n_rate] = 4
    return BswPairs(tgt, toff, tl, qry, qoff, ql, h0)


def write_bsw_file(path, pairs: BswPairs):
    """loadPairs format (main_banded.cpp:160-202): per pair 'h0', target, query lines of '0'..'4'."""
    with open(path, "wb") as f:
        for p in range(pairs.n):
            t = (pairs.tgt[pairs.toff[p]:pairs.toff[p] + pairs.tlen[p]] + 48).tobytes()
            q = (pairs.qry[pairs.qoff[p]:pairs.qoff[p] + pairs.qlen[p]] + 48).tobytes()
            f.write(b"%d\n%s\n%s\n" % (int(pairs.h0[p]), t, q))


def concat_bsw(parts):
    """Concatenate BswPairs sets (offsets rebased)."""
    tl = np.concatenate([p.tlen for p in parts])
    ql = np.concatenate([p.qlen for p in parts])
    toff = np.zeros(len(tl), np.int64)
    qoff = np.zeros(len(ql), np.int64)
    toff[1:] = np.cumsum(tl, dtype=np.int64)[:-1]
    qoff[1:] = np.cumsum(ql, dtype=np.int64)[:-1]
    return BswPairs(np.concatenate([p.tgt for p in parts]), toff, tl, np.concatenate([p.qry for p in parts]),
                    qoff, ql, np.concatenate([p.h0 for p in parts]))


BSW_LARGE_PAIRS = 10_606_460  # scripts/bsw_large:6
BSW_SMALL_PAIRS = 100_000     # scripts/bsw_outt:33


def bsw_dataset(num_pairs: int = BSW_LARGE_PAIRS, seed: int = 11, threads: int = 16, chunk: int = 1 << 18):
    """bsw_pairs at dataset scale: chunk c is bsw_pairs(chunk, seed=(seed, c)), generated on a thread
    pool (numpy releases the GIL) and concatenated."""
    from concurrent.futures import ThreadPoolExecutor
    sizes = [min(chunk, num_pairs - o) for o in range(0, num_pairs, chunk)]
    with ThreadPoolExecutor(max(1, threads)) as ex:
        parts = list(ex.map(lambda a: bsw_pairs(a[1], seed=[seed, a[0]]), enumerate(sizes)))
    return concat_bsw(parts) if parts else bsw_pairs(0, seed)
