"""Regenerate the committed golden vectors from the REFERENCE kernels (oracle/_ref, built from
/root/reference by `make -C oracle ref`). Run in the build container only:

    python tests/golden/make_golden.py

phmm_golden.npz: reads x haps cross product + edge pairs, expected outputs of the reference GKL
AVX2 kernels (compute_fp_avxs/avxd) driven like computelikelihoodsboth
(IntelPairHmmCSource.cpp:61-85): raw f32 bits, raw f64 bits (0 unless the f64 fallback ran) and
the final log10 likelihood bits. The AVX-512 kernels are cross-checked to agree bit for bit.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from genomicsbench_palisade_amd import gen  # noqa: E402
from genomicsbench_palisade_amd._tc import TestcaseArray  # noqa: E402
import oracle_lib  # noqa: E402


def phmm_inputs(seed=2024):
    rng = np.random.default_rng(seed)
    reads, haps = [], []
    # cross-product block: 40 reads x 25 haps, lengths chosen to hit stripe edges (64k, 64k+1)
    rlens = [1, 2, 7, 63, 64, 65, 100, 127, 128, 129, 150, 191, 192, 193, 250, 255, 256, 257, 300]
    while len(rlens) < 40:
        rlens.append(int(rng.integers(1, 320)))
    hlens = [1, 2, 5, 64, 100, 150, 200, 255, 302, 473, 511, 600]
    while len(hlens) < 25:
        hlens.append(int(rng.integers(1, 700)))
    src = gen.BASES[rng.integers(0, 4, 1200)]
    for hl in hlens:
        off = int(rng.integers(0, 400))
        h = gen._mutate(rng, src[off:off + hl], 0.03, 0.01)
        haps.append(h.tobytes())
    alphabet = np.frombuffer(b"ACGTNacgtX", dtype=np.uint8)
    for k, rl in enumerate(rlens):
        off = int(rng.integers(0, 400))
        b = src[off:off + rl].copy()
        sub = rng.random(rl) < [0.0, 0.02, 0.1, 0.3][k % 4]
        b[sub] = gen.BASES[rng.integers(0, 4, sub.sum())]
        if k % 5 == 4:  # exotic bytes: lowercase and unknown letters behave like 'A'
            ex = rng.random(rl) < 0.05
            b[ex] = alphabet[rng.integers(0, len(alphabet), ex.sum())]
        nm = rng.random(rl) < 0.02
        b[nm] = ord("N")
        if k % 7 == 3:   # full quality range incl. >=128 (only the low 7 bits count, &127)
            q = rng.integers(0, 256, rl)
            i = rng.integers(0, 256, rl)
            d = rng.integers(0, 256, rl)
            c = rng.integers(0, 256, rl)
        else:
            q = rng.integers(6, 41, rl)
            i = rng.integers(10, 60, rl)
            d = rng.integers(10, 60, rl)
            c = rng.integers(5, 20, rl)
        reads.append(tuple(np.asarray(x, np.uint8).tobytes() for x in (b, q, i, d, c)))
    # explicit pairs: the GKL KAT (PairHmmUnitTest.java:23-56) and tiny corner cases
    plus = b"+" * 4
    pairs = [((b"ACGT", plus, plus, plus, plus), b"ACGT"),
             ((b"A", b"\x06", b"\x2d", b"\x2d", b"\x0a"), b"A"),
             ((b"A", b"\x06", b"\x2d", b"\x2d", b"\x0a"), b"C"),
             ((b"N", b"\x28", b"\x2d", b"\x2d", b"\x0a"), b"G"),
             ((b"ACGTACGT", b"\x00" * 8, b"\x00" * 8, b"\x00" * 8, b"\x00" * 8), b"TTTTTTTTTTTT"),
             ((b"G" * 70, b"\x7f" * 70, b"\x7f" * 70, b"\x7f" * 70, b"\x7f" * 70), b"G" * 70),
             ((b"C" * 200, b"\x28" * 200, b"\x2d" * 200, b"\x2d" * 200, b"\x0a" * 200), b"A" * 300)]
    return reads, haps, pairs


def fmi_golden():
    """fmi_golden.npz: a 200 kbp genome-like reference, 600 reads (with N's, indels, a short read, an
    all-N read) and the SMEM intervals bwa v1's own code computes for them (tools/bwa/bwt.c
    bwt_smem1/bwt_seed_strategy1 driven like mem_collect_intv, bwamem.c:114-162), which bwa-mem2's
    SMEM search reproduces (cross-checked against oracle/fmi_oracle.c)."""
    import tempfile
    import fmi_util
    lib = fmi_util.ref_bwa()
    if lib is None:
        raise SystemExit("oracle/_ref/libref_bwa.so missing: run `make -C oracle ref` first")
    ref = gen.fmi_reference(200_000, seed=11)
    codes, lens = gen.fmi_reads(ref, 600, read_len=151, seed=12, sub_rate=0.02, n_rate=0.002)
    lens = lens.copy()
    lens[5] = 17            # shorter than min_seed_len
    lens[6] = 60
    codes[7, :] = 4         # all N
    codes[8, :] = 0         # poly-A
    with tempfile.TemporaryDirectory() as d:
        gen.write_fasta(d + "/ref.fa", ref)
        assert lib.ref_bwa_build((d + "/ref.fa").encode(), (d + "/ref").encode()) == 0
        pac = gen.read_pac(d + "/ref.pac")
        assert (pac == ref).all()
        bwt = lib.ref_bwa_load((d + "/ref.bwt").encode())
        per = fmi_util.bwa_smems(lib, bwt, codes, lens)
        lib.ref_bwa_free(bwt)
    rid = np.concatenate([[r] * len(x) for r, x in enumerate(per)]).astype(np.int32)
    flat = np.array([e for x in per for e in x], np.int64).reshape(-1, 5)
    np.savez_compressed(os.path.join(HERE, "fmi_golden.npz"), ref=ref, codes=codes, lens=lens,
                        rid=rid, m=flat[:, 0], n=flat[:, 1], k=flat[:, 2], l=flat[:, 3], s=flat[:, 4])
    print("wrote fmi_golden.npz:", len(rid), "SMEMs for", len(lens), "reads")


def sa_coords(sa, k, s, max_occ):
    """get_sa_entries' row sampling (FMI_search.cpp:1596-1619) over a full SA array."""
    out, cnt = [], []
    for kk, ss in zip(k.tolist(), s.tolist()):
        step = ss // max_occ if ss > max_occ else 1
        rows = list(range(kk, kk + ss, step))[:max_occ]
        out.extend(sa[rows].tolist())
        cnt.append(len(rows))
    return np.array(out, np.int64), np.array(cnt, np.int32)


def fmi_sa_golden():
    """fmi_sa_golden.npz: SA values from bwa v1's own suffix array (tools/bwa bwt_restore_sa + bwt_sa,
    bwt.c:86/421) over the fmi_golden reference -- every row whose SA value is < 64 (the walks that can
    meet the sentinel row) plus 20000 random rows -- and the SA coordinates of the golden SMEMs with
    max_occ 500 and 2 (get_sa_entries' sampling, FMI_search.cpp:1596-1619). bwa v1 stores SA[0] = -1
    for the '$' row; bwa-mem2 stores |text| (FMI_search.cpp:425), which is what is kept here."""
    import tempfile
    import fmi_util
    lib = fmi_util.ref_bwa()
    if lib is None:
        raise SystemExit("oracle/_ref/libref_bwa.so missing: run `make -C oracle ref` first")
    z = np.load(os.path.join(HERE, "fmi_golden.npz"))
    ref = z["ref"]
    n = 2 * len(ref) + 1
    with tempfile.TemporaryDirectory() as d:
        gen.write_fasta(d + "/ref.fa", ref)
        assert lib.ref_bwa_build((d + "/ref.fa").encode(), (d + "/ref").encode()) == 0
        bwt = lib.ref_bwa_load((d + "/ref.bwt").encode())
        sa = fmi_util.bwa_sa(lib, bwt, d + "/ref.sa", np.arange(n, dtype=np.int64))
        lib.ref_bwa_free(bwt)
    assert sa[0] == -1
    sa[0] = n - 1
    assert (np.sort(sa) == np.arange(n)).all()
    rng = np.random.default_rng(31)
    rows = np.unique(np.concatenate([np.nonzero(sa < 64)[0], rng.integers(0, n, 20000)]))
    c500, n500 = sa_coords(sa, z["k"], z["s"], 500)
    c2, n2 = sa_coords(sa, z["k"], z["s"], 2)
    np.savez_compressed(os.path.join(HERE, "fmi_sa_golden.npz"), rows=rows, sa=sa[rows],
                        coords500=c500, counts500=n500, coords2=c2, counts2=n2)
    print("wrote fmi_sa_golden.npz:", len(rows), "rows,", len(c500), "/", len(c2), "coordinates")


def chain_inputs(seed=41):
    """Small call set exercising every branch of chain_dp: tiny calls, duplicate x (dr == 0),
    multi-segment calls (n_segs > 1, seg ids in y bits 48..55), mixed strands, long calls."""
    rng = np.random.default_rng(seed)
    calls = gen.chain_dataset("small", num_calls=40, seed=seed, median_n=300, max_n=6000)
    offs, xs, ys, aq, p4 = [0], [], [], [], []
    for c in range(calls.ncalls):
        o0, o1 = calls.offsets[c], calls.offsets[c + 1]
        xs.append(calls.x[o0:o1]); ys.append(calls.y[o0:o1]); aq.append(calls.avg_qspan[c])
        p4.append(calls.params4[c]); offs.append(offs[-1] + (o1 - o0))
    extra = []
    # n = 1 and n = 2
    extra.append((np.array([5000], np.uint64), np.array([(15 << 32) | 100], np.uint64), 15.0, (5000, 5000, 500, 1)))
    extra.append((np.array([5000, 5010], np.uint64), np.array([(15 << 32) | 100, (15 << 32) | 110], np.uint64), 15.0, (5000, 5000, 500, 1)))
    # multi-segment (paired) call with duplicate positions and segment ids 0/1
    n = 800
    x = np.sort(rng.integers(10_000, 30_000, n)).astype(np.uint64)
    x[100:110] = x[100]  # dr == 0 runs
    seg = rng.integers(0, 2, n).astype(np.uint64)
    q = rng.integers(0, 3000, n).astype(np.uint64)
    y = (seg << np.uint64(48)) | (np.uint64(19) << np.uint64(32)) | q
    extra.append((x, y, 19.0, (5000, 1000, 200, 2)))
    # small max_dist / bw to hit those filters
    x2, y2, a2 = gen.chain_call(rng, 3000)
    extra.append((x2, y2, a2, (400, 300, 30, 1)))
    for x, y, a, p in extra:
        xs.append(np.asarray(x, np.uint64)); ys.append(np.asarray(y, np.uint64)); aq.append(a)
        p4.append(np.array(p, np.int32)); offs.append(offs[-1] + len(x))
    return gen.ChainCalls(np.array(offs), np.concatenate(xs), np.concatenate(ys), np.array(aq, np.float32),
                          np.stack(p4))


def chain_golden():
    """chain_golden.npz: reference scalar chain_dp outputs (tools/minimap2-acceleration/kernel/scalar,
    via oracle/_ref/libref_chain.so) for chain_inputs()."""
    lib = oracle_lib.ref_chain()
    if lib is None:
        raise SystemExit("oracle/_ref/libref_chain.so missing: run `make -C oracle ref` first")
    c = chain_inputs()
    sc, par, tg, pk = oracle_lib.ref_chain_run(lib, c, 4)
    np.savez_compressed(os.path.join(HERE, "chain_golden.npz"), offsets=c.offsets, x=c.x, y=c.y,
                        avg_qspan=c.avg_qspan, params4=c.params4, scores=sc, parents=par, targets=tg, peaks=pk)
    print("wrote chain_golden.npz:", c.ncalls, "calls,", c.nanchors, "anchors")


CHAIN_BT_PARAMS = [(3, 40), (1, 0), (2, 15)]  # (min_cnt, min_sc): minimap2 defaults, everything, between


def chain_bt_inputs(seed=43):
    """Single-segment calls (the testbed asserts sidi == sidj) with avg_qspan computed as the
    testbed does from the anchors ((float)sum_qspan / n, testbed/chain.c:40-41): generator calls,
    n = 1 and 2, a call with long duplicate-x runs (ties in the final reorder) and a long call."""
    rng = np.random.default_rng(seed)
    calls = gen.chain_dataset("small", num_calls=60, seed=seed, median_n=300, max_n=6000)
    offs, xs, ys = [0], [], []
    for c in range(calls.ncalls):
        o0, o1 = calls.offsets[c], calls.offsets[c + 1]
        xs.append(calls.x[o0:o1]); ys.append(calls.y[o0:o1]); offs.append(offs[-1] + (o1 - o0))
    extra = [(np.array([5000], np.uint64), np.array([(15 << 32) | 100], np.uint64)),
             (np.array([5000, 5010], np.uint64), np.array([(15 << 32) | 100, (15 << 32) | 110], np.uint64))]
    n = 1500
    x = np.sort(rng.integers(10_000, 14_000, n)).astype(np.uint64)
    x[200:260] = x[200]
    q = rng.integers(0, 4000, n).astype(np.uint64)
    y = (np.uint64(19) << np.uint64(32)) | q
    o = np.lexsort((y, x))
    extra.append((x[o], y[o]))
    x2, y2, _ = gen.chain_call(rng, 8000)
    extra.append((x2, y2))
    for x, y in extra:
        xs.append(np.asarray(x, np.uint64)); ys.append(np.asarray(y, np.uint64)); offs.append(offs[-1] + len(x))
    offs = np.array(offs)
    x, y = np.concatenate(xs), np.concatenate(ys)
    aq = []
    for c in range(len(offs) - 1):
        span = ((y[offs[c]:offs[c + 1]] >> np.uint64(32)) & np.uint64(0xff)).sum()
        aq.append(np.float32(int(span)) / np.float32(offs[c + 1] - offs[c]))
    nc = len(offs) - 1
    return gen.ChainCalls(offs, x, y, np.array(aq, np.float32), np.tile(np.array([5000, 5000, 500, 1], np.int32), (nc, 1)))


def chain_bt_golden():
    """chain_bt_golden.npz: chains of the reference minimap2-acceleration testbed mm_chain_dp (DP +
    backtrack + reorder, oracle/_ref/libref_chain_bt.so) for chain_bt_inputs(), per CHAIN_BT_PARAMS
    set k: u{k} (chains of all calls concatenated), nch{k} (chains per call), bx{k}/by{k} (anchors
    concatenated), nan{k} (anchors per call)."""
    lib = oracle_lib.ref_chain_bt()
    if lib is None:
        raise SystemExit("oracle/_ref/libref_chain_bt.so missing: run `make -C oracle ref` first")
    c = chain_bt_inputs()
    arrs = dict(offsets=c.offsets, x=c.x, y=c.y, avg_qspan=c.avg_qspan, params4=c.params4,
                bt_params=np.array(CHAIN_BT_PARAMS, np.int32))
    for k, (mc, ms) in enumerate(CHAIN_BT_PARAMS):
        us, an = oracle_lib.ref_chain_bt_run(lib, c, mc, ms)
        arrs[f"u{k}"] = np.concatenate(us) if us else np.zeros(0, np.uint64)
        arrs[f"nch{k}"] = np.array([len(u) for u in us], np.int64)
        arrs[f"bx{k}"] = np.concatenate([a[0] for a in an])
        arrs[f"by{k}"] = np.concatenate([a[1] for a in an])
        arrs[f"nan{k}"] = np.array([len(a[0]) for a in an], np.int64)
    np.savez_compressed(os.path.join(HERE, "chain_bt_golden.npz"), **arrs)
    print("wrote chain_bt_golden.npz:", c.ncalls, "calls,", c.nanchors, "anchors,",
          [int(arrs[f"nch{k}"].sum()) for k in range(len(CHAIN_BT_PARAMS))], "chains")


def bsw_inputs(seed=77):
    """Synthetic pairs shaped like the bsw datasets plus edge pairs: qlen 1 and 255 (the buffer
    maximum), tlen 1, a target much longer than query + w (empty bands), all-N sequences, identical
    long sequences (no zdrop), h0 0 and large."""
    p = gen.bsw_pairs(3000, seed=seed)
    rng = np.random.default_rng(seed + 1)
    extra = []
    q = rng.integers(0, 4, 255).astype(np.uint8)
    extra += [(q[:1], q[:1], 30), (q[:1], q[:5], 30), (q, q, 40), (np.concatenate([q, q[:50]]), q, 60),
              (q[:200], q[:10], 70), (np.full(40, 4, np.uint8), np.full(30, 4, np.uint8), 25),
              (rng.integers(0, 4, 2046).astype(np.uint8), q[:10], 20), (q[:60], q[:60], 0), (q[:60], q[:60], 250),
              (rng.integers(0, 4, 300).astype(np.uint8), q[:150], 5)]
    tg = [p.tgt] + [e[0] for e in extra]
    qq = [p.qry] + [e[1] for e in extra]
    tl = np.concatenate([p.tlen, np.array([len(e[0]) for e in extra], np.int32)])
    ql = np.concatenate([p.qlen, np.array([len(e[1]) for e in extra], np.int32)])
    h0 = np.concatenate([p.h0, np.array([e[2] for e in extra], np.int32)])
    toff = np.zeros(len(tl), np.int64); toff[1:] = np.cumsum(tl)[:-1]
    qoff = np.zeros(len(ql), np.int64); qoff[1:] = np.cumsum(ql)[:-1]
    return gen.BswPairs(np.concatenate(tg), toff, tl, np.concatenate(qq), qoff, ql, h0)


BSW_PARAM_SETS = [  # name, kwargs for bsw.default_params
    ("default", {}),
    ("narrow_w", {"w": 7}),
    ("no_zdrop", {"zdrop": 0}),
    ("small_zdrop", {"zdrop": 10}),
    ("asym_gaps", {"o_del": 4, "e_del": 2, "o_ins": 7, "e_ins": 3, "end_bonus": 0}),
    ("other_mat", {"match": 2, "mismatch": 3, "ambig": -2}),
]


def bsw_golden():
    """bsw_golden.npz: bwa v1 ksw_extend2 (the function scalarBandedSWA restates, compiled from
    tools/bwa via oracle/_ref/libref_bwa.so) outputs for bsw_inputs() under each of BSW_PARAM_SETS."""
    from genomicsbench_palisade_amd import bsw
    lib = oracle_lib.ref_bsw()
    if lib is None:
        raise SystemExit("oracle/_ref/libref_bwa.so missing: run `make -C oracle ref` first")
    p = bsw_inputs()
    arrs = dict(tgt=p.tgt, toff=p.toff, tlen=p.tlen, qry=p.qry, qoff=p.qoff, qlen=p.qlen, h0=p.h0)
    for name, kw in BSW_PARAM_SETS:
        par = bsw.default_params(**kw)
        arrs[name + "_params"] = par.as_array()
        arrs[name + "_mat"] = par.mat_array()
        arrs[name + "_out"] = oracle_lib.ref_bsw_run(lib, p, par)
    np.savez_compressed(os.path.join(HERE, "bsw_golden.npz"), **arrs)
    print("wrote bsw_golden.npz:", p.n, "pairs x", len(BSW_PARAM_SETS), "parameter sets")


def main():
    bsw_golden()
    chain_golden()
    chain_bt_golden()
    fmi_golden()
    ref = oracle_lib.ref_phmm()
    if ref is None:
        raise SystemExit("oracle/_ref/libref_phmm.so missing: run `make -C oracle ref` first")
    reads, haps, pairs = phmm_inputs()
    cross = TestcaseArray(reads, haps)
    extra = TestcaseArray.from_pairs(pairs)
    outs = []
    for ta in (cross, extra):
        n = ta.n
        res = {}
        for eng in (256, 512):
            out = np.zeros(n)
            rf = np.zeros(n, np.float32)
            rd = np.zeros(n)
            ref.ref_phmm_batch(ctypes.addressof(ta.arr), n, out.ctypes.data, rf.ctypes.data,
                               rd.ctypes.data, eng, 8)
            res[eng] = (out, rf, rd)
        for a, b in zip(res[256], res[512]):
            assert (a.view(np.uint8) == b.view(np.uint8)).all(), "AVX2 and AVX-512 disagree"
        outs.append(res[256])
    field = lambda k: [r[k] for r in reads]
    np.savez_compressed(
        os.path.join(HERE, "phmm_golden.npz"),
        read_bases=np.frombuffer(b"".join(field(0)), np.uint8),
        read_q=np.frombuffer(b"".join(field(1)), np.uint8),
        read_i=np.frombuffer(b"".join(field(2)), np.uint8),
        read_d=np.frombuffer(b"".join(field(3)), np.uint8),
        read_c=np.frombuffer(b"".join(field(4)), np.uint8),
        read_len=np.array([len(r[0]) for r in reads], np.int32),
        hap_bases=np.frombuffer(b"".join(haps), np.uint8),
        hap_len=np.array([len(h) for h in haps], np.int32),
        cross_final=outs[0][0], cross_raw_f=outs[0][1], cross_raw_d=outs[0][2],
        pair_read_bases=np.frombuffer(b"".join(p[0][0] for p in pairs), np.uint8),
        pair_read_q=np.frombuffer(b"".join(p[0][1] for p in pairs), np.uint8),
        pair_read_i=np.frombuffer(b"".join(p[0][2] for p in pairs), np.uint8),
        pair_read_d=np.frombuffer(b"".join(p[0][3] for p in pairs), np.uint8),
        pair_read_c=np.frombuffer(b"".join(p[0][4] for p in pairs), np.uint8),
        pair_read_len=np.array([len(p[0][0]) for p in pairs], np.int32),
        pair_hap_bases=np.frombuffer(b"".join(p[1] for p in pairs), np.uint8),
        pair_hap_len=np.array([len(p[1]) for p in pairs], np.int32),
        pair_final=outs[1][0], pair_raw_f=outs[1][1], pair_raw_d=outs[1][2],
    )
    print("wrote phmm_golden.npz:", cross.n, "cross testcases,", extra.n, "pairs; f64 fallbacks:",
          int((outs[0][1] < np.float32(1e-28)).sum()), "; KAT", outs[1][0][0])


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for what in sys.argv[1:]:
            globals()[what + "_golden"]() if what != "phmm" else main()
        raise SystemExit(0)
    main()
