#!/usr/bin/env python3
"""make-inputs.py -- write a synthetic <INPUTS_DIR> in the layout scripts/run-cpu.sh (and the
reference's own scripts/run-cpu.sh:24-86) reads, from the seeded generators of
genomicsbench_palisade_amd/gen.py (the real input-datasets tarball is not available):

    fmi/broad.pac, fmi/broad.bwt.2bit.64      512 Mbp genome-like reference (+RC index, built on the GPU)
    fmi/{small,large}/SRR7733443_{1m,10m}_1.fastq   151 bp reads
    bsw/{small,large}/bandedSWA_SRR7733443_{100k,1m}_input.txt   loadPairs format
    phmm/{small/5m.in,large/large.in}         read_batch format
    chain/{small/in-1k.txt,large/c_elegans_40x.10k.in}           read_call format

    python scripts/make-inputs.py <INPUTS_DIR> <small|large> [--scale F] [--only fmi,bsw,phmm,chain]

--scale multiplies every count (reads, pairs, batches, calls, reference length) for quick runs.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from genomicsbench_palisade_amd import gen  # noqa: E402


def write_pac(path, codes):
    """bwa .pac: 4 bases per byte, first base in the high bits, then (len % 4 == 0 ? 0x00 : nothing)
    and a final byte len % 4 (what pac_seq_len / pac2nt read, FMI_search.cpp:96-169)."""
    n = len(codes)
    pad = (-n) % 4
    b = np.concatenate([codes, np.zeros(pad, np.uint8)]).reshape(-1, 4)
    packed = (b[:, 0] << 6 | b[:, 1] << 4 | b[:, 2] << 2 | b[:, 3]).astype(np.uint8)
    tail = np.array([0, 0] if n % 4 == 0 else [n % 4], np.uint8)
    with open(path, "wb") as f:
        f.write(packed.tobytes())
        f.write(tail.tobytes())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("inputs_dir")
    ap.add_argument("size", choices=("small", "large"))
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--only", default="fmi,bsw,phmm,chain")
    a = ap.parse_args()
    legs = set(a.only.split(","))
    d, large, sc = a.inputs_dir, a.size == "large", a.scale

    def mk(*p):
        path = os.path.join(d, *p)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        return path

    if "fmi" in legs:
        ref = gen.fmi_reference(max(20_000, int(512e6 * sc)), seed=7)
        idx_prefix = mk("fmi", "broad")
        if not os.path.exists(idx_prefix + ".bwt.2bit.64"):
            write_pac(idx_prefix + ".pac", ref)
            from genomicsbench_palisade_amd import fmi
            fmi.Index.build(ref, out_path=idx_prefix + ".bwt.2bit.64").close()
        n = max(1, int((10_000_000 if large else 1_000_000) * sc))
        codes, lens = gen.fmi_reads(ref, n, read_len=151, seed=8 if large else 9)
        name = "large/SRR7733443_10m_1.fastq" if large else "small/SRR7733443_1m_1.fastq"
        gen.write_fastq(mk("fmi", *name.split("/")), codes, lens)
    if "bsw" in legs:
        n = max(1, int((gen.BSW_LARGE_PAIRS if large else gen.BSW_SMALL_PAIRS) * sc))
        name = "large/bandedSWA_SRR7733443_1m_input.txt" if large else "small/bandedSWA_SRR7733443_100k_input.txt"
        gen.write_bsw_file(mk("bsw", *name.split("/")), gen.bsw_dataset(n, seed=11))
    if "phmm" in legs:
        nb = max(1, int((64 if large else 256) * sc))
        name = "large/large.in" if large else "small/5m.in"
        gen.write_phmm_file(mk("phmm", *name.split("/")), gen.phmm_dataset(a.size, nb, seed=1))
    if "chain" in legs:
        nc = max(2, int((10_000 if large else 1_000) * sc))
        name = "large/c_elegans_40x.10k.in" if large else "small/in-1k.txt"
        gen.write_chain_file(mk("chain", *name.split("/")),
                             gen.chain_dataset(a.size, num_calls=nc, seed=5, max_n=max(100, int(87271 * min(1.0, sc * 10)))))


if __name__ == "__main__":
    main()
