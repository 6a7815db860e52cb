"""The FMI_search class drop-in (include/gb_compat/FMI_search.h -> libgb_fmi_dropin.so): the mangled
methods of tools/bwa-mem2/src/FMI_search.h:101-224 are exported, and tests/cpp/fmi_class_driver --
benchmarks/fmi/fmi.cpp:253-348's batch loop written against the class, run from several host threads
-- reproduces the oracle bit for bit: every batch's sorted SMEMs and phase counts, the raw (unsorted)
outputs of getSMEMsAllPosOneThread / getSMEMsOnePosOneThread / bwtSeedStrategyAllPosOneThread in the
reference's emission order with their side effects on the caller's arrays, the SA methods
(get_sa_entries_prefetch, get_sa_entry_compressed, call_one_step, get_sa_entry) and the
backwardExt count."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import fmi_util
import oracle_lib
from conftest import ROOT
from genomicsbench_palisade_amd import gen

LIB = os.path.join(ROOT, "genomicsbench_palisade_amd", "lib", "libgb_fmi_dropin.so")
DRIVER = os.path.join(ROOT, "tests", "_build", "fmi_class_driver")

MANGLED = [
    "_ZN10FMI_searchC1EPKc", "_ZN10FMI_searchD1Ev", "_ZN10FMI_search11build_indexEv", "_ZN10FMI_search10load_indexEv",
    "_ZN10FMI_search23getSMEMsOnePosOneThreadEPhPsPiS2_iiPK7bseq1_tS2_iiP11smem_structPl",
    "_ZN10FMI_search23getSMEMsAllPosOneThreadEPhPiS1_iiPK7bseq1_tS1_iiP11smem_structPl",
    "_ZN10FMI_search30bwtSeedStrategyAllPosOneThreadEPhPiiPK7bseq1_tS1_iP11smem_struct",
    "_ZN10FMI_search9sortSMEMsEP11smem_structPliii",
    "_ZN10FMI_search12get_sa_entryEl", "_ZN10FMI_search14get_sa_entriesEPlS0_ji",
    "_ZN10FMI_search14get_sa_entriesEP11smem_structPlPiji",
    "_ZN10FMI_search14get_sa_entriesEP11smem_structPlPijii",
    "_ZN10FMI_search23get_sa_entry_compressedEli", "_ZN10FMI_search13call_one_stepElRlS0_",
    "_ZN10FMI_search23get_sa_entries_prefetchEP11smem_structPlS2_liiRl",
    "_ZN10FMI_search8getSMEMsEPhiiiiiP11smem_structPl",
]


def test_dropin_exports_reference_mangled_methods():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [m for m in MANGLED if m not in syms]
    assert not missing, missing


SM = fmi_util.SMEM_DTYPE


def _parse(path, batch_sizes, bc0):
    raw = open(path, "rb").read()
    o = [0]

    def take(dt, n):
        a = np.frombuffer(raw, dt, count=n, offset=o[0])
        o[0] += a.nbytes
        return a
    nb = int(take(np.int64, 1)[0])
    n123, batches = [], []
    for _ in range(nb):
        c = take(np.int64, 3)
        n123.append(c)
        batches.append(take(SM, int(c.sum())))
    r = {"n123": np.array(n123), "sorted": np.concatenate(batches) if batches else np.zeros(0, SM),
         "batch_counts": np.array([len(b) for b in batches])}
    r["raw1"] = take(SM, int(take(np.int64, 1)[0]))
    r["rid_after"] = take(np.int32, bc0)
    r["intv_after"] = take(np.int32, bc0)
    r["qpos_after"] = take(np.int16, int(take(np.int64, 1)[0]))
    r["raw2"] = take(SM, int(take(np.int64, 1)[0]))
    r["raw3"] = take(SM, int(take(np.int64, 1)[0]))
    cc, cid = take(np.int64, 2)
    r["coords"] = take(np.int64, int(cc))
    r["coord_id"] = int(cid)
    r["compressed"] = take(np.int64, 64)
    r["one_step"] = take(np.int64, 3 * 64).reshape(64, 3)
    r["raw_sa"] = take(np.int64, 16)
    r["sentinel"], r["n"], r["calls"] = (int(x) for x in take(np.int64, 3))
    assert o[0] == len(raw)
    return r


def _fields(a):
    return np.stack([a["rid"].astype(np.int64), a["m"].astype(np.int64), a["n"].astype(np.int64),
                     a["k"], a["l"], a["s"]], axis=1) if len(a) else np.zeros((0, 6), np.int64)


def _oracle_phases(oi, codes, lens, bc, maxlen, min_seed_len):
    """fmi.cpp's batch-0 steps on the oracle's class-phase entry point (reference emission order)."""
    L = oracle_lib.oracle()
    L.fmi_oracle_phase.restype = ctypes.c_int64
    vp = ctypes.c_void_p
    L.fmi_oracle_phase.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int32, vp]
    q = np.ascontiguousarray(codes[:bc]).reshape(-1)
    ln = np.ascontiguousarray(lens[:bc], np.int32)
    cum = (np.arange(bc) * maxlen).astype(np.int32)
    cap = bc * maxlen * 4 + 64
    rid = np.arange(cap, dtype=np.int32)
    intv = np.ones(cap, np.int32)
    qpos = np.zeros(cap, np.int16)
    out = np.zeros(cap, SM)
    n1 = L.fmi_oracle_phase(oi.h, 0, q.ctypes.data, ln.ctypes.data, cum.ctypes.data, qpos.ctypes.data, intv.ctypes.data,
                            rid.ctypes.data, bc, maxlen, min_seed_len, out.ctypes.data)
    raw1 = out[:n1].copy()
    rid_after, intv_after = rid[:bc].copy(), intv[:bc].copy()
    split_len = int(min_seed_len * 1.5 + .499)
    pos = 0
    for p in raw1:
        start, end = int(p["m"]), int(p["n"]) + 1
        if end - start < split_len or p["s"] > 10:
            continue
        rid[pos], qpos[pos], intv[pos] = p["rid"], (end + start) >> 1, p["s"] + 1
        pos += 1
    n2 = L.fmi_oracle_phase(oi.h, 1, q.ctypes.data, ln.ctypes.data, cum.ctypes.data, qpos.ctypes.data, intv.ctypes.data,
                            rid.ctypes.data, pos, maxlen, min_seed_len, out.ctypes.data)
    raw2, qpos_after = out[:n2].copy(), qpos[:pos].copy()
    intv[:bc] = 20
    n3 = L.fmi_oracle_phase(oi.h, 2, q.ctypes.data, ln.ctypes.data, cum.ctypes.data, qpos.ctypes.data, intv.ctypes.data,
                            rid.ctypes.data, bc, maxlen, min_seed_len + 1, out.ctypes.data)
    return raw1, rid_after, intv_after, raw2, qpos_after, out[:n3].copy()


@pytest.mark.gpu
@pytest.mark.parametrize("size,nreads,L,batch,threads,seed,build,tile,wave",
                         [(300_000, 1500, 151, 512, 3, 3, False, "", ""), (120_000, 700, 101, 64, 2, 4, True, "", ""),
                          (200_000, 1100, 151, 512, 2, 5, False, "100", ""),
                          (300_000, 1500, 151, 512, 3, 3, False, "", "0"), (150_000, 600, 300, 128, 2, 6, False, "", "")])
def test_class_driver_matches_oracle(tmp_path, size, nreads, L, batch, threads, seed, build, tile, wave):
    """tile: GB_FMI_TASK_TILE, tasks per launch of the per-call kernels (the scratch bound; 100 forces
    several tiles per call, with the overflow pass inside each). wave: GB_FMI_TASK_WAVE -- reads up to
    256 bases run a wave per task (fmi_wave.h), "0" forces a lane per task; 300-base reads always take
    the lane kernel."""
    ref = gen.fmi_reference(size, seed=seed, repeat_frac=0.15)
    codes, lens = gen.fmi_reads(ref, nreads, read_len=L, seed=seed + 50, sub_rate=0.02, n_rate=0.003)
    lens = lens.copy()
    lens[::53] = np.maximum(1, lens[::53] // 2)  # ragged lengths
    prefix = str(tmp_path / "ref")
    oi = fmi_util.OracleIndex(ref, path_out=prefix + ".bwt.2bit.64")
    if build:  # build_index() from the .pac must reproduce the same file
        pac_codes = ref
        pad = (-len(pac_codes)) % 4
        b = np.concatenate([pac_codes, np.zeros(pad, np.uint8)]).reshape(-1, 4)
        packed = (b[:, 0] << 6 | b[:, 1] << 4 | b[:, 2] << 2 | b[:, 3]).astype(np.uint8)
        tail = np.array([0, len(ref) % 4] if len(ref) % 4 == 0 else [len(ref) % 4], np.uint8)
        open(prefix + ".pac", "wb").write(packed.tobytes() + tail.tobytes())
        assert gen.read_pac(prefix + ".pac").tolist() == ref.tolist()
        os.rename(prefix + ".bwt.2bit.64", prefix + ".oracle.bwt.2bit.64")
    rb = tmp_path / "reads.bin"
    with open(rb, "wb") as f:
        f.write(np.array([nreads, L], np.int32).tobytes() + lens.astype(np.int32).tobytes() + codes.tobytes())
    out = tmp_path / "out.bin"
    args = [DRIVER, prefix, str(rb), str(batch), "19", str(threads), str(out)] + (["build"] if build else [])
    env = dict(os.environ)
    if tile:
        env["GB_FMI_TASK_TILE"] = tile
    if wave:
        env["GB_FMI_TASK_WAVE"] = wave
    r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    if build:
        assert open(prefix + ".bwt.2bit.64", "rb").read() == open(prefix + ".oracle.bwt.2bit.64", "rb").read()
        assert (np.fromfile(prefix + ".0123", np.uint8) == np.concatenate([ref, 3 - ref[::-1]])).all()
    bc0 = min(batch, nreads)
    got = _parse(out, batch, bc0)
    exp, ebc, epc = oi.run(codes, lens, batch_size=batch)
    ecalls = oi.bwt_calls()
    assert (_fields(got["sorted"]) == _fields(exp)).all()
    assert (got["batch_counts"] == ebc).all()
    assert (got["n123"].sum(axis=0) == epc).all()
    raw1, rid_after, intv_after, raw2, qpos_after, raw3 = _oracle_phases(oi, codes, lens, bc0, L, 19)
    assert (_fields(got["raw1"]) == _fields(raw1)).all()
    assert (got["rid_after"] == rid_after).all() and (got["intv_after"] == intv_after).all()
    assert (_fields(got["raw2"]) == _fields(raw2)).all() and (got["qpos_after"] == qpos_after).all()
    assert (_fields(got["raw3"]) == _fields(raw3)).all()
    assert got["calls"] == ecalls
    # SA methods
    n, count5, cp, sa, sent = fmi_util.read_index_file(prefix + ".bwt.2bit.64")
    assert got["n"] == n and got["sentinel"] == sent
    b0 = got["sorted"][:got["batch_counts"][0]]
    ec, _ = oi.sa_entries(b0, max_occ=500, mode=1)
    assert (got["coords"] == ec).all() and got["coord_id"] == len(ec)
    rows = (np.arange(64) * 7919) % n
    assert (got["compressed"] == oi.sa_lookup(rows, 0)).all()
    loaded = count5 + 1
    for r_, row in enumerate((np.arange(64) * 104729) % n):
        assert tuple(got["one_step"][r_]) == fmi_util.call_one_step(loaded, cp, sa, int(row))
    assert (got["raw_sa"] == sa[:16]).all()
    oi.close()
