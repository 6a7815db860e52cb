"""Summarise rocprofv3 runs of bench.py into profiles/<tag>_pmc.json: per hot kernel the mean duration and the HBM bytes per launch from FETCH_SIZE and
WRITE_SIZE (separate passes), KiB x 1024.

Correction, as MI355X_MICROARCH.md's HBM section prescribes ("calibrate on a known byte count in
your own access pattern"), from tools/probes/pmc_calib.hip (profiles/r01g_pmc_calib.txt): WRITE_SIZE
is exact; FETCH_SIZE counts scattered line-granular reads at their true bytes (random 64-B lines
1.03, one 8-B word per line 1.00 of the lines, 32-B halves of lines 2.02 = a whole line each) and
coalesced 16-B/lane streaming reads at 1/2 (the guide's gfx950 case). Each hot kernel's fetch is
scaled by the factor of its dominant read class (KERNEL_CLASS); the raw counter is kept beside it.

    python tools/pmc_summary.py gpurun_out/pmc_fetch_TAG gpurun_out/pmc_write_TAG profiles/TAG_pmc.json
"""
import collections
import csv
import json
import os
import sys

HOT = {"phmm_forward<float": "phmm_forward<float>", "phmm_forward<double": "phmm_forward<double>",
       "smem_search": "smem_search", "chain_kernel": "chain_kernel", "chain_rows": "chain_rows", "verify_lanes": "verify_lanes", "bsw_extend_kernel": "bsw_extend_kernel",
       "bsw_lane_kernel": "bsw_lane_kernel", "sa_walk": "sa_walk", "smem_heavy": "smem_heavy"}

FETCH_FACTOR = {"gather": 1.0, "stream": 2.0}
# dominant read class per kernel: scattered per-lane line requests ("gather") or coalesced
# per-wave streams ("stream")
KERNEL_CLASS = {
    "smem_search": "gather",            # Occ32 blocks at random rows
    "sa_walk": "gather",                # Occ32 blocks and sampled-SA words at random rows
    "bsw_lane_kernel": "gather",        # each lane reads its own pair's sequences
    "bsw_extend_kernel": "stream",      # one pair per wave, lanes over the query
    "phmm_forward<float>": "stream",    # one testcase per wave, coalesced read/haplotype bytes
    "phmm_forward<double>": "stream",
    "chain_kernel": "stream",           # anchors in 64-anchor coalesced blocks
    "chain_rows": "stream",             # anchors staged in 32-anchor coalesced blocks per half
    "verify_lanes": "stream",           # one split anchor per lane, contiguous anchors per wave
}


def name_of(r):
    for k, v in HOT.items():
        if k in r["Kernel_Name"].replace(", ", "<").replace("(", "<"):
            return v
    return None


def load(d):
    """Per kernel name: one (bytes, ms) entry per dispatch; the variants of a multi-launch step
    (bsw_lane_kernel<NCH>) are merged per step by summing consecutive dispatches of one step.
    Launches of one kernel over different workloads (e.g. a second, smaller leg) would be averaged
    together, so the profiling passes run the large legs only and main() refuses a kernel whose
    launches differ in size by more than 10 %."""
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        n = name_of(r)
        # a one-workgroup dispatch of a hot kernel is gb_phmm_init's warm-up launch (no work), not a step
        if n and r.get("Grid_Size") and r.get("Workgroup_Size") and int(r["Grid_Size"]) <= int(r["Workgroup_Size"]):
            continue
        if n:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
            out[n].append((float(r["Counter_Value"]) * 1024.0, dur, r["Kernel_Name"]))
    res = {}
    for n, v in out.items():
        variants = len(set(k for _, _, k in v))
        if variants > 1:  # group dispatches into steps of `variants` launches
            v = [(sum(b for b, _, _ in v[i:i + variants]), sum(t for _, t, _ in v[i:i + variants]))
                 for i in range(0, len(v) - variants + 1, variants)]
        else:
            v = [(b, t) for b, t, _ in v]
        res[n] = v
    return res


def commit_digest(commit, leg=None):
    """bench.source_digest over the kernel sources as they are in `commit` (git), not the working tree:
    the stamp of a summary made after the profiled code has moved on."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from bench import _leg_match, digest_of
    names = subprocess.run(["git", "-C", root, "ls-tree", "-r", "--name-only", commit], check=True,
                           capture_output=True, text=True).stdout.split()
    keep = [r for r in names if (r.startswith("genomicsbench_palisade_amd/csrc/")
                                 or (r.startswith("include/") and r.endswith(".h") and r.count("/") <= 2)
                                 or r == "Makefile") and _leg_match(r, leg)]
    return digest_of([(r, subprocess.run(["git", "-C", root, "show", f"{commit}:{r}"], check=True,
                                         capture_output=True).stdout) for r in keep])


def main():
    fetch, write, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    f, w = load(fetch), load(write)
    res = {}
    for k in sorted(set(f) | set(w)):
        # the first launch of a leg is its checked pass (cold pages and caches): dropped when the
        # pass holds at least three launches of the kernel
        fl, wl = f.get(k, []), w.get(k, [])
        fl, wl = (fl[1:] if len(fl) >= 3 else fl), (wl[1:] if len(wl) >= 3 else wl)
        fb = [v for v, _ in fl]
        wb = [v for v, _ in wl]
        ms = [d for _, d in fl] + [d for _, d in wl]
        for vals in (fb, wb):
            if vals and max(vals) > 1.1 * min(vals):
                sys.exit(f"{k}: launches of different sizes ({min(vals):.3g} .. {max(vals):.3g} B); profile one leg")
        raw = sum(fb) / max(len(fb), 1)
        cls = KERNEL_CLASS.get(k, "gather")
        res[k] = {"launches": len(fb), "fetch_bytes": raw * FETCH_FACTOR[cls], "fetch_bytes_raw": raw,
                  "fetch_class": cls, "fetch_factor": FETCH_FACTOR[cls],
                  "write_bytes": sum(wb) / max(len(wb), 1), "mean_ms_under_pmc": sum(ms) / max(len(ms), 1)}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import LEG_SOURCES, source_digest
    commit = os.environ.get("GB_PMC_COMMIT")
    dig = (lambda leg=None: commit_digest(commit, leg)) if commit else source_digest
    res["_code"] = dig()  # bench.py marks traffic from other kernel code "stale"
    res["_code_legs"] = {leg: dig(leg) for leg in LEG_SOURCES}
    if commit:
        res["_code_commit"] = commit
    res["_note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), KiB x 1024 per launch; fetch "
                    "scaled by the calibrated factor of the kernel's read class (tools/probes/pmc_calib.hip, "
                    "profiles/r01g_pmc_calib.txt), write exact")
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
