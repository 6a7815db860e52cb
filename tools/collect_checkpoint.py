"""Copy one GPU checkpoint's evidence from gpurun_out/ (tools/gpu_checkpoint.sh TAG ...) into profiles/:
  profiles/TAG_bench.json          the headline line the driver parses
  profiles/TAG_bench_detail.json   the full record (shard proxies, drop-ins, traffic detail, checks)
  profiles/TAG_kernel_stats.csv    rocprofv3 --kernel-trace --stats summary (prof stage)
  profiles/TAG_pmc.json            FETCH_SIZE / WRITE_SIZE per launch (prof stage, tools/pmc_summary.py)
  profiles/TAG_human_pmc.json      the same for the human-scale fmi leg
  profiles/TAG_lds.json            SQ LDS / VALU counters (lds stage)
    python tools/collect_checkpoint.py TAG
"""
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    g, p = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")
    done = []
    for src, dst in ((f"bench_{tag}.json", f"{tag}_bench.json"),
                     (f"bench_{tag}_detail.json", f"{tag}_bench_detail.json"),
                     (f"lds_{tag}.json", f"{tag}_lds.json")):
        if os.path.exists(os.path.join(g, src)):
            shutil.copy(os.path.join(g, src), os.path.join(p, dst))
            done.append(dst)
    ks = glob.glob(os.path.join(g, f"prof_{tag}", "**", "*kernel_stats.csv"), recursive=True)
    if ks:
        shutil.copy(ks[0], os.path.join(p, f"{tag}_kernel_stats.csv"))
        done.append(f"{tag}_kernel_stats.csv")
    for pre, dst in (("pmc", f"{tag}_pmc.json"), ("pmch", f"{tag}_human_pmc.json")):
        # the box's own summary (gpu_checkpoint.sh pmcsum) is stamped against the tree that was profiled:
        # copy it as it is. Re-summarising here would stamp whatever tree is checked out now.
        boxed = os.path.join(g, f"pmcsum_{dst}")
        if os.path.exists(boxed):
            shutil.copy(boxed, os.path.join(p, dst))
            done.append(dst)
            continue
        fd = glob.glob(os.path.join(g, f"{pre}_fetch_{tag}", "**", "run_counter_collection.csv"), recursive=True)
        wd = glob.glob(os.path.join(g, f"{pre}_write_{tag}", "**", "run_counter_collection.csv"), recursive=True)
        if fd and wd:
            # no box summary: summarise here, but stamp the digest of the commit named by GB_PMC_COMMIT
            # (the profiled code; default HEAD), not of the working tree
            env = dict(os.environ, GB_PMC_COMMIT=os.environ.get("GB_PMC_COMMIT", "HEAD"))
            subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), os.path.dirname(fd[0]),
                            os.path.dirname(wd[0]), os.path.join(p, dst)], check=True, stdout=subprocess.DEVNULL, env=env)
            done.append(dst + " (re-summarised, stamped at " + env["GB_PMC_COMMIT"] + ")")
    print("copied:", ", ".join(done) or "nothing")


if __name__ == "__main__":
    main()
