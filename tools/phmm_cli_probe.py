"""bin/phmm end to end on the 'large'-shaped job written as a .in file (PairHMMUnitTest.cpp's input):
its 'Kernel runtime' line (the reference's timed region: testcase construction, pack, upload,
kernels, results) under each environment setting of PHMM_CLI_CONFIGS (';'-separated, VAR=VALUE
joined by '+', '' = defaults), each run in a fresh process as the reference's CLI would be.
    PHMM_CLI_CONFIGS=";GB_PHMM_PIPE=1;GB_PHMM_PIPE=2" python tools/phmm_cli_probe.py
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import gen  # noqa: E402

batches = gen.phmm_dataset("large", int(os.environ.get("PHMM_BATCHES", "64")), seed=1)
cells = sum(b.cells() for b in batches)
exe = os.path.join(ROOT, "genomicsbench_palisade_amd", "bin", "phmm")
with tempfile.TemporaryDirectory() as td:
    f = os.path.join(td, "large.in")
    gen.write_phmm_file(f, batches)
    for cfg in os.environ.get("PHMM_CLI_CONFIGS", "").split(";"):
        env = {k: v for k, v in os.environ.items() if not k.startswith("GB_PHMM")}
        for kv in [c for c in cfg.split("+") if c]:
            k, v = kv.split("=", 1)
            env[k] = v
        for rep in range(2):
            r = subprocess.run([exe, "-f", f, "-t", "1"], capture_output=True, text=True, timeout=300, env=env)
            if r.returncode:
                print(f"[{cfg or 'default'}] failed: {r.stderr[-400:]}", flush=True)
                break
            kr = [float(ln.split(":")[1].split()[0]) for ln in r.stdout.splitlines() if "Kernel runtime" in ln][0]
            host = [ln for ln in r.stderr.splitlines() if ln.startswith("[phmm host]")]
            print(f"[{cfg or 'default':28s}] run {rep}: Kernel runtime {kr * 1e3:7.1f} ms ({cells / kr / 1e9:7.1f} GCUPS)"
                  + (f"  host: {'; '.join(h[12:] for h in host)}" if host else ""), flush=True)
