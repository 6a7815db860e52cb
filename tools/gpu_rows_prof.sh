#!/bin/bash
# chain_rows vs chain_kernel on the 'large' set: rocprofv3 kernel-trace summary, then one SQ counter
# pass (waves, cycles, instruction mix, wait cycles), per kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export CHAIN_SETS=${PROF_SETS:-large}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rows_prof -o run -- python3 tools/chain_rows_probe.py > gpurun_out/rows_prof.log 2>&1 || { tail -20 gpurun_out/rows_prof.log; exit 1; }
cat gpurun_out/rows_prof.log
f=$(find gpurun_out/rows_prof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/rows_kernel_stats.csv; head -12 gpurun_out/rows_kernel_stats.csv | cut -c1-160
C=""
exit 0
f=$(find gpurun_out/rows_pmc -name '*counter_collection.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r['Kernel_Name'][:60]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    cnt[(k, r['Counter_Name'])] += 1
for k, d in acc.items():
    if 'chain' not in k and 'verify' not in k: continue
    n = cnt[(k, 'SQ_WAVES')]
    print(k, {c: round(v / max(n, 1), 1) for c, v in d.items()})
PY
