#!/bin/bash
# chain backtrack: parity tests, the timing probe, and a kernel-trace summary of the probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_chain_bt.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/bt_test.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/bt_test.log; exit 1; }
tail -1 gpurun_out/bt_test.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bt_prof -o run -- python3 tools/chain_bt_probe.py > gpurun_out/bt_probe.log 2>&1 || { tail -20 gpurun_out/bt_probe.log; exit 1; }
grep backtrack gpurun_out/bt_probe.log
f=$(find gpurun_out/bt_prof -name '*kernel_stats.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
