#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_chain_bt.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/chain_bt_test.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/chain_bt_test.log; exit 1; }
tail -1 gpurun_out/chain_bt_test.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bt -o run -- python3 bench.py --only chain --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bt.json 2> gpurun_out/prof_bt.err || { echo "failed"; tail gpurun_out/prof_bt.err; exit 1; }
python -c "
import csv,json
for r in csv.DictReader(open('gpurun_out/prof_bt/run_kernel_stats.csv')):
    n=r['Name'].split('(')[0][-40:]
    if float(r['AverageNs'])>50000: print(f\"{n:42s} {float(r['AverageNs'])/1e6:8.3f} ms\")
d=json.loads(open('gpurun_out/prof_bt.json').read().strip().splitlines()[-1]); print('bt', d['chain']['backtrack']['value'], d['chain']['backtrack']['kernels_ms'])"
