#!/bin/bash
# phmm-only GPU iteration: parity tests, then the phmm bench leg with the pair kernel and with the
# one-testcase-per-wave kernel (GB_PHMM_SINGLE=1), then kernel stats. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_phmm_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/phmm_test.log 2>&1 || { echo "phmm tests failed"; tail -30 gpurun_out/phmm_test.log; exit 1; }
tail -1 gpurun_out/phmm_test.log
timeout -k 10 300 python bench.py --only phmm --no-cpu-baseline > gpurun_out/phmm_pair.json 2> gpurun_out/phmm_pair.err || { echo "bench failed"; tail -20 gpurun_out/phmm_pair.err; exit 1; }
GB_PHMM_SINGLE=1 timeout -k 10 300 python bench.py --only phmm --no-cpu-baseline > gpurun_out/phmm_single.json 2> gpurun_out/phmm_single.err || { echo "bench single failed"; tail -20 gpurun_out/phmm_single.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_phmm -o run -- python3 bench.py --only phmm --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_phmm.json 2> gpurun_out/prof_phmm.err || { echo "rocprof failed"; tail -20 gpurun_out/prof_phmm.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/phmm_pair.json", "gpurun_out/phmm_single.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["unit"], d["kernels_ms"], round(d["roofline"]["frac"], 3))
PY
grep phmm gpurun_out/prof_phmm/run_kernel_stats.csv | cut -c1-160
