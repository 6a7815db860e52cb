#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_fmi_gpu.py -x -q > gpurun_out/pytest_fmi.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_fmi.log; exit 1; }
tail -2 gpurun_out/pytest_fmi.log
timeout -k 10 600 python bench.py --only fmi --steps 3 --warmup 1 --fmi-reads 2000000 > gpurun_out/bench_sa.json 2> gpurun_out/bench_sa.err || { echo "bench failed"; tail -20 gpurun_out/bench_sa.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_sa.json'))['fmi']; print(json.dumps(d['sa_lookup'], indent=1)); print(d['value'])"
