#!/bin/bash
# chain_rows development run: chain parity tests, then the rows A/B probe.
#   gpurun --timeout 900 -- 'bash tools/gpu_rows.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_chain.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/rows_test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/rows_test.log; exit 1; }
tail -3 gpurun_out/rows_test.log
timeout -k 10 300 python -u tools/chain_rows_probe.py > gpurun_out/rows_probe.log 2>&1 || { tail -20 gpurun_out/rows_probe.log; exit 1; }
cat gpurun_out/rows_probe.log
