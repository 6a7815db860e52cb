#!/bin/bash
# phmm f64-pass stacks: phmm GPU parity tests, smoke, then the full/shard probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_phmm_gpu.py tests/test_edges.py tests/test_dropin_threads.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/phmm_test.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/phmm_test.log; exit 1; }
tail -1 gpurun_out/phmm_test.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
PHMM_ROWS="default;GB_PHMM_F64_ROWS=2048;GB_PHMM_F64_ROWS=1024" timeout -k 10 300 python tools/phmm_shard_probe.py
