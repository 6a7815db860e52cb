#!/bin/bash
# r03zc: checkpoint after the tiled pointer jumping: all GPU tests, smoke, the bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_r03zc.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r03zc.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_r03zc.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 540 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03zc.json 2> gpurun_out/bench_r03zc.err; rc=$?; echo bench rc=$rc; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_r03zc.err; exit 1; }
