#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_phmm_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/phmm_test.log 2>&1 || { echo "phmm tests failed"; tail -30 gpurun_out/phmm_test.log; exit 1; }
tail -1 gpurun_out/phmm_test.log


timeout -k 10 300 python tools/phmm_probe.py > gpurun_out/probe.log 2>&1; rc=$?; tail -20 gpurun_out/probe.log; exit $rc
