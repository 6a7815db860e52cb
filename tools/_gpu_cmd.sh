#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fmi_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fmi_test.log 2>&1 || { echo "fmi tests failed"; tail -30 gpurun_out/fmi_test.log; exit 1; }
tail -1 gpurun_out/fmi_test.log
FMI_PROBE_FLAGS=0,4 timeout -k 10 300 python tools/fmi_probe.py > gpurun_out/fmi_probe.log 2>&1; rc=$?; tail -2 gpurun_out/fmi_probe.log; exit $rc
