#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/sa_probe.py > gpurun_out/sa_probe.log 2>&1; rc=$?; cat gpurun_out/sa_probe.log | tail -20; exit $rc
