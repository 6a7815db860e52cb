#!/bin/bash
# chain_rows probe with wave priorities on/off and segment lengths (GB_CHAIN_SPLIT) swept.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export CHAIN_SPLITS="${SPLITS:-2048,256;1024,256}"
timeout -k 10 300 python -u tools/chain_rows_probe.py > gpurun_out/rows_probe.log 2>&1 || { tail -20 gpurun_out/rows_probe.log; exit 1; }
cat gpurun_out/rows_probe.log
GB_CHAIN_PRIO=0 CHAIN_SPLITS= CHAIN_SETS=large,small timeout -k 10 300 python -u tools/chain_rows_probe.py > gpurun_out/rows_probe0.log 2>&1 || { tail -20 gpurun_out/rows_probe0.log; exit 1; }
echo "no priorities:"; cat gpurun_out/rows_probe0.log
GB_CHAIN_SPREAD=0 CHAIN_SPLITS= CHAIN_SETS=large,small,"large 1/8" timeout -k 10 300 python -u tools/chain_rows_probe.py > gpurun_out/rows_probe_ns.log 2>&1 || { tail -20 gpurun_out/rows_probe_ns.log; exit 1; }
echo "no spreading:"; cat gpurun_out/rows_probe_ns.log
