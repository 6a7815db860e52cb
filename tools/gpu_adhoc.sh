#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04i
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bsw.py -m gpu > gpurun_out/bsw_tests_$T.log 2>&1 || { tail -30 gpurun_out/bsw_tests_$T.log; exit 1; }
tail -2 gpurun_out/bsw_tests_$T.log
BSW_CONFIGS=";GB_BSW_REFILL=1,64;GB_BSW_REFILL=2,8;GB_BSW_REFILL=4,1;GB_BSW_REFILL=4,16;GB_BSW_REFILL=8,8;GB_BSW_REFILL=8,16;GB_BSW_REFILL=16,16;GB_BSW_REFILL=16,32" \
  timeout -k 10 400 python3 tools/bsw_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bsw_knobs_$T.log || exit 1
