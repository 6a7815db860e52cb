#!/bin/bash
# scratch GPU session, edited per experiment (the last one: an A/B of two libgb builds with
# tools/bsw_knob_probe.py); the checkpoints use tools/gpu_checkpoint.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-adhoc}
for rep in 1 2; do
  timeout -k 10 300 python3 tools/bsw_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/bsw_ab_$T.log || exit 1
  if [ -n "$BSW_LIB_B" ]; then
    BSW_LIB=$BSW_LIB_B timeout -k 10 300 python3 tools/bsw_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/bsw_ab_$T.log || exit 1
  fi
done
