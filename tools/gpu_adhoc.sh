#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04l
PROBE_VARIANTS="base:;wg12:GB_PHMM_F64_WG=12;wg17:GB_PHMM_F64_WG=17;wg20:GB_PHMM_F64_WG=20;wg24:GB_PHMM_F64_WG=24;wg32:GB_PHMM_F64_WG=32" \
  timeout -k 10 300 python3 tools/phmm_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/phmm_f64wg_$T.log || exit 1
