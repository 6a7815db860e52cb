#!/bin/bash
# round-5 GPU call zzh: phmm f32 early exit (GB_PHMM_EXIT=1, off by default) -- the phmm GPU tests on
# the default path, then default vs exit on the new build and the previous build's default, one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zzh}
timeout -k 10 600 python -u -m pytest tests/test_phmm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/phmm_tests_${T}.log 2>&1 || { tail -30 gpurun_out/phmm_tests_${T}.log; exit 1; }
tail -2 gpurun_out/phmm_tests_${T}.log
PHMM_LIB=tools/_ab/libgb_pre_exit.so PHMM_CONFIGS="" timeout -k 10 300 python -u tools/phmm_exit_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/phmm_exit_${T}.log
timeout -k 10 300 python -u tools/phmm_exit_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/phmm_exit_${T}.log
