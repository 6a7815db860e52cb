#!/bin/bash
# round-5 GPU call zzd: fmi heavy pass with reads taken one at a time and per-launch LDS -- the fmi
# GPU tests, then the 10 M-read set and its 1/8 shard against the previous build (same box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zzd}
timeout -k 10 600 python -u -m pytest tests/test_fmi_gpu.py tests/test_lds_poison.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/fmi_tests_${T}.log 2>&1 || { tail -30 gpurun_out/fmi_tests_${T}.log; exit 1; }
tail -2 gpurun_out/fmi_tests_${T}.log
for lib in tools/_ab/libgb_pre_heavy.so ""; do
  FMI_LIB=$lib FMI_CONFIGS="${CFG:-;GB_FMI_HEAVY_WAVES=20}" timeout -k 10 400 python -u tools/fmi_knob_probe.py \
    > gpurun_out/fmi_knobs_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_knobs_${T}.log; exit 1; }
  echo "lib ${lib:-current}" | tee -a gpurun_out/fmi_heavy_${T}.log
  grep -v amdgpu.ids gpurun_out/fmi_knobs_${T}.log | tee -a gpurun_out/fmi_heavy_${T}.log
done
