#!/bin/bash
# round-5 GPU call zze: bsw lane kernel with h = max3(M, e, f) forced (one 4.2-cycle op and one
# 2.5-cycle AND instead of two 4.2-cycle maxes per column) -- bsw GPU tests, then the 'large' set and
# its 1/8 shard against the previous build, alternating, on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zze}
timeout -k 10 600 python -u -m pytest tests/test_bsw.py tests/test_lds_poison.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/bsw_tests_${T}.log 2>&1 || { tail -30 gpurun_out/bsw_tests_${T}.log; exit 1; }
tail -2 gpurun_out/bsw_tests_${T}.log
for lib in ${AB_OLD:-tools/_ab/libgb_pre_max3.so} "" ${AB_OLD:-tools/_ab/libgb_pre_max3.so} ""; do
  BSW_LIB=$lib timeout -k 10 300 python -u tools/bsw_knob_probe.py > gpurun_out/bsw_ab_${T}.tmp 2>&1 || { tail -20 gpurun_out/bsw_ab_${T}.tmp; exit 1; }
  grep -v amdgpu.ids gpurun_out/bsw_ab_${T}.tmp | tee -a gpurun_out/bsw_ab_${T}.log
done
