#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04zd
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bsw.py tests/test_edges.py -m gpu > gpurun_out/bsw_tests_$T.log 2>&1 || { tail -30 gpurun_out/bsw_tests_$T.log; exit 1; }
tail -2 gpurun_out/bsw_tests_$T.log
for rep in 1 2; do
  BSW_LIB=genomicsbench_palisade_amd/lib/ab/libgb_old.so timeout -k 10 300 python3 tools/bsw_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/bsw_ab_$T.log || exit 1
  timeout -k 10 300 python3 tools/bsw_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/bsw_ab_$T.log || exit 1
done
