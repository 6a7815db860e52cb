#!/bin/bash
# round-5 GPU call q: bsw four-pairs-per-wave path: parity, small set + shard, large set
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05q}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bsw.py tests/test_lds_poison.py \
  tests/test_edges.py -m gpu > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
BSW_PAIRS=100000 BSW_CONFIGS="${BSW_CONFIGS:-;GB_BSW_GROUP=0;GB_BSW_TAIL=0.1;GB_BSW_TAIL=0.3;GB_BSW_TAIL=0.1+GB_BSW_GROUP=0}" timeout -k 10 300 python -u tools/bsw_knob_probe.py \
  > gpurun_out/bsw_small_${T}.log 2>&1 || { tail -20 gpurun_out/bsw_small_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bsw_small_${T}.log
BSW_CONFIGS=";GB_BSW_TAIL=0.05;GB_BSW_TAIL=0.2" timeout -k 10 400 python -u tools/bsw_knob_probe.py > gpurun_out/bsw_large_${T}.log 2>&1 \
  || { tail -20 gpurun_out/bsw_large_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bsw_large_${T}.log
