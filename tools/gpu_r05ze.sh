#!/bin/bash
# round-5 GPU call ze: phmm f64 regrouping: parity + A/B on 'large', its shards and 'small'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05ze}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_phmm_gpu.py -m gpu \
  > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
R="${ROWS:-default;GB_PHMM_F64_REGROUP=0;GB_PHMM_F64_ROWS=256;GB_PHMM_F64_ROWS=2048}"
PHMM_ROWS="$R" timeout -k 10 300 python -u tools/phmm_shard_probe.py > gpurun_out/phmm_rg_${T}.log 2>&1 \
  || { tail -20 gpurun_out/phmm_rg_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_rg_${T}.log
PHMM_KIND=small PHMM_BATCHES=256 PHMM_ROWS="$R" timeout -k 10 300 python -u tools/phmm_shard_probe.py > gpurun_out/phmm_rg_small_${T}.log 2>&1 \
  || { tail -20 gpurun_out/phmm_rg_small_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_rg_small_${T}.log
