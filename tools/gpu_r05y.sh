#!/bin/bash
# round-5 GPU call y: phmm tests + the new default stack height on 'large' / 'small' and their shards
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05y}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_phmm_gpu.py -m gpu \
  > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
for of in 8 4; do
  PHMM_OF=$of timeout -k 10 200 python -u tools/phmm_shard_probe.py > gpurun_out/phmm_def_${of}_${T}.log 2>&1 \
    || { tail -20 gpurun_out/phmm_def_${of}_${T}.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/phmm_def_${of}_${T}.log
done
PHMM_KIND=small PHMM_BATCHES=256 timeout -k 10 200 python -u tools/phmm_shard_probe.py > gpurun_out/phmm_def_small_${T}.log 2>&1 \
  || { tail -20 gpurun_out/phmm_def_small_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_def_small_${T}.log
