#!/bin/bash
# round-5 GPU call x: phmm stack height on the 'small' job (256 batches) and its 1/8 shard
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05x}
PHMM_KIND=small PHMM_BATCHES=256 PHMM_ROWS="default;256;512;1024;2048" timeout -k 10 200 python -u tools/phmm_shard_probe.py \
  > gpurun_out/phmm_rows_small_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_rows_small_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_rows_small_${T}.log
