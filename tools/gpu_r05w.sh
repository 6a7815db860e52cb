#!/bin/bash
# round-5 GPU call w: phmm stack height on 1/2, 1/4 and 1/8 shards
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05w}
for of in 2 4 8; do
  PHMM_OF=$of PHMM_ROWS="default;512;1024;2048" timeout -k 10 200 python -u tools/phmm_shard_probe.py > gpurun_out/phmm_rows_${of}_${T}.log 2>&1 \
    || { tail -20 gpurun_out/phmm_rows_${of}_${T}.log; exit 1; }
  grep shard gpurun_out/phmm_rows_${of}_${T}.log
done
