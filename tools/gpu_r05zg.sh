#!/bin/bash
# round-5 GPU call zg: phmm tests, per-batch calls and the job / shard defaults after the small-call changes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zg}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_phmm_gpu.py -m gpu \
  > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
PHMM_PERBATCH_CONFIGS="${CFG:-;GB_PHMM_PACK_MIN=65536;GB_PHMM_STACK_ROWS=512}" timeout -k 10 300 python -u tools/phmm_perbatch_probe.py \
  > gpurun_out/phmm_perbatch_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_perbatch_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_perbatch_${T}.log
timeout -k 10 200 python -u tools/phmm_shard_probe.py > gpurun_out/phmm_def_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_def_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_def_${T}.log
PHMM_KIND=small PHMM_BATCHES=256 timeout -k 10 200 python -u tools/phmm_shard_probe.py > gpurun_out/phmm_def_small_${T}.log 2>&1 \
  || { tail -20 gpurun_out/phmm_def_small_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_def_small_${T}.log
PHMM_CLI_CONFIGS=";" timeout -k 10 300 python -u tools/phmm_cli_probe.py > gpurun_out/phmm_cli_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cli_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cli_${T}.log | cut -c1-200
