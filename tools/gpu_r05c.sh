#!/bin/bash
# round-5 GPU call c: bsw routing (adaptive tail, segment kernel with prefetched target bases) parity
# and 'small'-set sweep, bin/phmm end-to-end variants, kernel traces of the 'small' chain shard
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05c}
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bsw.py tests/test_lds_poison.py -m gpu \
  > gpurun_out/pytest_${T}_bsw.log 2>&1 || { tail -40 gpurun_out/pytest_${T}_bsw.log; exit 1; }
tail -1 gpurun_out/pytest_${T}_bsw.log
BSW_PAIRS=100000 BSW_REBUILD=1 BSW_CONFIGS=";GB_BSW_TAIL=0.1;GB_BSW_TAIL=1;GB_BSW_TAIL=0+GB_BSW_SEG=1;GB_BSW_TAIL=0.02+GB_BSW_SEG=0.98;GB_BSW_TAIL=0.1+GB_BSW_SEG=0.9;GB_BSW_TAIL=0.3+GB_BSW_SEG=0.7;GB_BSW_TAIL=0.5+GB_BSW_SEG=0.5" \
  timeout -k 10 300 python -u tools/bsw_knob_probe.py > gpurun_out/bsw_small_${T}.log 2>&1 || { tail -20 gpurun_out/bsw_small_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bsw_small_${T}.log
BSW_CONFIGS=";GB_BSW_TAIL=0.02+GB_BSW_SEG=0.1" BSW_REBUILD=1 timeout -k 10 300 python -u tools/bsw_knob_probe.py > gpurun_out/bsw_large_${T}.log 2>&1 \
  || { tail -20 gpurun_out/bsw_large_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bsw_large_${T}.log
PHMM_CLI_CONFIGS=";GB_PHMM_PIPE=1;GB_PHMM_PIPE=2;GB_PHMM_HOSTPROF=1" timeout -k 10 300 python -u tools/phmm_cli_probe.py \
  > gpurun_out/phmm_cli_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cli_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cli_${T}.log | cut -c1-400
CHAIN_KIND=small timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_${T}_chain_small -o run -- \
  python3 tools/chain_shard_probe.py > gpurun_out/tl_${T}_chain_small.log 2>&1 || { tail -20 gpurun_out/tl_${T}_chain_small.log; exit 1; }
grep -v amdgpu.ids gpurun_out/tl_${T}_chain_small.log | tail -2
