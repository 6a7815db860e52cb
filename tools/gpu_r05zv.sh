#!/bin/bash
# round-5 GPU call zv: chain 'small' 1/8 shard step timeline (current code)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zv}
rm -rf gpurun_out/chain_sshard_trace_${T}
CHAIN_KIND=small timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chain_sshard_trace_${T} -- \
  python -u tools/chain_shard_probe.py > gpurun_out/chain_sshard_trace_${T}.log 2>&1 || { tail -20 gpurun_out/chain_sshard_trace_${T}.log; exit 1; }
python tools/kernel_timeline.py gpurun_out/chain_sshard_trace_${T} chain_rows > gpurun_out/chain_sshard_timeline_${T}.txt
cat gpurun_out/chain_sshard_timeline_${T}.txt
