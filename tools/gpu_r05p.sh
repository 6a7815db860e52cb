#!/bin/bash
# round-5 GPU call p: phmm 1/8 shard step: f32 / f64 split and its kernel timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05p}
PHMM_ROWS="${PHMM_ROWS:-default}" timeout -k 10 200 python -u tools/phmm_shard_probe.py > gpurun_out/phmm_shard_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_shard_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_shard_${T}.log
rm -rf gpurun_out/phmm_shard_trace_${T}
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/phmm_shard_trace_${T} -- \
  python -u tools/phmm_shard_probe.py > gpurun_out/phmm_shard_trace_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_shard_trace_${T}.log; exit 1; }
python tools/kernel_timeline.py gpurun_out/phmm_shard_trace_${T} phmm_finalize > gpurun_out/phmm_shard_timeline_${T}.txt
cat gpurun_out/phmm_shard_timeline_${T}.txt
