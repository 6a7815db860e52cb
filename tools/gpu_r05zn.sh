#!/bin/bash
# round-5 GPU call zn: kernel timeline of per-batch computelikelihoodsboth calls
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zn}
rm -rf gpurun_out/perbatch_trace_${T}
PHMM_PERBATCH_CONFIGS="" timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/perbatch_trace_${T} -- \
  python -u tools/phmm_perbatch_probe.py > gpurun_out/perbatch_trace_${T}.log 2>&1 || { tail -20 gpurun_out/perbatch_trace_${T}.log; exit 1; }
python tools/kernel_timeline.py gpurun_out/perbatch_trace_${T} all | tail -60 > gpurun_out/perbatch_timeline_${T}.txt
cat gpurun_out/perbatch_timeline_${T}.txt
ls gpurun_out/perbatch_trace_${T}/*/ | head
