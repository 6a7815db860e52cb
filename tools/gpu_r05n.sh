#!/bin/bash
# round-5 GPU call n: bin/phmm with huge-page testcase arrays, chunk counts, and its kernel timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05n}
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>&1 || true
PHMM_CLI_CONFIGS=";GB_PHMM_HOSTPROF=1;GB_PHMM_PIPE=2;GB_PHMM_PIPE=3;GB_PHMM_PIPE=6" \
  timeout -k 10 300 python -u tools/phmm_cli_probe.py > gpurun_out/phmm_cli_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cli_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cli_${T}.log | cut -c1-600
timeout -k 10 120 python tools/phmm_write_in.py /tmp/large.in
rm -rf gpurun_out/phmm_cli_trace_${T}
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/phmm_cli_trace_${T} -- \
  genomicsbench_palisade_amd/bin/phmm -f /tmp/large.in -t 1 > gpurun_out/phmm_cli_trace_${T}.log 2>&1 \
  || { tail -20 gpurun_out/phmm_cli_trace_${T}.log; exit 1; }
grep "Kernel runtime" gpurun_out/phmm_cli_trace_${T}.log
python tools/kernel_timeline.py gpurun_out/phmm_cli_trace_${T} all > gpurun_out/phmm_cli_timeline_${T}.txt
cat gpurun_out/phmm_cli_timeline_${T}.txt
