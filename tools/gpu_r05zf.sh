#!/bin/bash
# round-5 GPU call zf: computelikelihoodsboth per batch (the reference's call pattern)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zf}
PHMM_PERBATCH_CONFIGS="${CFG:-;GB_PHMM_PACK_MIN=8192;GB_PHMM_PACK_MIN=16384;GB_PHMM_PIPE=2;GB_PHMM_PACK_MIN=8192+GB_PHMM_PIPE=2}" \
  timeout -k 10 300 python -u tools/phmm_perbatch_probe.py > gpurun_out/phmm_perbatch_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_perbatch_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_perbatch_${T}.log
GB_PHMM_HOSTPROF=1 PHMM_PERBATCH_CONFIGS="GB_PHMM_HOSTPROF=1" timeout -k 10 300 python -u tools/phmm_perbatch_probe.py > gpurun_out/phmm_perbatch_prof_${T}.log 2>&1 || true
grep -c "phmm host" gpurun_out/phmm_perbatch_prof_${T}.log || true
