#!/bin/bash
# round-5 GPU call zm: phmm step unroll (4 default / 8 / 2) A/B builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zm}
for lib in genomicsbench_palisade_amd/lib/libgb.so tools/_ab/libgb_u8.so tools/_ab/libgb_u2.so genomicsbench_palisade_amd/lib/libgb.so; do
  echo "== $lib"
  PHMM_LIB=$lib timeout -k 10 200 python -u tools/phmm_shard_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/phmm_unroll_${T}.log
cat gpurun_out/phmm_unroll_${T}.log
