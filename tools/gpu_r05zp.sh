#!/bin/bash
# round-5 GPU call zp: phmm f64 kernel register budget (waves per SIMD 4 default / 5 / 6) A/B builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zp}
for lib in genomicsbench_palisade_amd/lib/libgb.so tools/_ab/libgb_w5.so tools/_ab/libgb_w6.so genomicsbench_palisade_amd/lib/libgb.so tools/_ab/libgb_w5.so; do
  echo "== $lib"
  PHMM_LIB=$lib timeout -k 10 200 python -u tools/phmm_shard_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/phmm_f64w_${T}.log
cat gpurun_out/phmm_f64w_${T}.log
