#!/bin/bash
# round-5 GPU call zz7: FMI_search class driver under GPU_MAX_HW_QUEUES 4 (HIP's default) / 8 / 16:
# are 16 calling threads bound by 4 hardware queues serialising their launches?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zz7}
D=/tmp/fmi_class_${T}
N=${READS:-1000000}
timeout -k 10 300 python -u tools/fmi_class_prep.py $D $N > gpurun_out/fmi_class_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_class_${T}.log; exit 1; }
for q in 4 8 16; do
  for th in 16 32; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 tests/_build/fmi_class_driver $D/ref $D/reads.bin 512 19 $th $D/out_${q}_${th}.bin 2> $D/err.txt > /dev/null || { tail -5 $D/err.txt; exit 1; }
    echo "queues $q threads $th: $(grep 'SMEM phase' $D/err.txt) for $N reads" | tee -a gpurun_out/fmi_class_${T}.log
  done
done
cmp $D/out_4_16.bin $D/out_16_16.bin && echo "outputs identical" | tee -a gpurun_out/fmi_class_${T}.log
