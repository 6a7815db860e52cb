#!/bin/bash
# round-5 GPU call zz4: FMI_search class driver, combined calls on the lane-per-task kernels
# (GB_FMI_TASK_WAVE=0) against the wave-per-task ones, 16 and 32 threads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zz4}
D=/tmp/fmi_class_${T}
N=${READS:-1000000}
timeout -k 10 300 python -u tools/fmi_class_prep.py $D $N > gpurun_out/fmi_class_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_class_${T}.log; exit 1; }
for cfg in "1 1" "1 0" "0 0" "0 1"; do
  set -- $cfg
  for th in ${THREADS:-16 32 64}; do
    GB_FMI_COMBINE=$1 GB_FMI_TASK_WAVE=$2 timeout -k 10 200 tests/_build/fmi_class_driver $D/ref $D/reads.bin 512 19 $th $D/out.bin 2> $D/err.txt > /dev/null || { tail -5 $D/err.txt; exit 1; }
    echo "combine $1 wave $2 threads $th: $(grep 'SMEM phase' $D/err.txt) for $N reads" | tee -a gpurun_out/fmi_class_${T}.log
  done
done
