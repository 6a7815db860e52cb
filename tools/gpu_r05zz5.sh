#!/bin/bash
# round-5 GPU call zz5: FMI_search class driver (pinned / packed copies, per-launch wave LDS), 8 / 16 / 32
# threads, twice; the class tests first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zz5}
timeout -k 10 600 python -u -m pytest tests/test_fmi_dropin.py tests/test_fmi_gpu.py tests/test_fmi_getsmems_pin.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/fmi_class_tests_${T}.log 2>&1 || { tail -30 gpurun_out/fmi_class_tests_${T}.log; exit 1; }
tail -2 gpurun_out/fmi_class_tests_${T}.log
D=/tmp/fmi_class_${T}
N=${READS:-1000000}
timeout -k 10 300 python -u tools/fmi_class_prep.py $D $N > gpurun_out/fmi_class_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_class_${T}.log; exit 1; }
for ll in 0 0; do
  for th in ${THREADS:-8 16 32}; do
    timeout -k 10 200 tests/_build/fmi_class_driver $D/ref $D/reads.bin 512 19 $th $D/out_${ll}_${th}.bin 2> $D/err.txt > /dev/null || { tail -5 $D/err.txt; exit 1; }
    echo "run $ll threads $th: $(grep 'SMEM phase' $D/err.txt) for $N reads" | tee -a gpurun_out/fmi_class_${T}.log
  done
done

