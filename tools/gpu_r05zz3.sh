#!/bin/bash
# round-5 GPU call zz3: FMI_search class methods combined across calling threads -- the fmi task /
# class drop-in tests, then the class driver timed (threads 1..32) with combining on and off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zz3}
timeout -k 10 600 python -u -m pytest tests/test_fmi_dropin.py tests/test_fmi_gpu.py tests/test_fmi_getsmems_pin.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/fmi_class_tests_${T}.log 2>&1 || { tail -30 gpurun_out/fmi_class_tests_${T}.log; exit 1; }
tail -3 gpurun_out/fmi_class_tests_${T}.log
D=/tmp/fmi_class_${T}
N=${READS:-1000000}
timeout -k 10 300 python -u tools/fmi_class_prep.py $D $N > gpurun_out/fmi_class_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_class_${T}.log; exit 1; }
for comb in 1 0; do
  for th in ${THREADS:-4 8 16 32}; do
    GB_FMI_COMBINE=$comb timeout -k 10 200 tests/_build/fmi_class_driver $D/ref $D/reads.bin 512 19 $th $D/out_${comb}_${th}.bin 2> $D/err.txt > /dev/null || { tail -5 $D/err.txt; exit 1; }
    echo "combine $comb threads $th: $(grep 'SMEM phase' $D/err.txt) for $N reads" | tee -a gpurun_out/fmi_class_${T}.log
  done
done
# the combined runs' outputs equal the uncombined ones (the tests check them against the oracle)
for th in ${THREADS:-4 8 16 32}; do cmp $D/out_1_${th}.bin $D/out_0_${th}.bin && echo "threads $th: outputs identical" | tee -a gpurun_out/fmi_class_${T}.log; done
