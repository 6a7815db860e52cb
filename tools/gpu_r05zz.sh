#!/bin/bash
# round-5 GPU call zz: the FMI_search class drop-in (fmi.cpp's batch loop, 512-read batches from
# 16 threads) timed and kernel-traced
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zz}
D=/tmp/fmi_class_${T}
N=${READS:-1000000}
timeout -k 10 300 python -u tools/fmi_class_prep.py $D $N > gpurun_out/fmi_class_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_class_${T}.log; exit 1; }
for th in ${THREADS:-16}; do
  timeout -k 10 200 tests/_build/fmi_class_driver $D/ref $D/reads.bin 512 19 $th $D/out.bin 2> $D/err.txt > /dev/null || { tail -5 $D/err.txt; exit 1; }
  echo "threads $th: $(grep 'SMEM phase' $D/err.txt) for $N reads" | tee -a gpurun_out/fmi_class_${T}.log
done
rm -rf gpurun_out/fmi_class_trace_${T}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fmi_class_trace_${T} -- \
  tests/_build/fmi_class_driver $D/ref $D/reads.bin 512 19 ${PROF_THREADS:-16} $D/out.bin 2> gpurun_out/fmi_class_prof_err_${T}.txt > /dev/null || { tail -5 gpurun_out/fmi_class_prof_err_${T}.txt; exit 1; }
grep 'SMEM phase' gpurun_out/fmi_class_prof_err_${T}.txt | tee -a gpurun_out/fmi_class_${T}.log
f=$(find gpurun_out/fmi_class_trace_${T} -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -12 | tee -a gpurun_out/fmi_class_${T}.log
python tools/kernel_timeline.py gpurun_out/fmi_class_trace_${T} all > gpurun_out/fmi_class_timeline_${T}.txt 2>&1 || true
tail -3 gpurun_out/fmi_class_timeline_${T}.txt
find gpurun_out/fmi_class_trace_${T} -name '*kernel_trace.csv' -delete
