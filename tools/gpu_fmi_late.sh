#!/bin/bash
# fmi late-read budget sweep (GB_FMI_HEAVY_LATE, the last round of reads): fmi leg + 8 shard proxies.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fmi_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/fmi_test.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fmi_test.log; exit 1; }
tail -1 gpurun_out/fmi_test.log
for b in ${LATES:-0 1000 500 250}; do
  GB_FMI_HEAVY_LATE=$b timeout -k 10 240 python bench.py --only fmi --steps 10 --warmup 2 --no-cpu-baseline --no-small --no-e2e > gpurun_out/fmi_late_$b.json 2> gpurun_out/fmi_late_$b.err || { echo "late $b failed"; tail gpurun_out/fmi_late_$b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/fmi_late_$b.json'))['fmi']
print('late $b:', d['value'], 'Mreads/s, shard worst', d['shard_proxy']['per_gpu_min'], 'ratio', round(d['shard_proxy']['ratio_min_vs_full'], 3))"
done
