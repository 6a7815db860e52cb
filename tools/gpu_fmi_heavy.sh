#!/bin/bash
# fmi hand-over budget sweep (GB_FMI_HEAVY): the 'large' fmi leg and its 8 shard proxies per budget.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in ${BUDGETS:-2000 1000 1400 3000}; do
  GB_FMI_HEAVY=$b timeout -k 10 240 python bench.py --only fmi --steps 10 --warmup 2 --no-cpu-baseline --no-small --no-e2e > gpurun_out/fmi_heavy_$b.json 2> gpurun_out/fmi_heavy_$b.err || { echo "budget $b failed"; tail gpurun_out/fmi_heavy_$b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/fmi_heavy_$b.json'))['fmi']
print('budget $b:', d['value'], 'Mreads/s, shard worst', d['shard_proxy']['per_gpu_min'], 'ratio', round(d['shard_proxy']['ratio_min_vs_full'], 3))"
done
