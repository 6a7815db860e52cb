#!/bin/bash
# fmi smem_search sensitivity to resident waves per CU (GB_FMI_WAVES_PER_CU), large set, one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${WAVES:-8 12 16}; do
  GB_FMI_WAVES_PER_CU=$w timeout -k 10 300 python bench.py --only fmi --steps 3 --warmup 1 --no-cpu-baseline --no-small --no-e2e > gpurun_out/fmi_w$w.json 2> gpurun_out/fmi_w$w.err || { tail gpurun_out/fmi_w$w.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/fmi_w$w.json').read().strip().splitlines()[-1])['fmi']; print('waves/CU $w', d['value'], 'Mreads/s', round(d['kernels_ms']['smem_search'],1), 'ms')"
done
