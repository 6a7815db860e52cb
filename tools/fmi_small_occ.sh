#!/bin/bash
# fmi 'small' (1 M reads) and 'large' search rate against resident waves per CU (GB_FMI_WAVES_PER_CU):
# with ~4 reads per lane at 16 waves/CU the small set's time is set by each wave's slowest lane.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${WAVES:-6 8 12 16}; do
  GB_FMI_WAVES_PER_CU=$w timeout -k 10 300 python bench.py --only fmi --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/fmi_s_w$w.json 2> gpurun_out/fmi_s_w$w.err || { tail gpurun_out/fmi_s_w$w.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/fmi_s_w$w.json').read().strip().splitlines()[-1]); print('waves/CU $w large', d['fmi']['value'], 'small', d['small']['fmi']['value'], 'Mreads/s')"
done
