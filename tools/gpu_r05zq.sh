#!/bin/bash
# round-5 GPU call zq: fmi human-scale index under prev-head sizes 4 / 5 / 6
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zq}
for top in 5 4 6; do
  GB_FMI_TOP=$top timeout -k 10 300 python -u bench.py --only fmi_human --steps 5 --warmup 2 --fmi-human-check 2000 \
    > gpurun_out/human_${top}_${T}.json 2> gpurun_out/human_${top}_${T}.err || { tail -20 gpurun_out/human_${top}_${T}.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); h=d.get('fmi',{}).get('human') or d; print(sys.argv[2], h.get('value'), h.get('ms_per_step'))" gpurun_out/human_${top}_${T}.json top=$top
done
