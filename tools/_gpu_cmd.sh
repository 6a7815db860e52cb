#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --only fmi --no-cpu-baseline > gpurun_out/fmi_bench.json 2> gpurun_out/fmi_bench.err || { echo "bench failed"; tail -20 gpurun_out/fmi_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/fmi_bench.json').read().strip().splitlines()[-1]); f=d['fmi']
print('fmi', f['value'], f['unit'], f['kernels_ms'], round(f['roofline']['frac'],3)); s=f.get('sa_lookup') or {}
print('sa', s.get('value'), s.get('kernels_ms'))"
