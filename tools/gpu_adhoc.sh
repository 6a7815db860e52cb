#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04u
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bsw.py -m gpu > gpurun_out/bsw_tests_$T.log 2>&1 || { tail -30 gpurun_out/bsw_tests_$T.log; exit 1; }
tail -2 gpurun_out/bsw_tests_$T.log
timeout -k 10 400 python3 bench.py --only bsw --steps 5 --warmup 2 --no-cpu-baseline --shard-of 0 --detail-out gpurun_out/bench_bsw_$T.json > gpurun_out/bench_bsw_$T.line 2> gpurun_out/bench_bsw_$T.err || { tail gpurun_out/bench_bsw_$T.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_bsw_$T.json'))['bsw']
print(d['value'], {k:(v.get('value'), v.get('seconds')) for k,v in d['dropin_e2e'].items()})"
BSW_REBUILD=1 BSW_CONFIGS=";GB_BSW_TCAP=20;GB_BSW_TCAP=40;GB_BSW_TCAP=70;GB_BSW_TCAP=40+GB_BSW_H0STEP=5" timeout -k 10 400 python3 tools/bsw_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/bsw_key_$T.log || exit 1
