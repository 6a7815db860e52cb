#!/bin/bash
# round-5 GPU call b: bsw segment kernel parity, phmm two-row register budgets A/B, the stale-LDS A/B
# against the pre-1da81ef chain_rows build, phmm drop-in end to end (pipelined), 'small'-set knob
# sweeps (bsw tail / segment routing, fmi heavy-read budget)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05b}
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bsw.py -m gpu \
  > gpurun_out/pytest_${T}_bsw.log 2>&1 || { tail -40 gpurun_out/pytest_${T}_bsw.log; exit 1; }
tail -1 gpurun_out/pytest_${T}_bsw.log
PHMM_ROWS="GB_PHMM_RPL=1;GB_PHMM_RPL=2;GB_PHMM_W2=6;GB_PHMM_W2=8;GB_PHMM_RPL=1" timeout -k 10 300 python -u tools/phmm_shard_probe.py \
  > gpurun_out/phmm_ab_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_ab_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_ab_${T}.log
GB_LIB=tools/_ab/libgb_pre1da81ef.so timeout -k 10 200 python -u tools/lds_poison_ab.py > gpurun_out/lds_ab_${T}.log 2>&1 \
  || { tail -20 gpurun_out/lds_ab_${T}.log; exit 1; }
timeout -k 10 200 python -u tools/lds_poison_ab.py >> gpurun_out/lds_ab_${T}.log 2>&1 || { tail -20 gpurun_out/lds_ab_${T}.log; exit 1; }
grep -E "wrong runs" gpurun_out/lds_ab_${T}.log
BSW_PAIRS=100000 BSW_REBUILD=1 BSW_CONFIGS=";GB_BSW_TAIL=0;GB_BSW_TAIL=0.3;GB_BSW_TAIL=1;GB_BSW_SEG=0.3;GB_BSW_SEG=0.6;GB_BSW_TAIL=0+GB_BSW_SEG=1;GB_BSW_TAIL=0.05+GB_BSW_SEG=0.5;GB_BSW_TAIL=0.02+GB_BSW_SEG=0.98" \
  timeout -k 10 300 python -u tools/bsw_knob_probe.py > gpurun_out/bsw_small_${T}.log 2>&1 || { tail -20 gpurun_out/bsw_small_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bsw_small_${T}.log
FMI_PROBE_READS=1000000 FMI_CONFIGS=";GB_FMI_HEAVY=1000;GB_FMI_HEAVY=500;GB_FMI_HEAVY=250;GB_FMI_HEAVY=120;GB_FMI_WAVES_PER_CU=8;GB_FMI_WAVES_PER_CU=24" \
  timeout -k 10 400 python -u tools/fmi_knob_probe.py > gpurun_out/fmi_small_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_small_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fmi_small_${T}.log
timeout -k 10 400 python -u bench.py --only phmm --no-small --shard-of 0 --steps 10 --warmup 3 --no-cpu-baseline \
  --detail-out gpurun_out/bench_${T}_phmm_detail.json > gpurun_out/bench_${T}_phmm.json 2> gpurun_out/bench_${T}_phmm.err \
  || { tail -20 gpurun_out/bench_${T}_phmm.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_phmm_detail.json')); print(d['value'], d['kernels_ms']); print(json.dumps(d['dropin_e2e'])[:1500])"
