#!/bin/bash
# LDS bank-conflict and VALU-busy counters per hot kernel (one rocprofv3 --pmc pass per bench leg,
# 7 SQ + 1 GRBM counters), summarised by tools/pmc_lds.py into gpurun_out/lds_${TAG}.json (tools/collect_checkpoint.py copies it to profiles/).
#   gpurun --timeout 900 -- 'bash tools/gpu_lds.sh r02'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
TAG=${1:-r02}
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-small --no-e2e --shard-of 0"
for leg in phmm chain bsw fmi; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/lds_${leg} -o run -- python3 bench.py --only $leg $ARGS > gpurun_out/lds_${leg}.json 2> gpurun_out/lds_${leg}.err || { echo "pmc $leg failed"; tail gpurun_out/lds_${leg}.err; exit 1; }
  echo "pmc $leg ok"
done
python3 tools/pmc_lds.py gpurun_out/lds_${TAG}.json gpurun_out/lds_phmm gpurun_out/lds_chain gpurun_out/lds_bsw gpurun_out/lds_fmi
