#!/bin/bash
# PMC pass over the phmm leg (pair kernel, then GB_PHMM_SINGLE=1): issue/wait counters and the
# effective clock (GRBM_GUI_ACTIVE / duration).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_phmm_pair -o run -- python3 bench.py --only phmm --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_phmm_pair.json 2> gpurun_out/pmc_phmm_pair.err || { echo "pmc pair failed"; tail gpurun_out/pmc_phmm_pair.err; exit 1; }
GB_PHMM_SINGLE=1 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_phmm_single -o run -- python3 bench.py --only phmm --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_phmm_single.json 2> gpurun_out/pmc_phmm_single.err || { echo "pmc single failed"; tail gpurun_out/pmc_phmm_single.err; exit 1; }
echo done
