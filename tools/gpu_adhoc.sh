#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04g
GB_FMI_PLAYOUT=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fmi_gpu.py > gpurun_out/fmi_tests_playout_$T.log 2>&1 || { tail -30 gpurun_out/fmi_tests_playout_$T.log; exit 1; }
tail -2 gpurun_out/fmi_tests_playout_$T.log
FMI_CONFIGS=";GB_FMI_PLAYOUT=1;GB_FMI_TOP=8+GB_FMI_WAVES_PER_CU=11+GB_FMI_PLAYOUT=1;GB_FMI_TOP=0+GB_FMI_WAVES_PER_CU=16+GB_FMI_PLAYOUT=1" \
  timeout -k 10 300 python3 tools/fmi_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/fmi_knobs_$T.log || exit 1
for C in WRITE_SIZE FETCH_SIZE; do
  FMI_PROBE_READS=2000000 FMI_CONFIGS=";GB_FMI_PLAYOUT=1" timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_playout_${C}_$T -o run -- python3 tools/fmi_knob_probe.py > gpurun_out/pmc_playout_${C}_$T.log 2>&1 || { tail -20 gpurun_out/pmc_playout_${C}_$T.log; exit 1; }
  d=$(dirname "$(find gpurun_out/pmc_playout_${C}_$T -name run_counter_collection.csv | head -1)")
  python3 tools/pmc_kernel.py "$d" smem_search | tee gpurun_out/pmc_playout_${C}_$T.txt
done
