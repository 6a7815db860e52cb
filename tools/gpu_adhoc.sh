#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04zb
A=genomicsbench_palisade_amd/lib/ab
timeout -k 10 200 python3 tools/phmm_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ilp_$T.log || exit 1
PHMM_LIB=$A/libgb_ilp_phmm.so timeout -k 10 200 python3 tools/phmm_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ilp_$T.log || exit 1
timeout -k 10 300 python3 tools/bsw_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ilp_$T.log || exit 1
BSW_LIB=$A/libgb_ilp_bsw.so timeout -k 10 300 python3 tools/bsw_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ilp_$T.log || exit 1
timeout -k 10 300 python3 tools/fmi_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ilp_$T.log || exit 1
FMI_LIB=$A/libgb_ilp_fmi.so timeout -k 10 300 python3 tools/fmi_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ilp_$T.log || exit 1
