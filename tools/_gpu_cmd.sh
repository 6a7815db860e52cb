set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_fmi_gpu.py tests/test_chain.py -x -q -m gpu 2>&1 | tail -3
GB_FMI_WAVES_PER_CU=20 timeout -k 10 300 python tools/fmi_probe.py 2>&1 | grep -v amdgpu.ids
GB_CHAIN_PROF=1 timeout -k 10 300 python tools/chain_probe.py 2>&1 | grep -v amdgpu.ids | head -8
