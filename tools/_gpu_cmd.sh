set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_fmi_gpu.py -x -q 2>&1 | tail -3
timeout -k 10 300 python tools/fmi_probe.py 2>&1 | grep -v amdgpu.ids
