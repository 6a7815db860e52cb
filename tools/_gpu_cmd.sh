set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_phmm_gpu.py -x -q 2>&1 | tail -2
timeout -k 10 300 python tools/phmm_probe.py 2>&1 | grep -v amdgpu.ids
