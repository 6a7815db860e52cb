set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_bsw.py -x -q -m gpu 2>&1 | tail -2
GB_BSW_PROF=1 timeout -k 10 300 python tools/bsw_probe.py 2>&1 | grep -v amdgpu.ids | tail -7
