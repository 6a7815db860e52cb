set -o pipefail
export TMPDIR=/tmp
GB_CHAIN_PROF=1 timeout -k 10 300 python tools/chain_probe.py 2>&1 | grep -v amdgpu.ids | sed -n 5,6p
