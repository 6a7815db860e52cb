# r03y: host_chain_kernel host/GPU phase breakdown
mkdir -p gpurun_out
export TMPDIR=/tmp
DROPIN_LEGS=chain GB_CHAIN_HOSTPROF=1 timeout -k 10 300 python -u tools/dropin_probe.py 2>&1 | grep -v amdgpu.ids | tail -20
