# r03q: per-XCD hand-over queues: fmi tests, then the routine's speed inside smem_search vs smem_heavy
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fmi_gpu.py -m gpu > gpurun_out/pytest_r03q.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r03q.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/fmi_help_probe.py 2>&1 | tee gpurun_out/help_r03q.log | grep -v amdgpu.ids
