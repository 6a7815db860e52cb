# r03z: host_chain_kernel in overlapped pieces: chain GPU tests, then the drop-in probe per piece count
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_chain.py -m gpu > gpurun_out/pytest_r03z.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r03z.log; [ $rc -eq 0 ] || exit 1
for k in 1 4 8 2; do
  echo "== GB_CHAIN_CHUNKS=$k"
  GB_CHAIN_CHUNKS=$k DROPIN_LEGS=chain GB_CHAIN_HOSTPROF=1 timeout -k 10 300 python -u tools/dropin_probe.py 2>&1 | grep -v amdgpu.ids | grep -v "^\[gb_chain\]" | tail -3 || exit 1
done
