# r03h: chain drop-in (upload/plan overlap) and the per-batch phmm drop-in's kernel breakdown
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_chain.py -m gpu > gpurun_out/pytest_r03h.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r03h.log; [ $rc -eq 0 ] || exit 1
DROPIN_LEGS=chain GB_CHAIN_HOSTPROF=1 timeout -k 10 200 python -u tools/dropin_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/phmm_pb_r03h -o run -- python3 tools/phmm_dropin_probe.py > gpurun_out/phmm_pb_r03h.log 2>&1; echo prof rc=$?
