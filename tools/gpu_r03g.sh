# r03g: parity (bsw small path + combiner, chain, abi, fmi incl. heavy pass and class drop-in wave
# kernels), drop-in probe, fmi NT-gather A/B with FETCH_SIZE / WRITE_SIZE passes
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bsw.py tests/test_chain.py tests/test_abi.py tests/test_fmi_gpu.py tests/test_fmi_dropin.py -m gpu > gpurun_out/pytest_r03g.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r03g.log; [ $rc -eq 0 ] || exit 1
GB_CHAIN_HOSTPROF=1 timeout -k 10 300 python -u tools/dropin_probe.py > gpurun_out/dropin_r03g.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/dropin_r03g.log; [ $rc -eq 0 ] || exit 1
for NT in 0 1; do
  GB_FMI_NT=$NT FMI_PROBE_READS=4000000 timeout -k 10 120 python -u tools/fmi_probe.py 2>&1 | grep -v amdgpu.ids | sed "s/^/NT=$NT /" || exit 1
  GB_FMI_NT=$NT FMI_PROBE_READS=4000000 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ntf_r03g_$NT -o run -- python3 tools/fmi_probe.py > /dev/null 2>&1 || exit 1
  GB_FMI_NT=$NT FMI_PROBE_READS=4000000 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ntw_r03g_$NT -o run -- python3 tools/fmi_probe.py > /dev/null 2>&1 || exit 1
done
echo pmc done
timeout -k 10 200 python -u tools/phmm_dropin_probe.py 2>&1 | grep -v amdgpu.ids
for PF in 1 0; do GB_FMI_PREFETCH=$PF FMI_TAIL_TAG=r03g_pf$PF timeout -k 10 240 python -u tools/fmi_tail_probe.py 2>&1 | grep -v amdgpu.ids | sed "s/^/PF=$PF /"; done
