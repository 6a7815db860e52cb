# r03k: fmi `prev`-list head in LDS (GB_FMI_TOP): parity, timing and FETCH/WRITE_SIZE A/B, then the
# r03j rocprof checkpoint if the first part passes
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fmi_gpu.py tests/test_fmi_large.py -m gpu > gpurun_out/pytest_r03k.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r03k.log; [ $rc -eq 0 ] || exit 1
for T in 0 1; do
  GB_FMI_TOP=$T FMI_PROBE_READS=4000000 timeout -k 10 120 python -u tools/fmi_probe.py 2>&1 | grep -v amdgpu.ids | sed "s/^/TOP=$T /" || exit 1
  GB_FMI_TOP=$T FMI_PROBE_READS=4000000 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/topf_r03k_$T -o run -- python3 tools/fmi_probe.py > /dev/null 2>&1 || exit 1
  GB_FMI_TOP=$T FMI_PROBE_READS=4000000 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/topw_r03k_$T -o run -- python3 tools/fmi_probe.py > /dev/null 2>&1 || exit 1
done
GB_FMI_TOP=1 FMI_TAIL_TAG=r03k timeout -k 10 240 python -u tools/fmi_tail_probe.py 2>&1 | grep -v amdgpu.ids | grep -v "^ "
echo done
