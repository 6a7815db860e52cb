# r03x: fmi at r03n + the 16-lane slot sort: fmi GPU tests, same-box A/B against the r03n library
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fmi_gpu.py tests/test_phmm_gpu.py -m gpu > gpurun_out/pytest_r03x.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r03x.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  FMI_LIB=tools/_ab/genomicsbench_palisade_amd/lib/libgb.so timeout -k 10 200 python -u tools/fmi_lib_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/r03n /" | tee -a gpurun_out/ab_r03x.log || exit 1
  timeout -k 10 200 python -u tools/fmi_lib_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/tree /" | tee -a gpurun_out/ab_r03x.log || exit 1
done
