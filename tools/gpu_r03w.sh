# r03w: fmi hand-over records via smem_heavy only + list trigger; phmm two stacks per wave (packed
# f32): their GPU tests, then same-box A/Bs
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fmi_gpu.py tests/test_phmm_gpu.py -m gpu > gpurun_out/pytest_r03w.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r03w.log; [ $rc -eq 0 ] || exit 1
PHMM_ROWS="GB_PHMM_PAIR=0;GB_PHMM_PAIR=1" timeout -k 10 300 python -u tools/phmm_shard_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/phmm_pair_r03w.log || exit 1
for rep in 1 2; do
  FMI_LIB=tools/_ab/genomicsbench_palisade_amd/lib/libgb.so timeout -k 10 200 python -u tools/fmi_lib_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/r03n /" | tee -a gpurun_out/ab_r03w.log || exit 1
  timeout -k 10 200 python -u tools/fmi_lib_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/list32 /" | tee -a gpurun_out/ab_r03w.log || exit 1
  GB_FMI_LIST=0 timeout -k 10 200 python -u tools/fmi_lib_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/list0 /" | tee -a gpurun_out/ab_r03w.log || exit 1
done
