# r03v: same-box A/B of the fmi search: r03n library (tools/_ab), the tree's, and diagnostic variants
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in _ab _ab1 _ab2 .; do
    L=tools/$v/genomicsbench_palisade_amd/lib/libgb.so; [ $v = . ] && L=genomicsbench_palisade_amd/lib/libgb.so
    FMI_LIB=$L timeout -k 10 200 python -u tools/fmi_lib_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a gpurun_out/ab_r03v.log || exit 1
  done
done
