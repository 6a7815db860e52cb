# r03m: fmi occupancy A/B with the LDS list head: read codes staged in LDS (11 waves per CU fit) or
# read from global memory (the list head alone: 12 / 14 / 16 waves per CU)
mkdir -p gpurun_out
export TMPDIR=/tmp
GB_FMI_QLDS=1 FMI_PROBE_READS=4000000 timeout -k 10 120 python -u tools/fmi_probe.py 2>&1 | grep -v amdgpu.ids | sed "s/^/QLDS=1 /" || exit 1
for W in 11 12 14 16; do
  GB_FMI_QLDS=0 GB_FMI_WAVES_PER_CU=$W FMI_PROBE_READS=4000000 timeout -k 10 120 python -u tools/fmi_probe.py 2>&1 | grep -v amdgpu.ids | sed "s/^/QLDS=0 W=$W /" || exit 1
done
echo done
