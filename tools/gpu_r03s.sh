# r03s: same-box A/B of the fmi hand-over settings
mkdir -p gpurun_out
export TMPDIR=/tmp
FMI_AB="GB_FMI_HELP=0,GB_FMI_DRAIN=0,GB_FMI_LIST=0;GB_FMI_HELP=1,GB_FMI_DRAIN=0,GB_FMI_LIST=0;GB_FMI_HELP=1,GB_FMI_DRAIN=2,GB_FMI_LIST=0;GB_FMI_HELP=1,GB_FMI_DRAIN=0,GB_FMI_LIST=32;GB_FMI_HELP=1,GB_FMI_DRAIN=2,GB_FMI_LIST=32;GB_FMI_HELP=1,GB_FMI_DRAIN=0,GB_FMI_LIST=48" FMI_AB_REPS=3 timeout -k 10 600 python -u tools/fmi_ab_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_r03s.log
