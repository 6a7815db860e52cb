# r03p: fmi tail trace with the helper waves (drain 0 and 4) vs the post-pass (help 0)
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "0 1" "2 1" "4 1" "8 1"; do
  set -- $v
  GB_FMI_DRAIN=$1 GB_FMI_HELP=$2 FMI_TAIL_TAG=r03p_$1_$2 timeout -k 10 240 python -u tools/fmi_tail_probe.py > gpurun_out/tail_r03p_$1_$2.log 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/tail_r03p_$1_$2.log; exit 1; }
  echo "== drain $1 help $2"; grep -v "^max RSS" gpurun_out/tail_r03p_$1_$2.log | tail -4
done
