# r03o: fmi tail hand-over (resumable records, helper waves): fmi GPU tests, then the fmi leg with
# its shard proxy per GB_FMI_DRAIN / GB_FMI_HELP setting
mkdir -p gpurun_out
export TMPDIR=/tmp
true
for v in "4 1" "0 1" "2 1" "8 1" "16 1" "4 0"; do
  set -- $v
  GB_FMI_DRAIN=$1 GB_FMI_HELP=$2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --only fmi --no-cpu-baseline --no-small --no-e2e > gpurun_out/fmi_r03o_$1_$2.json 2> gpurun_out/fmi_r03o_$1_$2.err || { echo "bench $v failed"; tail -5 gpurun_out/fmi_r03o_$1_$2.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/fmi_r03o_$1_$2.json')); f=d['fmi'] if 'fmi' in d else d
sp=f.get('shard_proxy',{}); print('drain $1 help $2:', f['value'], 'Mreads/s', f['ms_per_step'], 'ms; shard', sp.get('per_gpu_min'), sp.get('ratio_min_vs_full'), f.get('kernels_ms'))"
done
