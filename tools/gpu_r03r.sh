# r03r: fmi hand-over triggers: list length (GB_FMI_LIST), tail lane count (GB_FMI_DRAIN), tail call
# count (GB_FMI_DRAIN_CALLS); fmi leg + shard proxy per setting
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fmi_gpu.py -m gpu -k heavy > gpurun_out/pytest_r03r.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r03r.log; [ $rc -eq 0 ] || exit 1
for v in "2 32 0" "0 0 0" "2 0 0" "2 16 0" "2 64 0" "2 32 1000" "0 32 0"; do
  set -- $v
  t=$1_$2_$3
  GB_FMI_DRAIN=$1 GB_FMI_LIST=$2 GB_FMI_DRAIN_CALLS=$3 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --only fmi --no-cpu-baseline --no-small --no-e2e > gpurun_out/fmi_r03r_$t.json 2> gpurun_out/fmi_r03r_$t.err || { echo "bench $v failed"; tail -5 gpurun_out/fmi_r03r_$t.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/fmi_r03r_$t.json')); f=d['fmi'] if 'fmi' in d else d
sp=f.get('shard_proxy',{}); print('drain $1 list $2 dcalls $3:', f['value'], 'Mreads/s', f['ms_per_step'], 'ms; shard', sp.get('per_gpu_min'), round(sp.get('ratio_min_vs_full'),4))"
done
