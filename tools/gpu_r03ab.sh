# r03ab: bsw small-batch tail balance: bsw GPU tests, then the bsw legs per GB_BSW_TAIL
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bsw.py -m gpu > gpurun_out/pytest_r03ab.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r03ab.log; [ $rc -eq 0 ] || exit 1
for f in 0 0.02 0.05 0.1 0.2; do
  GB_BSW_TAIL=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --only bsw --no-cpu-baseline --no-e2e --shard-of 0 > gpurun_out/bsw_r03ab_$f.json 2> gpurun_out/bsw_r03ab_$f.err || { echo "bench $f failed"; tail -5 gpurun_out/bsw_r03ab_$f.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bsw_r03ab_$f.json')); b=d['bsw'] if 'bsw' in d else d
print('tail $f: large', b['value'], 'small', d.get('small',{}).get('bsw',{}).get('value'), d.get('small',{}).get('bsw',{}).get('ms_per_step'))"
done
