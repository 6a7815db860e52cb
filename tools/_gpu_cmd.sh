set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r01c
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; st=$?; tail -3 gpurun_out/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 1000 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; st=$?; tail -2 gpurun_out/bench_${TAG}.err; [ $st -eq 0 ] || exit $st
python3 -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}.json'))
print('phmm', d['value'], d['roofline']['frac']); 
for k in ('fmi','chain','bsw'): print(k, d[k]['value'], d[k]['unit'], d[k]['roofline']['frac'], (d[k]['cpu_baseline'] or {}).get('value'))
"
