set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_bsw.py -x -q -m gpu 2>&1 | tail -2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bsw3 -o run -- python3 tools/bsw_probe.py > /dev/null 2>&1
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_bsw3/run_kernel_stats.csv')))[:6]: print(r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e6)
"
