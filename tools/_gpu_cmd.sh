set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_bsw.py -x -q -m gpu > gpurun_out/pytest_bsw.log 2>&1; st=$?; tail -30 gpurun_out/pytest_bsw.log; [ $st -eq 0 ] || exit $st
timeout -k 10 600 python bench.py --only chain,bsw --steps 5 --warmup 1 > gpurun_out/bench_cb.json 2> gpurun_out/bench_cb.err; st=$?; tail -5 gpurun_out/bench_cb.err; cat gpurun_out/bench_cb.json; exit $st
