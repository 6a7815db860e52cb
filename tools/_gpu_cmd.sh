set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r01b
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; st=$?; tail -15 gpurun_out/pytest_gpu.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; st=$?; tail -3 gpurun_out/smoke.log; [ $st -eq 0 ] || exit $st
timeout -k 10 1000 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; st=$?; tail -3 gpurun_out/bench_${TAG}.err; cat gpurun_out/bench_${TAG}.json; exit $st
