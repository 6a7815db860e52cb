# r03y: checkpoint (fmi slot sort on the r03n lane kernel, bsw small-batch tail balance): all GPU tests, smoke, the bench line, rocprof + PMC
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_r03y.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r03y.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 1100 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03y.json 2> gpurun_out/bench_r03y.err; rc=$?; echo bench rc=$rc; [ $rc -eq 0 ] || exit 1
bash tools/gpu_prof.sh r03y
