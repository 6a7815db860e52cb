mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_chain.py tests/test_fmi_dropin.py > gpurun_out/pytest_r03c.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r03c.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_r03c.json 2> gpurun_out/bench_r03c.err; echo bench rc=$?; tail -2 gpurun_out/bench_r03c.err
