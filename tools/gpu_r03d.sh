# r03d: phmm parity with adaptive stack heights, the shard probe, the human-scale fmi leg
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_phmm_gpu.py tests/test_edges.py > gpurun_out/pytest_r03d.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r03d.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/phmm_shard_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python -u bench.py --only fmi_human --steps 5 --warmup 1 > gpurun_out/bench_r03d_human.json 2> gpurun_out/bench_r03d_human.err; echo human rc=$?; tail -3 gpurun_out/bench_r03d_human.err
