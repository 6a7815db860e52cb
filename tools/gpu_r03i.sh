# r03i: phmm chunked f32/f64 overlap: parity, shard probe, per-batch drop-in probe
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_phmm_gpu.py tests/test_edges.py tests/test_dropin_threads.py -m gpu > gpurun_out/pytest_r03i.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r03i.log; [ $rc -eq 0 ] || exit 1
for C in 1 0; do
  if [ $C = 1 ]; then export GB_PHMM_CHUNKS=1; else unset GB_PHMM_CHUNKS; fi
  echo "GB_PHMM_CHUNKS=${GB_PHMM_CHUNKS:-auto}"
  timeout -k 10 200 python -u tools/phmm_shard_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  PHMM_RANK=4 timeout -k 10 200 python -u tools/phmm_shard_probe.py 2>&1 | grep -v amdgpu.ids | grep shard || exit 1
  timeout -k 10 200 python -u tools/phmm_dropin_probe.py 2>/dev/null | grep -v amdgpu.ids || exit 1
done
