#!/bin/bash
# round-5 GPU call: phmm two-rows-per-lane parity + A/B, stale-LDS tests, 2-rank bench rehearsal on
# one GPU, a phmm shard kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05a}
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_phmm_gpu.py tests/test_edges.py \
  tests/test_lds_poison.py -m gpu > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -2 gpurun_out/pytest_${T}.log
PHMM_ROWS="GB_PHMM_RPL=1;GB_PHMM_RPL=2" timeout -k 10 300 python -u tools/phmm_shard_probe.py > gpurun_out/phmm_ab_${T}.log 2>&1 \
  || { tail -20 gpurun_out/phmm_ab_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_ab_${T}.log
timeout -k 10 900 python -u bench.py --gpus 2 --steps 10 --warmup 3 --detail-out gpurun_out/bench_${T}_n2_detail.json \
  > gpurun_out/bench_${T}_n2.json 2> gpurun_out/bench_${T}_n2.err || { tail -30 gpurun_out/bench_${T}_n2.err; exit 1; }
tail -2 gpurun_out/bench_${T}_n2.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_${T}_phmm -o run -- \
  python3 tools/phmm_shard_probe.py > gpurun_out/phmm_probe_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_probe_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_probe_${T}.log | tail -3
