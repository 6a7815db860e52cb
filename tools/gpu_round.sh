#!/bin/bash
# One checkpoint on the GPU box: parity tests, smoke, the bench line, rocprofv3 kernel stats and the
# PMC HBM-traffic passes (tools/gpu_prof.sh). Stops at the first failure. Usage: gpu_round.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
echo "bench ok"
bash tools/gpu_prof.sh ${TAG} || exit 1
