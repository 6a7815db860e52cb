#!/bin/bash
# Kernel-trace statistics of the chain leg alone (bench.py --only chain). Usage: gpu_chain_prof.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-chain}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cprof_${TAG} -o run -- python3 bench.py --only chain --steps 5 --warmup 1 --no-cpu-baseline --no-small --no-e2e > gpurun_out/cprof_${TAG}.json 2> gpurun_out/cprof_${TAG}.err || { echo "chain profile failed"; tail -20 gpurun_out/cprof_${TAG}.err; exit 1; }
find gpurun_out/cprof_${TAG} -name "*kernel_stats.csv" | head -3
