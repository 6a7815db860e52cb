#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of a short bench run, then HBM traffic from
# PMC counters in their own passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-small --no-e2e"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err || { echo "kernel-trace run failed"; tail -20 gpurun_out/prof_${TAG}.err; exit 1; }
echo "kernel trace ok"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_${TAG} -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-small --no-e2e > gpurun_out/pmc_fetch_${TAG}.json 2> gpurun_out/pmc_fetch_${TAG}.err || { echo "FETCH_SIZE run failed"; tail -20 gpurun_out/pmc_fetch_${TAG}.err; exit 1; }
echo "fetch ok"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_${TAG} -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-small --no-e2e > gpurun_out/pmc_write_${TAG}.json 2> gpurun_out/pmc_write_${TAG}.err || { echo "WRITE_SIZE run failed"; tail -20 gpurun_out/pmc_write_${TAG}.err; exit 1; }
echo "write ok"
find gpurun_out/prof_${TAG} gpurun_out/pmc_fetch_${TAG} gpurun_out/pmc_write_${TAG} -name "*.csv" | head -20
