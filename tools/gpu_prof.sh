#!/bin/bash
# rocprofv3 evidence for one checkpoint: kernel-trace stats of a short bench run of the four legs, then
# HBM traffic from PMC counters in their own passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on
# gfx950), and the same two passes for the human-scale fmi leg alone (its smem_search launches would
# otherwise mix with the 512 Mbp leg's). Usage: gpu_prof.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
LEGS="--only phmm,fmi,chain,bsw --no-cpu-baseline --no-small --no-e2e --shard-of 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 5 --warmup 1 $LEGS > gpurun_out/prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err || { echo "kernel-trace run failed"; tail -20 gpurun_out/prof_${TAG}.err; exit 1; }
echo "kernel trace ok"
for C in FETCH_SIZE WRITE_SIZE; do
  c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_${c}_${TAG} -o run -- python3 bench.py --steps 2 --warmup 1 $LEGS > gpurun_out/pmc_${c}_${TAG}.json 2> gpurun_out/pmc_${c}_${TAG}.err || { echo "$C run failed"; tail -20 gpurun_out/pmc_${c}_${TAG}.err; exit 1; }
  echo "$C ok"
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmch_${c}_${TAG} -o run -- python3 bench.py --steps 2 --warmup 1 --only fmi_human --no-cpu-baseline --fmi-human-reads 2000000 > gpurun_out/pmch_${c}_${TAG}.json 2> gpurun_out/pmch_${c}_${TAG}.err || { echo "human $C run failed"; tail -20 gpurun_out/pmch_${c}_${TAG}.err; exit 1; }
  echo "human $C ok"
done
find gpurun_out/prof_${TAG} gpurun_out/pmc_*_${TAG} gpurun_out/pmch_*_${TAG} -name "*.csv" | head -20
