#!/bin/bash
# One checkpoint on the GPU box, stage by stage, stopping at the first failure:
#   tests  -m gpu parity suite            -> gpurun_out/pytest_TAG.log
#   smoke  __graft_entry__.smoke()
#   bench  the driver's command           -> gpurun_out/bench_TAG.json (headline) + bench_TAG_detail.json
#   prof   kernel-trace stats + FETCH/WRITE PMC passes (tools/gpu_prof.sh)
#   lds    LDS-conflict / VALU-busy SQ counters per leg (tools/gpu_lds.sh)
# Usage: gpu_checkpoint.sh TAG [stages...]   (default stages: tests smoke bench)
#   gpurun --timeout 1200 -- 'bash tools/gpu_checkpoint.sh r04a tests smoke bench prof'
# Then, here: python tools/collect_checkpoint.py TAG  (copies the summaries into profiles/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:?tag}
shift
STAGES=${*:-tests smoke bench}
BENCH_ARGS=${BENCH_ARGS:---steps 20 --warmup 5}
for s in $STAGES; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
        > gpurun_out/pytest_${TAG}.log 2>&1; rc=$?
      tail -2 gpurun_out/pytest_${TAG}.log
      [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_${TAG}.log; exit 1; } ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
        || { cat gpurun_out/smoke_${TAG}.log; exit 1; }
      grep -v amdgpu.ids gpurun_out/smoke_${TAG}.log | tail -3 ;;
    bench)
      timeout -k 10 600 python -u bench.py $BENCH_ARGS --detail-out gpurun_out/bench_${TAG}_detail.json \
        > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; rc=$?
      echo "bench rc=$rc, headline $(wc -c < gpurun_out/bench_${TAG}.json) bytes"
      [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; } ;;
    prof)
      bash tools/gpu_prof.sh ${TAG} || exit 1 ;;
    lds)
      bash tools/gpu_lds.sh ${TAG} || exit 1 ;;
    *)
      echo "unknown stage $s"; exit 2 ;;
  esac
done
