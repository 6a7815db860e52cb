#!/bin/bash
# One checkpoint on the GPU box, stage by stage, stopping at the first failure:
#   tests  -m gpu parity suite            -> gpurun_out/pytest_TAG.log
#   smoke  __graft_entry__.smoke()
#   bench  the driver's command           -> gpurun_out/bench_TAG.json (headline) + bench_TAG_detail.json
#   prof   kernel-trace stats + FETCH/WRITE PMC passes (tools/gpu_prof.sh)
#   pmcsum those passes summarised into profiles/TAG_pmc.json on the box (run before bench, so the
#          bench line's traffic is this checkpoint's)
#   lds    LDS-conflict / VALU-busy SQ counters per leg (tools/gpu_lds.sh)
#   probe  one probe script per call: PROBE="tools/x.py args" -> gpurun_out/probe_TAG.log
# Usage: gpu_checkpoint.sh TAG [stages...]   (default stages: tests smoke bench)
#   gpurun --timeout 1200 -- 'bash tools/gpu_checkpoint.sh r04a tests smoke bench prof'
# Environment: TESTS (pytest paths / -k, default "tests"), BENCH_ARGS (default "--steps 20 --warmup 5"),
#   PROBE (the probe stage's command line, run under python3)
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
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests} -m gpu \
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
    pmcsum)
      # the prof stage's PMC passes summarised into profiles/ on the box, so a bench stage after it
      # cites this checkpoint's traffic (copies come back under gpurun_out/ for collect_checkpoint)
      for pre in pmc pmch; do
        fd=$(find gpurun_out/${pre}_fetch_${TAG} -name run_counter_collection.csv | sort | tail -1)
        wd=$(find gpurun_out/${pre}_write_${TAG} -name run_counter_collection.csv | sort | tail -1)
        [ -n "$fd" ] && [ -n "$wd" ] || { echo "pmcsum: no ${pre} passes for ${TAG}"; exit 1; }
        dst=profiles/${TAG}_pmc.json
        [ $pre = pmch ] && dst=profiles/${TAG}_human_pmc.json
        python3 tools/pmc_summary.py "$(dirname "$fd")" "$(dirname "$wd")" $dst > /dev/null || exit 1
        cp $dst gpurun_out/pmcsum_$(basename $dst)
      done
      echo "pmcsum ok" ;;
    lds)
      bash tools/gpu_lds.sh ${TAG} || exit 1 ;;
    probe)
      timeout -k 10 ${PROBE_TIMEOUT:-300} python3 -u ${PROBE:?PROBE} > gpurun_out/probe_${TAG}.log 2>&1; rc=$?
      grep -v amdgpu.ids gpurun_out/probe_${TAG}.log | tail -${PROBE_TAIL:-30}
      [ $rc -eq 0 ] || exit 1 ;;
    *)
      echo "unknown stage $s"; exit 2 ;;
  esac
done
