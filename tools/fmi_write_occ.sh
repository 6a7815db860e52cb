#!/bin/bash
# fmi smem_search: HBM-side write bytes (rocprofv3 WRITE_SIZE, its own pass) and search time against
# resident waves per CU (GB_FMI_WAVES_PER_CU). The per-lane `prev` lists' hot set scales with the
# resident waves of an XCD, so this measures how much of WRITE_SIZE is their eviction from L2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--only fmi --steps 1 --warmup 1 --no-cpu-baseline --no-small --no-e2e"
for w in ${WAVES:-8 12 16}; do
  GB_FMI_WAVES_PER_CU=$w timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/fmi_wr_w$w -o run -- python3 bench.py $ARGS > gpurun_out/fmi_wr_w$w.json 2> gpurun_out/fmi_wr_w$w.err || { echo "WRITE_SIZE pass failed (waves $w)"; tail gpurun_out/fmi_wr_w$w.err; exit 1; }
  f=$(find gpurun_out/fmi_wr_w$w -name "run_counter_collection.csv" | head -1)
  echo "waves/CU $w"; python3 tools/pmc_kernel.py "$(dirname "$f")" smem_search | tail -3
done
