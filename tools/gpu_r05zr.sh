#!/bin/bash
# round-5 GPU call zr: the 2-rank rehearsal of bench.py --gpus 2 on the final code (ranks share the GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zr}
timeout -k 10 900 python -u bench.py --gpus 2 --steps 10 --warmup 3 --detail-out gpurun_out/bench_${T}_n2_detail.json \
  > gpurun_out/bench_${T}_n2.json 2> gpurun_out/bench_${T}_n2.err || { tail -30 gpurun_out/bench_${T}_n2.err; exit 1; }
tail -2 gpurun_out/bench_${T}_n2.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_n2.json')); print({k: d.get(k) for k in ('n_gpus','value','rank_check_bit_exact')})"
