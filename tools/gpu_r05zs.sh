#!/bin/bash
# round-5 GPU call zs: bench stdout is exactly one JSON line at N=1 and N=2 (self-launch and torchrun)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zs}
A="--only phmm --no-small --no-e2e --no-cpu-baseline --steps 3 --warmup 1 --shard-of 0"
timeout -k 10 300 python -u bench.py $A > gpurun_out/out1_${T}.txt 2> gpurun_out/err1_${T}.txt || { tail -20 gpurun_out/err1_${T}.txt; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 2 $A > gpurun_out/out2_${T}.txt 2> gpurun_out/err2_${T}.txt || { tail -20 gpurun_out/err2_${T}.txt; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 $A > gpurun_out/out3_${T}.txt 2> gpurun_out/err3_${T}.txt || { tail -20 gpurun_out/err3_${T}.txt; exit 1; }
for f in 1 2 3; do
  python3 - gpurun_out/out${f}_${T}.txt <<'PY'
import json, sys
lines = open(sys.argv[1]).read().splitlines()
ok = len(lines) == 1 and json.loads(lines[0])["value"] is not None
print(sys.argv[1], "lines", len(lines), "one JSON line" if ok else "NOT ONE JSON LINE", lines[0][:80] if lines else "")
PY
done
