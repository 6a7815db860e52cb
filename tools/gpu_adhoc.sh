#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_chain.py tests/test_chain_bt.py tests/test_edges.py -m gpu 2>&1 | tail -3 || exit 1
for L in genomicsbench_palisade_amd/lib/ab/libgb_A.so genomicsbench_palisade_amd/lib/libgb.so genomicsbench_palisade_amd/lib/ab/libgb_A.so genomicsbench_palisade_amd/lib/libgb.so; do
CHAIN_LIB=$L CHAIN_CONFIGS=";GB_CHAIN_SPLIT=-1,128,0,5000" timeout -k 10 200 python3 tools/chain_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/chain_ab_r04d.log || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chainshard_r04d -o run -- python3 tools/chain_shard_probe.py > gpurun_out/chainshard_r04d.log 2>&1 || { tail -20 gpurun_out/chainshard_r04d.log; exit 1; }
CHAIN_OF=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chainfull_r04d -o run -- python3 tools/chain_shard_probe.py > gpurun_out/chainfull_r04d.log 2>&1 || { tail -20 gpurun_out/chainfull_r04d.log; exit 1; }
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/lds_chain_r04d -o run -- python3 bench.py --only chain --steps 2 --warmup 1 --no-cpu-baseline --no-small --no-e2e --shard-of 0 > gpurun_out/lds_chain_r04d.json 2> gpurun_out/lds_chain_r04d.err || { tail gpurun_out/lds_chain_r04d.err; exit 1; }
python3 tools/pmc_lds.py gpurun_out/lds_r04d.json gpurun_out/lds_chain_r04d
