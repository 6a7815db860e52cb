# r03t: phmm shard breakdown (f32 / f64 / step) per stack height
mkdir -p gpurun_out
export TMPDIR=/tmp
PHMM_ROWS="default;GB_PHMM_F64_ROWS=0;GB_PHMM_F64_ROWS=2048;GB_PHMM_F64_ROWS=8192;GB_PHMM_STACK_ROWS=1024,GB_PHMM_F64_ROWS=4096" timeout -k 10 400 python -u tools/phmm_shard_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/phmm_shard_r03t.log
