set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "cli" > gpurun_out/pytest_cli.log 2>&1; st=$?; tail -30 gpurun_out/pytest_cli.log; exit $st
