# Run one GPU test file (argument) under a time limit.
set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 500 python -u -m pytest "$1" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s4/pytest_one.log 2>&1
