set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 400 python -u -m pytest tests/test_multiproc_gpu.py tests/test_api_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s4/pytest_mp.log 2>&1
