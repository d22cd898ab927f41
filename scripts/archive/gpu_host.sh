# Host-path GPU tests and the N=1 bench line.
set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 400 python -u -m pytest tests/test_api_gpu.py tests/test_multiproc_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s4/pytest_host.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/s4/bench_n1.json 2> gpurun_out/s4/bench_n1.err
