# The N=1 bench line alone.
set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 400 python -u bench.py > gpurun_out/s4/bench_n1.json 2> gpurun_out/s4/bench_n1.err
