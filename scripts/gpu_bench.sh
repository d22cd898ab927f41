# The zero-copy probe and the N=1 bench line (no test suite).
set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 180 python -u tools/zero_copy_probe.py > gpurun_out/s4/zero_copy.jsonl 2> gpurun_out/s4/zero_copy.err && \
timeout -k 10 400 python -u bench.py > gpurun_out/s4/bench_n1.json 2> gpurun_out/s4/bench_n1.err
