set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 120 tools/bin/reduce_map_tune 256 5 > gpurun_out/s4/reduce_map_256MiB.txt 2>&1 && \
timeout -k 10 120 tools/bin/reduce_map_tune 1024 3 > gpurun_out/s4/reduce_map_1024MiB.txt 2>&1
