set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 500 python -u tools/host_unpack_ab.py > gpurun_out/s4/host_unpack_ab.jsonl 2> gpurun_out/s4/host_unpack_ab.err
