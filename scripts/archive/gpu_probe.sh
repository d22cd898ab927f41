set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 240 python -u tools/zero_copy_probe.py > gpurun_out/s4/zero_copy2.jsonl 2> gpurun_out/s4/zero_copy2.err
