# Run one measurement tool (argument: tools/<name>.py) under a time limit.
set -o pipefail
mkdir -p gpurun_out/s4
n=$(basename "$1" .py)
timeout -k 10 300 python -u "$1" > gpurun_out/s4/$n.jsonl 2> gpurun_out/s4/$n.err
