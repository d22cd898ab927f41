#!/bin/bash
# Rehearsal of the N>1 bench on ONE GPU: N processes on cuda:0, point-to-point over gloo host
# copies (bench.py --rehearse, tools/gloo_transport.py). Exercises every N>1 leg of bench.py
# before the driver's 8-GPU run; the numbers are not measurements.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${N:-2}
timeout -k 10 ${RT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port ${PORT:-29555} bench.py --gpus $N --steps 5 --warmup 2 --bucket-mib ${MIB:-8} --size-sweep-max-mib 16 \
  --rehearse > gpurun_out/rehearse$N.json 2> gpurun_out/rehearse$N.err
rc=$?; echo "rehearse N=$N rc=$rc"; tail -c 600 gpurun_out/rehearse$N.json; exit $rc
