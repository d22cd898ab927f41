#!/bin/bash
# r06 s16: the driver's N>1 launch form (torch.distributed.run, one rank per process) over real
# two-rank RCCL on one GPU (--rehearse-rccl), with a heartbeat.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s16; mkdir -p $O
export NCCL_DEBUG=WARN
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --rehearse-rccl --steps 3 --warmup 1 --bucket-mib 8 --no-size-sweep --no-config-sweep > $O/torchrun2.json 2> $O/torchrun2.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; echo "alive $(grep -c . $O/torchrun2.err) stderr lines"; done
wait $pid; rc=$?; echo "torchrun rc=$rc"
python3 -c "
import json; d=json.loads([l for l in open('$O/torchrun2.json').read().splitlines() if l.startswith('{')][-1])
print('n_gpus', d['n_gpus'], 'transport', d.get('transport'), 'parity', d.get('parity_vs_mpich_order', {}).get('bit_exact'), 'leg_errors', d.get('leg_errors'), 'incomplete', d.get('incomplete'))" || tail -20 $O/torchrun2.err
exit $rc
