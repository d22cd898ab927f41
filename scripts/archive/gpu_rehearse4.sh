#!/bin/bash
# The spawned 4-rank bench line rehearsed on one GPU (gloo), every N>1 leg, with a heartbeat.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-rehearse4}; mkdir -p $O
start=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 4 --rehearse --steps 3 --warmup 1 --bucket-mib ${MIB:-32} --no-size-sweep > $O/rehearse4.json 2> $O/rehearse4.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; echo "alive $(( $(date +%s) - start ))s"; done
wait $pid; rc=$?; echo "rehearse4 rc=$rc wall=$(( $(date +%s) - start ))s"
python3 -c "
import json; d=json.loads(open('$O/rehearse4.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'transport', d.get('transport'), 'parity', d.get('parity_vs_mpich_order',{}).get('bit_exact'))
print('leg_errors', d.get('leg_errors')); print('incomplete', d.get('incomplete')); print('cu_mask_ab', d.get('compute_cu_mask_ab'))
print(sorted(d.keys()))" || tail -20 $O/rehearse4.err
exit $rc
