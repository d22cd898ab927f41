#!/bin/bash
# The spawned 8-rank bench line rehearsed on one GPU (gloo point-to-point; every N>1 leg runs),
# at a small bucket (the gloo host staging is slow); a heartbeat line every 30 s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-rehearse8}; mkdir -p $O
start=$(date +%s)
timeout -k 10 800 python3 bench.py --gpus 8 --rehearse --steps 3 --warmup 1 --bucket-mib ${MIB:-8} --no-size-sweep --no-config-sweep > $O/rehearse8_spawn.json 2> $O/rehearse8_spawn.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; echo "alive $(( $(date +%s) - start ))s: $(grep -c . $O/rehearse8_spawn.err) stderr lines"; done
wait $pid; rc=$?; echo "rehearse8 rc=$rc wall=$(( $(date +%s) - start ))s"
python3 -c "
import json; d=json.loads(open('$O/rehearse8_spawn.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'transport', d.get('transport'), 'parity', d.get('parity_vs_mpich_order'))
print('leg_errors', d.get('leg_errors')); print('incomplete', d.get('incomplete')); print(sorted(d.keys()))" || tail -20 $O/rehearse8_spawn.err
exit $rc
