#!/bin/bash
# The spawned N-rank bench line rehearsed on one GPU (gloo point-to-point; every N>1 leg runs,
# the CPU baseline legs at P = N included), for each N in $NS (default "2 4 8"), at a small
# bucket (the gloo host staging is slow); a heartbeat line every 30 s; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-rehearse}; mkdir -p $O
for N in ${NS:-2 4 8}; do
  start=$(date +%s)
  timeout -k 10 ${LIMIT:-500} python3 bench.py --gpus $N ${MODE:---rehearse} --steps 3 --warmup 1 --bucket-mib ${MIB:-8} --no-size-sweep --no-config-sweep ${EXTRA:-} > $O/rehearse${N}_spawn.json 2> $O/rehearse${N}_spawn.err &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 30; echo "N=$N alive $(( $(date +%s) - start ))s: $(grep -c . $O/rehearse${N}_spawn.err) stderr lines"; done
  wait $pid; rc=$?; echo "rehearse$N rc=$rc wall=$(( $(date +%s) - start ))s"
  python3 -c "
import json; d=json.loads(open('$O/rehearse${N}_spawn.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'transport', d.get('transport'), 'parity', d.get('parity_vs_mpich_order', {}).get('bit_exact'))
print('cpu_baseline', d.get('cpu_baseline')); print('keys', [k for k in ('cpu_baseline', 'cpu_reference_path', 'roofline', 'link_roofline', 'transport') if k in d])
print('leg_errors', d.get('leg_errors')); print('incomplete', d.get('incomplete'))" || tail -20 $O/rehearse${N}_spawn.err
  [ $rc -ne 0 ] && exit $rc
done
exit 0
