#!/bin/bash
# r06 s19: the N = 2 line over real RCCL with the size sweeps on (eager and graph-captured) after
# the captured graphs are released before teardown (s18's run printed its line, then hung in
# teardown); heartbeat, Python stacks if it stalls again.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s19; mkdir -p $O
export NCCL_DEBUG=WARN
start=$(date +%s)
timeout -k 10 400 python bench.py --gpus 2 --rehearse-rccl --steps 3 --warmup 1 --bucket-mib 8 --no-config-sweep --size-sweep-max-mib 16 --watchdog-s 300 > $O/rehearse2_sweeps.json 2> $O/rehearse2_sweeps.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; echo "alive $(( $(date +%s) - start ))s $(grep -c . $O/rehearse2_sweeps.json) json lines"; done
wait $pid; rc=$?; echo "rehearse rc=$rc wall=$(( $(date +%s) - start ))s"
python3 -c "
import json; d=json.loads([l for l in open('$O/rehearse2_sweeps.json').read().splitlines() if l.startswith('{')][-1])
print('graph', [(c['bytes'], c['replay_exact']) for c in d.get('size_sweep_graph_fp32', [])]); print('errors', d.get('leg_errors'), d.get('incomplete'))"
exit $rc
