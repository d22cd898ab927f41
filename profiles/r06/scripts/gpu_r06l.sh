#!/bin/bash
# r06 s18: hipGraph capture over real multi-rank RCCL (P = 2, 3), then the N = 2 line over it with
# the size sweeps on (eager and graph-captured, replayed sums checked).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s18; mkdir -p $O
export NCCL_DEBUG=WARN
timeout -k 10 500 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_multiproc_rccl_gpu.py -k graph_capture > $O/pytest_graph_rccl.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; echo "alive $(grep -c . $O/pytest_graph_rccl.log) lines"; done
wait $pid; rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error|assert" $O/pytest_graph_rccl.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 2 --rehearse-rccl --steps 3 --warmup 1 --bucket-mib 8 --no-config-sweep --size-sweep-max-mib 16 > $O/rehearse2_sweeps.json 2> $O/rehearse2_sweeps.err
rc=$?; echo "rehearse rc=$rc"
python3 -c "
import json; d=json.loads([l for l in open('$O/rehearse2_sweeps.json').read().splitlines() if l.startswith('{')][-1])
print('graph', d.get('size_sweep_graph_fp32')); print('eager', [(c['bytes'], c['us'], c.get('schedule')) for c in d.get('size_sweep_fp32', [])]); print('errors', d.get('leg_errors'))"
exit $rc
