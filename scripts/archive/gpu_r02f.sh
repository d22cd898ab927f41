#!/bin/bash
# r02 (session 2): capture-pattern mimic, graph probes, graph-capture tests, N=1 bench with the
# hipGraph sweep column, N=2 rehearsal. Stops at the first crash-class exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02f
mkdir -p $O
for T in 1 2; do
  timeout -k 5 30 ./tools/bin/capture_patterns 9 $T > $O/pattern_9_$T.log 2>&1; echo "pattern 9 T=$T rc=$?"; tail -2 $O/pattern_9_$T.log
done
MODES="ring2 local fold gather loop" bash scripts/gpu_graph_probe.sh || exit $?
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_graph.log 2>&1
rc=$?; echo "pytest graph rc=$rc"; tail -15 $O/pytest_graph.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-variants --no-host --no-fusion --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json;d=json.load(open('$O/bench.json'))
for p in d['sweep_fp32']: print(p)" ; [ $rc -eq 0 ] || exit $rc
N=2 RT=400 bash scripts/rehearse_multi.sh; rc=$?
cp gpurun_out/rehearse2.json gpurun_out/rehearse2.err $O/ 2>/dev/null
python3 -c "
import json;d=json.load(open('$O/rehearse2.json'));print(d.get('leg_errors'), d.get('size_sweep_graph_fp32'))"
exit $rc
