#!/bin/bash
# DAG capture (capture_mode 2): the graph tests first (a crash stops here), then the whole GPU suite + smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-dag}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -u -X faulthandler -m pytest tests/test_graph_gpu.py -v -x --timeout 120 --timeout-method thread > $O/pytest_graph.log 2>&1
rc=$?; echo "pytest graph rc=$rc"; grep -E "FAILED|Error|passed|failed" $O/pytest_graph.log | tail -8
if [ $rc -ne 0 ]; then tail -40 $O/pytest_graph.log; exit $rc; fi
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; grep -E "FAILED" $O/pytest_gpu.log | head; tail -2 $O/pytest_gpu.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
exit $rc
