#!/bin/bash
# r03: API + graph GPU tests, verbose
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_api_gpu.py tests/test_graph_gpu.py tests/test_reduce_gpu.py -v -x --timeout 100 --timeout-method thread > $O/pytest_api.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "FAILED|Error|assert |Timeout" $O/pytest_api.log | head -30; tail -5 $O/pytest_api.log
exit $rc
