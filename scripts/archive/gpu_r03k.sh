#!/bin/bash
# r03: the multi-process engine checks (new: config mismatch, keyed-round order) at P = 2 and 3, verbose
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03k; mkdir -p $O
DDL_MP_TIMEOUT=60 timeout -k 10 400 python -u -m pytest tests/test_multiproc_gpu.py -v -s -x -k "2-1 or 3-1" --timeout 300 --timeout-method thread > $O/pytest_mp.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "PASSED|FAILED|Error|error|assert|\[P=" $O/pytest_mp.log | tail -40
exit $rc
