#!/bin/bash
# r03: the thread-world broadcast / allgatherv with the posting trace (a segfault in r03h)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03i; mkdir -p $O
DDL_LOG_LEVEL=4 timeout -k 10 200 python -u -X faulthandler -m pytest tests/test_thread_world_gpu.py -q -x -k "broadcast_allgatherv or repeated or dropping" --timeout 150 --timeout-method thread > $O/pytest_bcast.log 2>&1
rc=$?; echo "rc=$rc"; grep -v "^  File" $O/pytest_bcast.log | tail -30
exit $rc
