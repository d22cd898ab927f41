#!/bin/bash
# Host keyed path: tests, then the C5 batch's engine-thread timeline vs copy threads / chunk size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-host_tl}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_api_gpu.py -q -x -k "keyed_host" --timeout 100 --timeout-method thread > $O/pytest_host.log 2>&1
rc=$?; echo "pytest host rc=$rc"; tail -2 $O/pytest_host.log; [ $rc -ne 0 ] && exit $rc
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/nproc.txt
timeout -k 10 500 python -u tools/host_keyed_threads.py > $O/host_threads.jsonl 2> $O/host_threads.err
rc=$?; echo "threads rc=$rc"; cat $O/host_threads.jsonl; cat $O/nproc.txt
exit $rc
