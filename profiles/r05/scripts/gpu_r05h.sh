#!/bin/bash
# r05 s12: communicators are destroyed off the handler's own threads (CommunicatorDeleter): the
# API / multi-process / thread-world tests, then a P = 5 soak (size-1 splits detached every round).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s12}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py tests/test_api_collectives_gpu.py tests/test_multiproc_gpu.py tests/test_deployment_lib_gpu.py -q --timeout 150 --timeout-method thread > $O/pytest_sub.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_sub.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python3 tools/soak_mp.py 5 10 > $O/soak5.log 2>&1
rc=$?; echo "soak5 rc=$rc"; tail -3 $O/soak5.log
