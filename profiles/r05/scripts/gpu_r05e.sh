#!/bin/bash
# r05 s9: the tests added after s8 (the DP example on the deployment library), then a soak of the
# N>1 engine on one GPU with the native completion groups (tools/soak_mp.py, P = 5 and 8).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s9}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_examples_gpu.py tests/test_deployment_lib_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest_examples.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_examples.log
if crashed $rc; then exit $rc; fi
timeout -k 10 400 python3 tools/soak_mp.py 5 20 > $O/soak5.log 2>&1
rc=$?; echo "soak5 rc=$rc"; tail -3 $O/soak5.log
if crashed $rc; then exit $rc; fi
timeout -k 10 400 python3 tools/soak_mp.py 8 8 > $O/soak8.log 2>&1
rc=$?; echo "soak8 rc=$rc"; tail -3 $O/soak8.log
