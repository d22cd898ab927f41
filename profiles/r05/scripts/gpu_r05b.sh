#!/bin/bash
# r05 s2: the GPU suite and smoke on the split libraries (tests drive libddl_amd_testing.so,
# test_deployment_lib_gpu.py the deployment library alone).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s2}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=25 --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -5 $O/pytest_gpu.log
grep -E 'FAILED|ERROR' $O/pytest_gpu.log | head -30
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
