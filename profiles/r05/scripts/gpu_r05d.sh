#!/bin/bash
# r05 s4: the keyed-path GPU tests after the completion-group change, then the N = 2, 4, 8
# rehearsals of the N>1 bench line (every leg, CPU baselines at P = N) on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s4}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_api_gpu.py tests/test_api_collectives_gpu.py tests/test_deployment_lib_gpu.py -q --timeout 150 --timeout-method thread > $O/pytest_sub.log 2>&1
rc=$?; echo "pytest_sub rc=$rc"; tail -3 $O/pytest_sub.log; grep -E '^FAILED|^ERROR' $O/pytest_sub.log | head
if crashed $rc; then exit $rc; fi
TAG=${TAG:-r05s4} LIMIT=420 bash scripts/gpu_rehearse.sh
