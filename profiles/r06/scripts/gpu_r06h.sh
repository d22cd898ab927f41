#!/bin/bash
# r06 s9: the multi-rank RCCL tests as the suite runs them (pytest), then the bench's N>1 line over
# real multi-rank RCCL on one GPU (--rehearse-rccl) at N = 2, 4 and 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s9; mkdir -p $O
export NCCL_DEBUG=WARN DDL_MP_PROGRESS_FILE=$PWD/$O/progress.txt
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_multiproc_rccl_gpu.py > $O/pytest_mp_rccl.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; echo "alive: $(tail -1 $O/progress.txt 2>/dev/null)"; done
wait $pid; rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_mp_rccl.log | tail -12
case $rc in 0) ;; *) exit $rc;; esac
MODE=--rehearse-rccl NS="2 4 8" LIMIT=500 TAG=r06/s9 bash scripts/gpu_rehearse.sh
