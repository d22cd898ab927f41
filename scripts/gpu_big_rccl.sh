#!/bin/bash
# The whole multi-process worker at P = 5 and 8 over real multi-rank RCCL on one GPU (the suite runs
# it at P <= 4; DDL_TEST_RCCL_BIG=1 adds these), as pytest runs it; heartbeat + per-check progress.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-big_rccl}; mkdir -p $O
export NCCL_DEBUG=WARN DDL_TEST_RCCL_BIG=1 DDL_MP_PROGRESS_FILE=$PWD/$O/progress.txt
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests/test_multiproc_rccl_gpu.py -k "engine_over_multirank_rccl and (5 or 8)" > $O/pytest_big.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; echo "alive: $(tail -1 $O/progress.txt 2>/dev/null)"; done
wait $pid; rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed" $O/pytest_big.log | tail -5
exit $rc
