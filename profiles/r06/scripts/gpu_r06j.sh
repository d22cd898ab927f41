#!/bin/bash
# r06 s12: C3 and the P = 5 pre-fold at full size over real multi-rank RCCL on one GPU, by hash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s12; mkdir -p $O
export NCCL_DEBUG=WARN
timeout -k 10 700 python -u -m pytest -v --timeout 320 --timeout-method thread "tests/test_multiproc_rccl_gpu.py::test_full_size_hash_equals_mpich_over_multirank_rccl" > $O/pytest_fullsize_rccl.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; echo "alive $(grep -c . $O/pytest_fullsize_rccl.log) lines"; done
wait $pid; rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" $O/pytest_fullsize_rccl.log | tail -8
exit $rc
