#!/bin/bash
# r06 s11: the DP example as two processes over a real two-rank RCCL communicator (deployment
# library), then bench.py --gpus 8 --rehearse-rccl with a watchdog long enough for every leg over
# sockets on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s11; mkdir -p $O
export NCCL_DEBUG=WARN
timeout -k 10 330 python -u -m pytest -v --timeout 320 --timeout-method thread "tests/test_multiproc_rccl_gpu.py::test_data_parallelism_example_over_two_rccl_ranks" > $O/pytest_dp_example.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" $O/pytest_dp_example.log | tail -5
[ $rc -ne 0 ] && exit $rc
MODE=--rehearse-rccl NS="8" LIMIT=900 EXTRA="--watchdog-s 840" TAG=r06/s11 bash scripts/gpu_rehearse.sh
