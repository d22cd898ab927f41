#!/bin/bash
# CU-mask tests (thread world, loopback) and the CU-mask probe with pack / unpack.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-cum}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_thread_world_gpu.py tests/test_rccl_loopback_gpu.py -q -x --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^E |FAILED" $O/pytest.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/cu_mask_probe.py > $O/cu_mask_probe3.jsonl 2> $O/probe.err
rc=$?; cat $O/cu_mask_probe3.jsonl; exit $rc
