#!/bin/bash
# r04 s2: the new GPU tests (control link lost mid-round, registration-cache address reuse, the
# thread world over RCCL, the keyed host data plane) and the C4 batched fold form A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04s2; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_multiproc_gpu.py::test_control_link_lost_mid_round \
    tests/test_api_gpu.py::test_registration_cache_address_reuse tests/test_thread_world_rccl_gpu.py \
    tests/test_api_gpu.py::test_keyed_host_requests_data_plane -m gpu -v --timeout 200 --timeout-method thread \
    --durations=10 > $O/new_tests.log 2>&1
rc=$?; tail -30 $O/new_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python tools/host_numa_ab.py > $O/host_numa_ab.jsonl 2>&1
rc2=$?; tail -8 $O/host_numa_ab.jsonl
[ $rc -ne 0 ] && exit $rc
exit $rc2
