#!/bin/bash
# r06 s4: multi-rank RCCL on one GPU (per-rank NCCL_HOSTID, RCCL's socket transport over loopback):
# the transport RCCL picked (NCCL_DEBUG=INFO, P = 2), the whole multi-process worker at
# P = 2, 3, 4, 5, 8, then the bench's N>1 line over it at N = 2 and 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s4; mkdir -p $O
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,NET timeout -k 10 200 python -u -c "
import sys; sys.path.insert(0, 'tests')
import test_multiproc_rccl_gpu as t
t._run(2, ['check_reference_known_answers'], timeout=150); print('probe P=2 ok')
" > $O/probe2_nccl_info.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -E "via NET|NET/|Channel 00|nRanks|probe" $O/probe2_nccl_info.log | head -20
[ $rc -ne 0 ] && exit $rc
export NCCL_DEBUG=WARN
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_multiproc_rccl_gpu.py > $O/pytest_mp_rccl.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_mp_rccl.log | tail -12
case $rc in 0|1) ;; *) exit $rc;; esac
MODE=--rehearse-rccl NS="2 8" LIMIT=400 TAG=r06/s4 bash scripts/gpu_rehearse.sh
