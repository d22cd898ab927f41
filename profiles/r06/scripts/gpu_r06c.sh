#!/bin/bash
# r06 s3: first multi-rank RCCL communicators on one GPU (NCCL_HOSTID per process, socket transport
# over loopback): a P = 2 probe of the known answers, then the whole worker at P = 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s3; mkdir -p $O
export NCCL_DEBUG=WARN
timeout -k 10 240 python -u -c "
import sys, time; sys.path.insert(0, 'tests')
import test_multiproc_rccl_gpu as t
t0 = time.time(); t._run(2, ['check_reference_known_answers'], timeout=180); print('probe P=2 ok', round(time.time() - t0, 1), 's')
" > $O/probe2.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -30 $O/probe2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread "tests/test_multiproc_rccl_gpu.py::test_engine_over_multirank_rccl[2]" > $O/pytest_p2.log 2>&1
rc=$?; echo "pytest P=2 rc=$rc"; tail -30 $O/pytest_p2.log
exit $rc
