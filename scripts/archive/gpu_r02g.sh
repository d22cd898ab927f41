#!/bin/bash
# r02 (session 3): full -m gpu suite on the current tree (direct-gather + graph commits), then the
# default N=1 bench line and an N=4 rehearsal. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 ${PT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_n1.err; exit $rc; }
N=4 RT=300 PORT=29556 bash scripts/rehearse_multi.sh; rc=$?
cp gpurun_out/rehearse4.json gpurun_out/rehearse4.err $O/ 2>/dev/null
exit $rc
