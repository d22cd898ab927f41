#!/bin/bash
# r02 session 5: GPU suite + smoke + N=1 bench on the current tree, then the DP overlap probe.
# Stops at the first crash-class exit (fault / abort / segfault / timeout); a plain test failure
# (pytest exit 1) continues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s5; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 ${PYTEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -q --maxfail=25 --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -5 $O/pytest_gpu.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log
if crashed $rc; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench_n1.json; tail -3 $O/bench_n1.err
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -u tools/dp_overlap_probe.py > $O/dp_overlap.json 2> $O/dp_overlap.err
rc=$?; echo "dp_overlap rc=$rc"; cat $O/dp_overlap.json; tail -3 $O/dp_overlap.err
exit $rc
