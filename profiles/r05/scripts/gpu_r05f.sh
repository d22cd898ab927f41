#!/bin/bash
# r05 s10: after the size-1 handler fix (its data-plane pointer no longer owns the communicator):
# the whole GPU suite + smoke (the world communicator at size 1 is now destroyed at finalize),
# then the soaks that found the leak (tools/soak_mp.py, P = 5 and 8): thread counts must stay flat.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s10}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=25 --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 $O/pytest_gpu.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
if crashed $rc; then exit $rc; fi
timeout -k 10 400 python3 tools/soak_mp.py 5 20 > $O/soak5.log 2>&1
rc=$?; echo "soak5 rc=$rc"; tail -3 $O/soak5.log
if crashed $rc; then exit $rc; fi
timeout -k 10 400 python3 tools/soak_mp.py 8 8 > $O/soak8.log 2>&1
rc=$?; echo "soak8 rc=$rc"; tail -3 $O/soak8.log
