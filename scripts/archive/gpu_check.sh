#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, bench (N=1), bench N>1 code path at world 1.
# Stops at the first crash-class exit (fault / abort / segfault / timeout); a plain test failure
# (pytest exit 1) continues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -q --maxfail=25 --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if crashed $rc; then exit $rc; fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.json; tail -5 gpurun_out/bench.err
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python bench.py --force-multi --steps 10 --warmup 3 > gpurun_out/bench_multi1.json 2> gpurun_out/bench_multi1.err
rc=$?; echo "bench force-multi rc=$rc"; tail -c 2500 gpurun_out/bench_multi1.json; tail -5 gpurun_out/bench_multi1.err
exit $rc
