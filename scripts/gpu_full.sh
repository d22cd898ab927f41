#!/bin/bash
# Full pass on the current tree: GPU suite + smoke + default N=1 bench, then the rocprofv3
# kernel trace / stats and FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_profile.sh).
# Usage: TAG=r03p bash scripts/gpu_full.sh     (SKIP_TESTS=1 / SKIP_PROF=1 to drop a part)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-full}
O=gpurun_out/$TAG; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1050 python -u -m pytest tests -m gpu -q --maxfail=25 --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_gpu rc=$rc"; tail -3 $O/pytest_gpu.log
  if crashed $rc; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
  if crashed $rc; then exit $rc; fi
fi
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $O/bench_n1.json; echo
if crashed $rc; then exit $rc; fi
if [ -z "$SKIP_PROF" ]; then TAG=$TAG bash scripts/gpu_profile.sh; fi
