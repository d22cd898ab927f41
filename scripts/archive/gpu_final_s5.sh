#!/bin/bash
# r02 s5 closing pass: GPU suite + smoke + N=1 bench (scripts/gpu_s5.sh, without the overlap
# probe), then rocprofv3 kernel trace + stats and the FETCH_SIZE / WRITE_SIZE PMC passes of the
# N=1 bench (scripts/gpu_profile.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=25 --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 $O/pytest_gpu.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
if crashed $rc; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $O/bench_n1.json
if crashed $rc; then exit $rc; fi
TAG=r02s5 bash scripts/gpu_profile.sh
