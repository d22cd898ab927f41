#!/bin/bash
# r05 s16: the standalone reduce's size bands (kReduceBands, from the s15 A/Bs): the reduce tests
# (every band at full size, bit-exact), then the N=1 bench without the host / fusion / CPU legs (its
# sweep is where the bands show).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s16}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 500 python -u -m pytest tests/test_reduce_gpu.py -q --timeout 150 --timeout-method thread > $O/pytest_reduce.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_reduce.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python bench.py --no-host --no-fusion --no-cpu-baseline > $O/bench_sweep.json 2> $O/bench_sweep.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $O/bench_sweep.json
