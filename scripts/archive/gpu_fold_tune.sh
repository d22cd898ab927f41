#!/bin/bash
# fold kernel tile shapes and cache policies (tools/fold_tune.hip, built on the CPU side)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02h; mkdir -p $O
for M in 32 128 4 1; do
  timeout -k 10 120 ./tools/bin/fold_tune $M 5 > $O/fold_tune_${M}MiB.txt 2>&1; rc=$?
  echo "chunk $M MiB rc=$rc"; cat $O/fold_tune_${M}MiB.txt; [ $rc -eq 0 ] || exit $rc
done
