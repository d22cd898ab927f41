#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02n; mkdir -p $O
for M in 32 4 1; do
  timeout -k 10 120 ./tools/bin/fold_tune $M 5 > $O/fold_tune_${M}MiB.txt 2>&1 || exit 1
  grep -E "shipped|plain|write-through|NT loads  " $O/fold_tune_${M}MiB.txt
done
