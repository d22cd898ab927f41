#!/bin/bash
# write-through vs non-temporal stores in the pack / unpack and fold kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02m; mkdir -p $O
for R in 1 2; do
  for S in 0 1; do
    echo "pack_store=$S round=$R" >> $O/pack_store_ab.txt
    DDL_PACK_STORE=$S VARIANTS=1 timeout -k 10 200 python3 tools/pack_tune.py >> $O/pack_store_ab.txt 2>&1 || exit 1
  done
done
cat $O/pack_store_ab.txt
for M in 32 4; do
  timeout -k 10 120 ./tools/bin/fold_tune $M 5 > $O/fold_tune_${M}MiB.txt 2>&1 || exit 1
  grep -E "shipped|plain|write-through|NT loads  " $O/fold_tune_${M}MiB.txt
done
