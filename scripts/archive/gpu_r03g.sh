#!/bin/bash
# r03: fold kernel shapes (buffer form, input skews) at the bench's chunk sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03g; mkdir -p $O
for args in "32 5 0" "32 5 4096" "32 5 69632" "2 7 0" "4 5 0"; do
  set -- $args
  timeout -k 10 120 ./tools/bin/fold_tune $1 $2 $3 > $O/fold_tune_${1}MiB_skew$3.txt 2>&1; rc=$?
  echo "chunk $1 MiB skew $3 rc=$rc"; cat $O/fold_tune_${1}MiB_skew$3.txt; [ $rc -eq 0 ] || exit $rc
done
