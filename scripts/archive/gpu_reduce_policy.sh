#!/bin/bash
# reduce kernel cache bits per access (tools/reduce_policy_tune.hip, built on the CPU side)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02k; mkdir -p $O
for M in ${SIZES:-256 1024 64}; do
  timeout -k 10 120 ./tools/bin/reduce_policy_tune $M 5 > $O/reduce_policy_${M}MiB.txt 2>&1; rc=$?
  echo "bucket $M MiB rc=$rc"; cat $O/reduce_policy_${M}MiB.txt; [ $rc -eq 0 ] || exit $rc
done
