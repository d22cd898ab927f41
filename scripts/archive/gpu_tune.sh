#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune
for S in ${SIZES:-256 1024 64}; do
  timeout -k 10 300 tools/bin/reduce_tune $S ${ROUNDS:-5} > gpurun_out/tune/tune_$S.txt 2>&1
  rc=$?; echo "tune $S rc=$rc"; head -${TOP:-25} gpurun_out/tune/tune_$S.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
