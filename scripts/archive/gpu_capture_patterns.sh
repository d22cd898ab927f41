#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02f; mkdir -p $O
for k in ${PATTERNS:-1 2 3 4 6 7 5 8}; do
  timeout -k 5 30 ./tools/bin/capture_patterns $k > $O/pattern_$k.log 2>&1
  rc=$?; echo "pattern $k rc=$rc"; tail -3 $O/pattern_$k.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
