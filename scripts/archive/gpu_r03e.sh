#!/bin/bash
# r03: which capture shapes does HIP accept (tools/capture_patterns.hip 10-13); stops at the first crash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03e; mkdir -p $O
for k in ${PATS:-10 13 11 12}; do
  timeout -k 10 60 ./tools/bin/capture_patterns $k 3 > $O/pattern_$k.log 2>&1
  rc=$?; echo "pattern $k rc=$rc"; tail -1 $O/pattern_$k.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
