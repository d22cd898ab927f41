#!/bin/bash
# r03: does the loopback structure (one transport stream per tick) capture forked?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03f; mkdir -p $O
for m in ${CMODES:-loop5 bcast3 gatherv3}; do
  DDL_LOG_LEVEL=${LL:-0} timeout -k 10 90 ./tools/bin/capture_engine $m 1 > $O/capture_engine_$m.log 2>&1
  rc=$?; echo "capture_engine $m forked rc=$rc"; tail -1 $O/capture_engine_$m.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
