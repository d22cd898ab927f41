#!/bin/bash
# r03: capture diagnosis — the harness serially (control), then forked with the posting trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03b; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
for m in direct3 bcast3; do
  timeout -k 10 60 ./tools/bin/capture_engine $m 0 > $O/capture_serial_$m.log 2>&1
  rc=$?; echo "capture_engine $m serial rc=$rc"; tail -1 $O/capture_serial_$m.log
  if crashed $rc; then exit $rc; fi
done
DDL_LOG_LEVEL=4 timeout -k 10 60 ./tools/bin/capture_engine direct3 1 > $O/capture_forked_direct3.log 2>&1
rc=$?; echo "capture_engine direct3 forked rc=$rc"; tail -12 $O/capture_forked_direct3.log
exit $rc
