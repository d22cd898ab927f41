#!/bin/bash
# Single-stream DAG posting under capture (tools/capture_replay.hip flag D): the engine's forked
# P = 3 direct program (whose forked-stream capture segfaults in hipStreamEndCapture)
# replayed with every op on the origin stream and its dependencies set explicitly.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-capture_dag}; mkdir -p $O
for f in DCK DC DK D; do
  timeout -k 10 60 ./tools/bin/capture_replay tools/traces/engine_trace_direct3_forked.txt $f > $O/replay_$f.log 2>&1
  rc=$?; echo "replay $f rc=$rc"; tail -3 $O/replay_$f.log
  case $rc in 0|1) ;; *) exit $rc;; esac
done
exit 0
