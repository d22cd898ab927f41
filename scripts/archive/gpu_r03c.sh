#!/bin/bash
# r03: bisect the forked-capture crash by replaying the engine's posting trace with fresh objects,
# simplest first; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03c; mkdir -p $O
T=profiles/r03/graph/engine_trace_direct3_forked.txt
for fl in ${FLAGS:-CK:1,2,4,6,8,9,12,13,14,22 CK:1,2,4,6,8,9,13,14,23 CK:1,2,4,6,8,9,13,14,22,23 CK:1,2,4,6,8,9,12,13,14,22,23}; do
  timeout -k 10 60 ./tools/bin/capture_replay $T $fl > $O/replay_$fl.log 2>&1
  rc=$?; echo "replay $fl rc=$rc"; tail -2 $O/replay_$fl.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
