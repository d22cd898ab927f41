#!/bin/bash
# r03: the anchor fix for forked captures — the raw trace replay with anchors, then the engine's
# own programs captured forked from C++ and from torch. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03d; mkdir -p $O
T=profiles/r03/graph/engine_trace_direct3_forked.txt
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
for fl in CKA ECKA; do
  timeout -k 10 60 ./tools/bin/capture_replay $T $fl > $O/replay_$fl.log 2>&1
  rc=$?; echo "replay $fl rc=$rc"; tail -1 $O/replay_$fl.log
  [ $rc -ne 0 ] && exit $rc
done
for m in direct3 ring2 bcast3 gatherv3 loop5; do
  timeout -k 10 90 ./tools/bin/capture_engine $m 1 > $O/capture_engine_$m.log 2>&1
  rc=$?; echo "capture_engine $m forked rc=$rc"; tail -1 $O/capture_engine_$m.log
  [ $rc -ne 0 ] && exit $rc
done
for m in local ring2 loop rawlocal; do
  timeout -k 10 120 python -u -X faulthandler tools/graph_probe.py $m 1 1 > $O/probe_forked_$m.log 2>&1
  rc=$?; echo "probe $m forked rc=$rc"; grep -v "^  File\|^Thread\|^Extension\|^$\|Current thread\|amdgpu.ids" $O/probe_forked_$m.log | tail -4
  [ $rc -ne 0 ] && exit $rc
done
exit 0
