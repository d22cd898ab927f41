#!/bin/bash
# hipGraph capture probe: one mode per process, continue past crashes of the probe itself
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02f; mkdir -p $O
for m in ${MODES:-fold ring2 rawlocal}; do
  timeout -k 10 90 python -u -X faulthandler tools/graph_probe.py $m > $O/probe_$m.log 2>&1
  rc=$?; echo "probe $m rc=$rc"; grep -v "^  File\|^Thread\|^Extension\|^$\|Current thread\|amdgpu.ids" $O/probe_$m.log | tail -8
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
done
exit 0
