#!/bin/bash
# host-side placement probe for the keyed host-tensor path (tools/numa_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 120 python tools/numa_probe.py topo 2>/dev/null | tee $O/numa.jsonl || exit $?
for spec in "default 7" "local 7" "remote 7" "local 15" "default 15"; do
  timeout -k 10 240 python tools/numa_probe.py run $spec 2>>$O/numa.err | tee -a $O/numa.jsonl
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 $O/numa.err; exit $rc; }
done
