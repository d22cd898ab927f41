#!/bin/bash
# Keyed host C5 (pageable and pinned) vs the CPU set the engine's threads run on (tools/numa_probe.py),
# interleaved: default / local (the GPU's NUMA node) / remote, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-numa}; mkdir -p $O
timeout -k 10 60 python3 tools/numa_probe.py topo > $O/numa.jsonl 2>> $O/numa.err
for rep in 1 2 3; do for m in default nobind local remote; do
  timeout -k 10 240 python3 tools/numa_probe.py run $m 7 >> $O/numa.jsonl 2>> $O/numa.err
  rc=$?; echo "$m rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/numa.err; exit $rc; }
done; done
cat $O/numa.jsonl
