#!/bin/bash
# Replay time of captured allreduces, single-stream DAG vs serial (tools/capture_overlap.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-capture_overlap}; mkdir -p $O
for w in local rccl; do
  timeout -k 10 200 python -u tools/capture_overlap.py $w 4 > $O/capture_overlap_${w}_P4.jsonl 2> $O/capture_overlap_${w}.err
  rc=$?; echo "$w rc=$rc"; cat $O/capture_overlap_${w}_P4.jsonl; [ $rc -ne 0 ] && { tail -5 $O/capture_overlap_${w}.err; exit $rc; }
done
timeout -k 10 200 python -u tools/capture_overlap.py local 8 > $O/capture_overlap_local_P8.jsonl 2>> $O/capture_overlap_local.err
rc=$?; echo "local P8 rc=$rc"; cat $O/capture_overlap_local_P8.jsonl
exit $rc
