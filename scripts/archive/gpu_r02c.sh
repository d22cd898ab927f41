#!/bin/bash
# r02 profiles: rocprofv3 kernel stats + PMC of the N=1 bench (scripts/gpu_profile.sh), pack XCD
# grouping A/B, keyed host C5 vs memcpy threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r02 bash scripts/gpu_profile.sh || exit 1
O=gpurun_out/r02/pack
mkdir -p $O
for X in 1 0 1 0; do
  DDL_PACK_XCD=$X VARIANTS=1 timeout -k 10 200 python3 tools/pack_tune.py >> $O/pack_xcd_ab.txt 2>&1; echo "xcd=$X rc=$?" >> $O/pack_xcd_ab.txt
done
cat $O/pack_xcd_ab.txt
timeout -k 10 300 python3 tools/host_keyed_threads.py > gpurun_out/r02/host_keyed_threads.jsonl 2>&1; echo "host threads rc=$?"
cat gpurun_out/r02/host_keyed_threads.jsonl
