#!/bin/bash
# Negotiation latency A/B on the GPU box's host cores (no GPU use): the star control channel
# (current library) vs the r02 ring (tools/bin/ring_lib, built from the commit before the star).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/neg_ab; mkdir -p $O
RING=$PWD/tools/bin/ring_lib/libddl_amd.so
for rep in 1 2; do
  for kind in star ring; do
    if [ $kind = ring ]; then export ddl_lib=$RING; else unset ddl_lib; fi
    NEG_KEYS=1 NEG_ROUNDS=500 timeout -k 10 120 python tools/negotiation_bench.py 2 4 8 16 > $O/${kind}_1key_$rep.json 2>&1 || exit 1
    NEG_KEYS=4096 NEG_ROUNDS=20 timeout -k 10 120 python tools/negotiation_bench.py 2 4 8 > $O/${kind}_4096keys_$rep.json 2>&1 || exit 1
    echo "$kind rep $rep"; cat $O/${kind}_1key_$rep.json $O/${kind}_4096keys_$rep.json
  done
done
