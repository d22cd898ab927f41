#!/bin/bash
# N=1 bench with 128- and 256-lane reduce workgroups, interleaved (measurement only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune
for r in 1 2; do
  for t in 256 128 64; do
    DDL_REDUCE_THREADS=$t timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-sweep --no-host --no-fusion --no-cpu-baseline > gpurun_out/tune/thr_${t}_$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/tune/thr_${t}_$r.json'));print('threads $t round $r', d['roofline']['achieved'], d['variants_achieved_GBs'], d['reduce_half_dtypes_achieved_GBs'])"
  done
done
