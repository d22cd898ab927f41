#!/bin/bash
# fold kernel cache-policy variants on the N=1 bench's fold leg (measurement only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune
for r in 1 2; do
  for v in ${FOLD_VARIANTS:-3 0}; do
    DDL_FOLD_VARIANT=$v timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-sweep --no-host --no-fusion --no-cpu-baseline > gpurun_out/tune/fold_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/tune/fold_$v.json'));print('fold variant $v round $r', d['fold_kernel'])"
  done
done
