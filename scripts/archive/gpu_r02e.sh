#!/bin/bash
# pack: byte vs int32 tile index on one box, and the reduce kernel as a box-speed reference
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02/pack2
mkdir -p $O
for I in 8 32 8 32; do
  echo "index=$I" >> $O/pack_index_ab2.txt
  DDL_PACK_INDEX=$I VARIANTS=1 timeout -k 10 200 python3 tools/pack_tune.py >> $O/pack_index_ab2.txt 2>&1 || exit 1
done
cat $O/pack_index_ab2.txt
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-sweep --no-variants --no-host --no-fusion --no-cpu-baseline > $O/bench_ref.json 2>/dev/null; echo "bench rc=$?"
python3 -c "import json;d=json.load(open('$O/bench_ref.json'));print('reduce kernel', d['roofline']['achieved'])"
