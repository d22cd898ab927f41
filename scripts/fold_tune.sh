mkdir -p gpurun_out/tune
timeout -k 10 200 tools/bin/reduce_tune 1024 3 > gpurun_out/tune/tune_1024.txt 2>&1 || exit 1
timeout -k 10 200 tools/bin/reduce_tune 256 5 > gpurun_out/tune/tune_256.txt 2>&1 || exit 1
for v in 0 1 2 3 0; do
  DDL_FOLD_VARIANT=$v timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-sweep --no-host --no-fusion --no-cpu-baseline > gpurun_out/tune/fold_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/tune/fold_$v.json'));print('fold variant $v', d['fold_kernel']['achieved_GBs'])"
done
head -14 gpurun_out/tune/tune_1024.txt
head -14 gpurun_out/tune/tune_256.txt
