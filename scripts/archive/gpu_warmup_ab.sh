# N=1 headline with short and long warm-ups / timed regions, interleaved (measurement only).
set -o pipefail
mkdir -p gpurun_out/s4
out=gpurun_out/s4/warmup_ab.txt; : > $out
for r in 1 2 3; do
  for cfg in "10 50" "200 50" "10 400" "300 300"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --warmup $1 --steps $2 --no-sweep --no-variants --no-host --no-fusion --no-cpu-baseline > gpurun_out/s4/w.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s4/w.json'));print('round $r warmup $1 steps $2', d['value'], d['roofline']['achieved'], d['roofline']['kernel_ms'], d['ms_per_step'])" >> $out
  done
done
cat $out
