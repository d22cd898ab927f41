#!/bin/bash
# rocprofv3 kernel traces: (1) the C5 fusion path of bench.py, (2) the single-GPU ring rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r01b}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/fusion -o fusion --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-sweep --no-variants --no-cpu-baseline --no-host > $OUT/bench_fusion.json 2> $OUT/fusion.err
rc=$?; echo "fusion trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/fusion.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ring -o ring --output-format csv -- python3 tools/local_ring_bench.py --ranks 2 8 --reps 3 > $OUT/local_ring.json 2> $OUT/ring.err
rc=$?; echo "ring trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/ring.err; exit $rc; }
timeout -k 10 300 python3 tools/local_ring_bench.py --ranks 2 4 8 --reps 5 > $OUT/local_ring_noprof.json 2> $OUT/ring_noprof.err
echo "ring noprof rc=$?"; cat $OUT/local_ring_noprof.json; cat $OUT/bench_fusion.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d.get('fusion_c5'))"
cat $OUT/fusion/fusion_kernel_stats.csv | cut -c1-200 | head -12
cat $OUT/ring/ring_kernel_stats.csv | cut -c1-200 | head -12
