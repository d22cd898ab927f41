#!/bin/bash
# rocprofv3 summaries of the N=1 bench: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950). Plus the reduce tuning harness.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BARGS="--steps 30 --warmup 5 --no-sweep --no-cpu-baseline --no-forced-data-plane --no-host-steady ${EXTRA_BARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py $BARGS > $OUT/bench_trace.json 2> $OUT/trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/trace.err; exit $rc; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$C -o pmc --output-format csv -- python3 bench.py $BARGS > $OUT/bench_$C.json 2> $OUT/pmc_$C.err
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/pmc_$C.err; exit $rc; }
done
if [ -x tools/bin/reduce_tune ]; then
  timeout -k 10 300 tools/bin/reduce_tune 256 5 > $OUT/tune_256.txt 2>&1; echo "tune256 rc=$?"
  timeout -k 10 300 tools/bin/reduce_tune 1024 3 > $OUT/tune_1024.txt 2>&1; echo "tune1024 rc=$?"
  cat $OUT/tune_256.txt | head -50
fi
python3 scripts/prof_summarize.py $OUT
find $OUT -type f | head -30
