#!/bin/bash
# Pack traffic (PMC, XCD-grouped tiles), fold cache policy at small sizes, pack / reduce tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02/pack
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_reduce_gpu.py tests/test_api_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/pack_tune.py > $O/pack_tune.txt 2>&1; echo "pack_tune rc=$?"; cat $O/pack_tune.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_$C -o pmc --output-format csv -- python3 tools/pack_tune.py child > $O/pmc_$C.out 2> $O/pmc_$C.err
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/pmc_$C.err; exit $rc; }
done
python3 scripts/prof_summarize.py $O
for V in 0 3; do
  DDL_FOLD_VARIANT=$V timeout -k 10 120 python3 tools/small_latency.py --no-loopback > $O/small_fold_v$V.jsonl 2>&1; echo "fold v$V rc=$?"
done
grep fold $O/small_fold_v*.jsonl
