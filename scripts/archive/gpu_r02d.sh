#!/bin/bash
# pack with the one-byte tile index: tests, speed, PMC traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02/pack2
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_reduce_gpu.py -k pack tests/test_api_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do VARIANTS=1 timeout -k 10 200 python3 tools/pack_tune.py >> $O/pack_tune.txt 2>&1; done; cat $O/pack_tune.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_$C -o pmc --output-format csv -- python3 tools/pack_tune.py child > $O/pmc_$C.out 2> $O/pmc_$C.err
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/pmc_$C.err; exit $rc; }
done
python3 scripts/prof_summarize.py $O
