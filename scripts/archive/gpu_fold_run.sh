#!/bin/bash
# The fold's run form: parity tests, the bench's fold legs (run vs tile form), the kernel trace and
# FETCH / WRITE / SQ PMC passes of tools/fold_pmc.py (each pass its own SIGKILL timeout).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fold_run}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_reduce_gpu.py -q -x -k "fold" --timeout 120 --timeout-method thread > $O/pytest_fold.log 2>&1
rc=$?; echo "pytest fold rc=$rc"; tail -2 $O/pytest_fold.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_fold.log | head; exit $rc; }
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-sweep --no-host --no-fusion --no-cpu-baseline > $O/bench_fold.json 2> $O/bench_fold.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_fold.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'])
for k in ('fold_kernel','fold_kernel_reference_order','fold_kernel_tile_form','fold_kernel_fp16_c4'): print(k, json.dumps({x: d.get(k,{}).get(x) for x in ('kernel','us','achieved_GBs','frac_of_peak')}))
" || tail -5 $O/bench_fold.err; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/fold_trace -o trace --output-format csv -- python3 tools/fold_pmc.py > $O/fold_trace.log 2>&1
echo "fold trace rc=$?"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/fold_pmc_$C -o pmc --output-format csv -- python3 tools/fold_pmc.py > $O/fold_pmc_$C.log 2>&1
  echo "pmc $C rc=$?"
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -d $O/fold_pmc_sq -o pmc --output-format csv -- python3 tools/fold_pmc.py > $O/fold_pmc_sq.log 2>&1
echo "pmc sq rc=$?"
ls $O
exit 0
