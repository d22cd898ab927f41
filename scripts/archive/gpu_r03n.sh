#!/bin/bash
# r03: host keyed legs after the merged registration (bench N=1, no sweep), the fold's rocprof
# kernel trace + PMC passes (one block per pass; each under its own SIGKILL timeout)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_api_gpu.py -q -x -k "keyed_host_requests_data_plane" --timeout 100 --timeout-method thread > $O/pytest_host.log 2>&1
rc=$?; echo "pytest host rc=$rc"; tail -3 $O/pytest_host.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-sweep --no-variants --no-cpu-baseline > $O/bench_host.json 2> $O/bench_host.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_host.json').read().strip().splitlines()[-1])
for k in ('keyed_host_c5','keyed_host_c5_pinned','keyed_host_c5_pinned_direct_dma','keyed_host_c5_registered'): print(k, json.dumps({x: d.get(k,{}).get(x) for x in ('ms','device_unpack_plans_per_step','host_registered_bytes','host_register_failures')}))
"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/fold_trace -o trace --output-format csv -- python3 tools/fold_pmc.py > $O/fold_trace.log 2>&1
echo "fold trace rc=$?"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -d $O/fold_pmc_sq -o pmc --output-format csv -- python3 tools/fold_pmc.py > $O/fold_pmc_sq.log 2>&1
echo "pmc sq rc=$?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fold_pmc_fetch -o pmc --output-format csv -- python3 tools/fold_pmc.py > $O/fold_pmc_fetch.log 2>&1
echo "pmc fetch rc=$?"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/fold_pmc_write -o pmc --output-format csv -- python3 tools/fold_pmc.py > $O/fold_pmc_write.log 2>&1
echo "pmc write rc=$?"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_BUSY_max --kernel-trace -d $O/fold_pmc_grbm -o pmc --output-format csv -- python3 tools/fold_pmc.py > $O/fold_pmc_grbm.log 2>&1
echo "pmc grbm rc=$?"
find $O -name "*.csv" | head -20
exit 0
