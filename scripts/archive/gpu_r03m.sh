#!/bin/bash
# r03: the whole GPU suite, smoke, the N=1 bench, the spawned 4-rank rehearsal; then the
# minimal EndCapture reproducer (expected to segfault: last).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03m; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; grep -E "FAILED" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
if crashed $rc; then exit $rc; fi
timeout -k 10 600 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'kernel_ms', d['roofline']['kernel_ms'])
for k in ('fold_kernel','fold_kernel_reference_order','fold_kernel_fp16_c4'): print(k, d.get(k,{}).get('frac_of_peak'), d.get(k,{}).get('us'))
for k in ('keyed_host_c5','keyed_host_c5_pinned','keyed_host_c5_pinned_direct_dma','keyed_host_c5_registered'): print(k, d.get(k,{}).get('ms'), d.get(k,{}).get('device_unpack_plans_per_step'))
print('cpu_baseline', d.get('cpu_baseline'))
" || tail -20 $O/bench_n1.err
if crashed $rc; then exit $rc; fi
timeout -k 10 500 python3 bench.py --gpus 4 --rehearse --steps 3 --warmup 1 --no-size-sweep --no-config-sweep > $O/rehearse4_spawn.json 2> $O/rehearse4_spawn.err
rc=$?; echo "rehearse4 spawn rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/rehearse4_spawn.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'transport', d.get('transport'), 'parity', d.get('parity_vs_mpich_order'))" || tail -5 $O/rehearse4_spawn.err
if crashed $rc; then exit $rc; fi
timeout -k 10 60 ./tools/bin/capture_patterns 14 > $O/pattern_14.log 2>&1; echo "pattern 14 (minimal EndCapture crash) rc=$?"; tail -3 $O/pattern_14.log
exit 0
