#!/bin/bash
# r03: new GPU tests (thread world, C2 sizes, host keyed modes, multi-process with the config and
# round-order checks), fold tuning, the N=1 bench; then the loop-mode forked capture probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03h; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_thread_world_gpu.py tests/test_reduce_gpu.py tests/test_api_gpu.py tests/test_multiproc_gpu.py tests/test_graph_gpu.py -q -x --timeout 240 --timeout-method thread > $O/pytest_new.log 2>&1
rc=$?; echo "pytest new rc=$rc"; tail -15 $O/pytest_new.log
if crashed $rc; then exit $rc; fi
bash scripts/gpu_r03g.sh > $O/fold_tune.log 2>&1; rc=$?; echo "fold tune rc=$rc"; grep -E "chunk|fold_buf|shipped|T64 U1 pol3" $O/fold_tune.log
if crashed $rc; then exit $rc; fi
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'])
for k in ('fold_kernel','fold_kernel_fp16_c4'): print(k, d.get(k,{}).get('frac_of_peak'), d.get(k,{}).get('us'))
for k in ('keyed_host_c5','keyed_host_c5_pinned','keyed_host_c5_pinned_direct_dma','keyed_host_c5_registered'): print(k, d.get(k,{}).get('ms'), d.get(k,{}).get('device_unpack_plans_per_step'))
" || tail -20 $O/bench_n1.err
if crashed $rc; then exit $rc; fi
timeout -k 10 60 ./tools/bin/capture_patterns 14 > $O/pattern_14.log 2>&1; echo "pattern 14 (minimal EndCapture crash) rc=$?"; tail -3 $O/pattern_14.log
