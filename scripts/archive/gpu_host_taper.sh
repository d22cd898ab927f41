#!/bin/bash
# Tapered final host chunks: host-path tests (one process and 2..8 processes), then the bench's host legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-taper}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py tests/test_multiproc_gpu.py tests/test_configs_gpu.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^E |FAILED" $O/pytest.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-sweep --no-variants --no-cpu-baseline > $O/tl.json 2> $O/tl.err
rc=$?; python3 -c "
import json; d=json.loads(open('$O/tl.json').read().strip().splitlines()[-1])
for k in ('host_resident','keyed_host_c5','keyed_host_c5_pinned','keyed_host_c5_registered'): print(k, d[k]['ms'], d[k].get('engine_thread'))
"; exit $rc
