#!/bin/bash
# Quarter chunks at both ends of host transfers: host-path tests (one process and 2..8 processes),
# the taper / chunk A/B, then the bench's host legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-taper2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py tests/test_multiproc_gpu.py tests/test_configs_gpu.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^E |FAILED" $O/pytest.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/host_taper_ab.py > $O/host_taper_ab.jsonl 2> $O/host_taper_ab.err
rc=$?; [ $rc -ne 0 ] && { tail -5 $O/host_taper_ab.err; exit $rc; }
python3 -c "
import json, collections
d = collections.defaultdict(list)
for l in open('$O/host_taper_ab.jsonl'):
    r = json.loads(l); d[(r['leg'], r['host_taper'], r['chunk_MiB'])].append(r['ms'])
for k in sorted(d): print(k, d[k])
"
