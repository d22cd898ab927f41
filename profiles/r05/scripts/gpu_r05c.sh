#!/bin/bash
# r05 s3: the tests touched since s2, the batched fold's cache-policy A/B, the N=1 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s3}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py tests/test_batch_gpu.py tests/test_deployment_lib_gpu.py tests/test_api_collectives_gpu.py -q --timeout 150 --timeout-method thread > $O/pytest_sub.log 2>&1
rc=$?; echo "pytest_sub rc=$rc"; tail -3 $O/pytest_sub.log; grep -E '^FAILED|^ERROR' $O/pytest_sub.log | head
if crashed $rc; then exit $rc; fi
timeout -k 10 200 python3 tools/fold_batch_policy_ab.py > $O/fold_batch_policy_ab.json 2> $O/fold_batch_policy_ab.err
rc=$?; echo "policy ab rc=$rc"; cat $O/fold_batch_policy_ab.json
if crashed $rc; then tail $O/fold_batch_policy_ab.err; exit $rc; fi
timeout -k 10 500 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"
python3 -c "
import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
print('value', d['value'], d['roofline']['frac']); s=d.get('keyed_host_c5_steady', {})
print({k: (v.get('median_ms'), v.get('p90_ms'), v.get('last_ms')) for k, v in s.items() if isinstance(v, dict)})
print({k: d[k]['ms'] for k in ('keyed_host_c5', 'keyed_host_c5_pinned', 'keyed_host_c5_registered') if k in d})"
