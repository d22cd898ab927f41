#!/bin/bash
# r02 s5: keyed GPU tests + one-rank round probe + the N>1 bench path at world 1 after the
# inline completion of small rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s5g; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_api_gpu.py tests/test_multiproc_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_keyed.log 2>&1
rc=$?; echo "pytest keyed rc=$rc"; tail -2 $O/pytest_keyed.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/round_pipeline_probe.py > $O/round_pipeline.jsonl 2> $O/round_pipeline.err
rc=$?; echo "round_pipeline rc=$rc"; cat $O/round_pipeline.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --force-multi --steps 10 --warmup 3 > $O/bench_multi1.json 2> $O/bench_multi1.err
rc=$?; python -c "
import json;d=json.loads(open('$O/bench_multi1.json').read().strip().splitlines()[-1])
print({k:d.get(k) for k in ('value','leg_errors','keyed_c1_latency')})"; exit $rc
