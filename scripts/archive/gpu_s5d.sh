#!/bin/bash
# r02 s5: keyed GPU tests, the one-rank round probe and N=2/4 rehearsals after a handler change.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s5d; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_api_gpu.py tests/test_multiproc_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_keyed.log 2>&1
rc=$?; echo "pytest keyed rc=$rc"; tail -2 $O/pytest_keyed.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/round_pipeline_probe.py > $O/round_pipeline.jsonl 2> $O/round_pipeline.err
rc=$?; echo "round_pipeline rc=$rc"; cat $O/round_pipeline.jsonl; [ $rc -eq 0 ] || exit $rc
O=$O bash scripts/gpu_s5c.sh
