#!/bin/bash
# r05 s22: the pending map's nodes from a pool: the keyed-path GPU tests, the keyed batch's host
# phases (tools/keyed_overhead.py, vs s21), a P = 5 soak.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s22}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "keyed or batch or async or optimizer or callback or example or completion or deployment or broadcast or token or split or multiproc" --timeout 150 --timeout-method thread > $O/pytest_sub.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_sub.log
if crashed $rc || [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/keyed_overhead.py > $O/keyed_overhead.jsonl 2> $O/keyed_overhead.err
rc=$?; echo "overhead rc=$rc"; cat $O/keyed_overhead.jsonl; grep round: $O/keyed_overhead.err
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python3 tools/soak_mp.py 5 10 > $O/soak5.log 2>&1
rc=$?; echo "soak5 rc=$rc"; tail -2 $O/soak5.log
