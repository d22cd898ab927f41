#!/bin/bash
# r05 s11: the keyed / batch / DP tests after the torch mirror's leaner batch submission, then the
# pageable host C5 leg twice (fresh vs fresh_native: the mirror's per-batch cost).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s11}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 500 python -u -m pytest tests -m gpu -q -k "keyed or batch or async or optimizer or callback or example or completion or deployment" --timeout 150 --timeout-method thread > $O/pytest_sub.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_sub.log
if crashed $rc; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python tools/host_steady_leg.py > $O/host_steady_$i.json 2> $O/host_steady_$i.err
  rc=$?; echo "steady$i rc=$rc"; tail -c 600 $O/host_steady_$i.json
  if crashed $rc; then exit $rc; fi
done
