#!/bin/bash
# r05 s14: the keyed / batch / DP / example / deployment tests after the mirror's argument checks
# moved ahead of its completion groups.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s14}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -q -k "keyed or batch or async or optimizer or callback or example or completion or deployment or broadcast" --timeout 150 --timeout-method thread > $O/pytest_sub.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_sub.log; exit $rc
