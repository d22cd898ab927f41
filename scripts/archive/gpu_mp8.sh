#!/bin/bash
# The 8-process GPU test's per-check times with the engine's placement knobs on (defaults) and off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-mp8}; mkdir -p $O
for cfg in ${CFGS:-"1 0" "0 8" "1 8" "0 0"}; do set -- $cfg
  DDL_MP_NUMA_BIND=$1 DDL_MP_CU_MASK=$2 DDL_MP_TIMEOUT=400 timeout -k 10 450 python -u -m pytest tests/test_multiproc_gpu.py -q -s -k "8-1" --timeout 440 --timeout-method thread > $O/mp8_bind$1_mask$2.log 2>&1
  rc=$?; echo "bind=$1 mask=$2 rc=$rc"; grep -h "\[P=8\]" $O/mp8_bind$1_mask$2.log; tail -1 $O/mp8_bind$1_mask$2.log
  case $rc in 0|1) ;; *) exit $rc;; esac
done
exit 0
