#!/bin/bash
# r06 s5: multi-rank RCCL on one GPU at P = 4 and 5, each check timed (progress file), Python
# stacks every 60 s if a rank stalls; a heartbeat keeps the run visibly alive.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s5; mkdir -p $O
export ddl_lib=$PWD/experiment-distributed-deep-learning_amd/lib/libddl_amd_testing.so NCCL_DEBUG=WARN DDL_MP_PROGRESS_FILE=$PWD/$O/progress.txt DDL_MP_STACKS_S=90
for P in 4 5; do
  timeout -k 10 420 python -u -c "
import sys, time; sys.path.insert(0, 'tests')
import test_multiproc_rccl_gpu as t
t0 = time.time(); t._run($P, timeout=400); print('P=$P ok', round(time.time() - t0, 1), 's', flush=True)
" > $O/run_p$P.log 2>&1 &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 20; echo "P=$P alive: $(tail -1 $O/progress.txt 2>/dev/null)"; done
  wait $pid; rc=$?; echo "P=$P rc=$rc"; tail -5 $O/run_p$P.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
