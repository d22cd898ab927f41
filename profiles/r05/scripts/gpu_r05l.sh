#!/bin/bash
# r05 s24: same-box A/B of the keyed batch's host phases, the library before the pooled pending map
# (built from 8610599 into lib_ab/ by hand, not committed, removed after the run) against the
# current one, alternated 3 times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r05s24}; mkdir -p $O
OLD=$PWD/experiment-distributed-deep-learning_amd/lib_ab/libddl_amd_testing_prepool.so
NEW=$PWD/experiment-distributed-deep-learning_amd/lib/libddl_amd_testing.so
for i in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=$NEW; fi
    ddl_lib=$L timeout -k 10 150 python tools/keyed_overhead.py > $O/${v}_$i.jsonl 2> $O/${v}_$i.err || exit $?
    echo "$v $i: $(grep -c round: $O/${v}_$i.err) phase lines"
  done
done
