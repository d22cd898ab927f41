#!/bin/bash
# r04 pass on the current tree: smoke + default N=1 bench, then rocprofv3 kernel trace / stats and
# the FETCH_SIZE / WRITE_SIZE passes of the bench (scripts/gpu_profile.sh) with the per-(kernel,
# grid) summary (scripts/prof_summarize.py). Usage: TAG=r04s1 bash scripts/gpu_r04a.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04}
O=gpurun_out/$TAG; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
if crashed $rc; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $O/bench_n1.json; echo
if crashed $rc; then exit $rc; fi
if [ -z "$SKIP_PROF" ]; then TAG=$TAG bash scripts/gpu_profile.sh; fi
