#!/bin/bash
# r05 s1: the N=1 bench with the new C4 residency legs and the pageable steady-state host leg;
# the C4 dispatch probe and the bench's fold legs under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05s1}; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_deployment_lib_gpu.py tests/test_abi.py -x -v --timeout 240 --timeout-method thread > $O/pytest_deploy.log 2>&1
rc=$?; echo "pytest deploy rc=$rc"; tail -5 $O/pytest_deploy.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
if crashed $rc; then exit $rc; fi
timeout -k 10 500 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $O/bench_n1.json; echo
if crashed $rc; then tail -20 $O/bench_n1.err; exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_probe -o probe --output-format csv -- python3 tools/c4_dispatch_probe.py > $O/c4_probe.json 2> $O/c4_probe.err
rc=$?; echo "probe rc=$rc"; cat $O/c4_probe.json
if crashed $rc; then tail -20 $O/c4_probe.err; exit $rc; fi
python3 scripts/prof_summarize.py $O/prof_probe > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o trace --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-sweep --no-cpu-baseline --no-forced-data-plane --no-host --no-fusion > $O/bench_trace.json 2> $O/bench_trace.err
rc=$?; echo "bench trace rc=$rc"
if crashed $rc; then tail -20 $O/bench_trace.err; exit $rc; fi
python3 scripts/prof_summarize.py $O/prof_bench > /dev/null
find $O -name '*.csv' -size +2M -delete
ls -la $O $O/prof_probe $O/prof_bench | head -40
