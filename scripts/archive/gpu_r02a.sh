#!/bin/bash
# Round-2 measurement pass: N=1 bench, N=2/4 rehearsal of the N>1 legs, small-bucket latency
# (plain and under rocprofv3 kernel trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r02/bench_n1.json 2> gpurun_out/r02/bench_n1.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r02/bench_n1.err; exit $rc; }
N=2 RT=300 bash scripts/rehearse_multi.sh || exit 1
N=4 RT=300 PORT=29556 bash scripts/rehearse_multi.sh || exit 1
timeout -k 10 200 python3 tools/small_latency.py > gpurun_out/r02/small_latency.jsonl 2> gpurun_out/r02/small_latency.err
rc=$?; echo "small rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r02/small_latency.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02/small_prof -o small --output-format csv -- python3 tools/small_latency.py --reps 100 > gpurun_out/r02/small_latency_prof.jsonl 2> gpurun_out/r02/small_prof.err
rc=$?; echo "small prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r02/small_prof.err; exit $rc; }
python3 scripts/prof_small.py gpurun_out/r02/small_prof
