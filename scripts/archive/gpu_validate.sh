# One GPU pass over the tree: the -m gpu suite, smoke(), the N=1 bench line, and the rocprofv3
# kernel-trace summary of the same bench command.
set -o pipefail
mkdir -p gpurun_out/s4
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s4/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s4/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/s4/bench_n1.json 2> gpurun_out/s4/bench_n1.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/s4/prof -o bench -- python3 -u bench.py --no-sweep --no-cpu-baseline --no-forced-data-plane > gpurun_out/s4/bench_under_rocprof.json 2> gpurun_out/s4/rocprof.err
