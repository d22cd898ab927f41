# One GPU pass over the tree: the -m gpu suite, smoke(), the zero-copy probe, the N=1 bench.
set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s4/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s4/smoke.log 2>&1 && \
timeout -k 10 180 python -u tools/zero_copy_probe.py > gpurun_out/s4/zero_copy.jsonl 2> gpurun_out/s4/zero_copy.err && \
timeout -k 10 400 python -u bench.py > gpurun_out/s4/bench_n1.json 2> gpurun_out/s4/bench_n1.err
