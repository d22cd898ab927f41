#!/bin/bash
# r03 first pass: GPU suite + smoke, the spawned N>1 rehearsal line, the 1-GPU refusal of
# --gpus 8, then the hipGraph capture experiments: the engine's forked-stream
# programs captured from C++ (tools/capture_engine.hip, one HIP runtime) and from torch
# (tools/graph_probe.py with the runtime matched by soname). Stops at the first crash or timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03a; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=25 --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_gpu rc=$rc"; tail -4 $O/pytest_gpu.log
  if crashed $rc; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
  if crashed $rc; then exit $rc; fi
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 500 python3 bench.py --gpus 4 --rehearse --steps 3 --warmup 1 --no-size-sweep --no-config-sweep > $O/rehearse4_spawn.json 2> $O/rehearse4_spawn.err
  rc=$?; echo "rehearse4 spawn rc=$rc"; head -c 600 $O/rehearse4_spawn.json; echo
  if crashed $rc; then exit $rc; fi
  timeout -k 10 120 python3 bench.py --gpus 8 > $O/gpus8.json 2> $O/gpus8.err
  rc=$?; echo "gpus8 on one GPU rc=$rc (want non-zero, no line)"; wc -c < $O/gpus8.json; grep -h "GPUs" $O/gpus8.err | head -2
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then exit $rc; fi
fi
for m in ${CMODES:-direct3 ring2 bcast3 gatherv3 loop5}; do
  timeout -k 10 90 ./tools/bin/capture_engine $m 1 > $O/capture_engine_$m.log 2>&1
  rc=$?; echo "capture_engine $m forked rc=$rc"; tail -2 $O/capture_engine_$m.log
  if crashed $rc; then exit $rc; fi
done
for m in ${PMODES:-local ring2 loop rawlocal}; do
  timeout -k 10 120 python -u -X faulthandler tools/graph_probe.py $m 1 1 > $O/probe_forked_$m.log 2>&1
  rc=$?; echo "probe $m forked rc=$rc"; grep -v "^  File\|^Thread\|^Extension\|^$\|Current thread\|amdgpu.ids" $O/probe_forked_$m.log | tail -6
  if crashed $rc; then exit $rc; fi
done
exit 0
