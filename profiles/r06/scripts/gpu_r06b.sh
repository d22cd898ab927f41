#!/bin/bash
# r06 s2: the whole GPU suite after the RCCL config plumbing, the unpack-lane instrumentation, the
# device-unpack failure drain and the deferred-deletion reaper; smoke; the N=1 bench (host legs
# carry the lane split); the lane copy probe; the N=8 rehearsal (the CTA sweep and the C4 tuner table).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s2; mkdir -p $O
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=25 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -5 $O/pytest_gpu.log
if crashed $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
if crashed $rc; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $O/bench_n1.json; echo
if crashed $rc; then exit $rc; fi
timeout -k 10 200 tools/bin/lane_copy_probe > $O/lane_copy_probe.jsonl 2> $O/lane_copy_probe.err
rc=$?; echo "lane probe rc=$rc"; cat $O/lane_copy_probe.jsonl
if crashed $rc; then exit $rc; fi
NS=8 LIMIT=560 TAG=r06/s2 bash scripts/gpu_rehearse.sh
