#!/bin/bash
# r06 s1: the full-size MPICH hash tests and the tightened fp16 bounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/s1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_fullsize_mpich_gpu.py "tests/test_configs_gpu.py::test_c4_fp16_64x16mib_tolerance" \
  "tests/test_ring_gpu.py::test_fp16_tolerance_vs_fp64" \
  "tests/test_thread_world_gpu.py::test_thread_world_c4_fp16_full_size" \
  "tests/test_thread_world_rccl_gpu.py::test_rccl_threads_c4_fp16_full_size" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest.log; exit $rc
