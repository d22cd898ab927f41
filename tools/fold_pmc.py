"""Launches the direct schedule's fold kernel (k_sumN_run / k_sumN_tile) in the two shapes the N>1 path runs, for
rocprofv3 PMC passes (the counters that bound them):
  fp32: one P = 8 chunk of the C3 bucket (32 MiB, 7 received inputs + own, non-temporal loads,
        write-through store) — 40 launches over 2 rotating buffer sets;
  fp16: one P = 8 chunk of a C4 bucket (2 MiB fp16, widened to fp32, one rounding) — 200 launches
        on cache-resident inputs, as RCCL has just written them.
    rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES ... --kernel-trace -- python3 tools/fold_pmc.py
Diagnostic only (not a measurement of record: bench.py times the kernels with HIP events)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
from ddl.torch.cpp_backend import CPPBackend, check  # noqa: E402


def run(lib, chunk_bytes, half, reps, sets):
    dt, es = (19, 2) if half else (1, 4)
    n = chunk_bytes // es
    bufs = [[torch.rand(n, device='cuda').to(torch.float16 if half else torch.float32) for _ in range(9)]
            for _ in range(sets)]
    P = ctypes.c_void_p * 7
    s = torch.cuda.current_stream().cuda_stream
    for k in range(reps):
        b = bufs[k % sets]
        check(lib.ddl_reduce_fold_ordered(b[8].data_ptr(), b[0].data_ptr(), P(*[t.data_ptr() for t in b[1:8]]), 7, n,
                                          dt, 0, s), 'ddl_reduce_fold_ordered')
    torch.cuda.synchronize()


def main():
    lib = CPPBackend.c_api()
    torch.cuda.set_device(0)
    run(lib, 32 << 20, False, 40, 2)  # the run form (k_sumN_run, the default above 8 MiB)
    check(lib.ddl_set_config(b'fold_form', 1), 'fold_form')
    run(lib, 32 << 20, False, 40, 2)  # the tile form of the same chunk (A/B)
    check(lib.ddl_set_config(b'fold_form', 0), 'fold_form')
    run(lib, 2 << 20, True, 200, 1)
    print('fold_pmc: done', flush=True)


if __name__ == '__main__':
    main()
