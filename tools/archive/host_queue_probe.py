"""Does the number of HIP streams a process made before the host pipeline's own three streams
(Communicator::allreduce_host creates them on first use) change ddl_allreduce_host's rate?
One fresh process per count k: k streams from hipStreamCreateWithFlags, then 256 MiB fp32
pinned -> device -> pinned, 6 timed calls (measurement)."""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(k, variant):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
    import torch
    from ddl.torch.communicator import Communicator
    from ddl.torch.cpp_backend import CPPBackend, check
    torch.cuda.set_device(0)
    lib = CPPBackend.c_api()
    comm = Communicator.world()
    hip = ctypes.CDLL('libamdhip64.so')
    keep = []
    for _ in range(k):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
        keep.append(s)
    n = (256 << 20) // 4
    src = torch.rand(n, pin_memory=True)
    dst = torch.empty(n, pin_memory=True)
    check(lib.ddl_allreduce_host(comm.id, src.data_ptr(), dst.data_ptr(), n, 1, 0), 'ddl_allreduce_host')
    t0 = time.perf_counter()
    for _ in range(6):
        check(lib.ddl_allreduce_host(comm.id, src.data_ptr(), dst.data_ptr(), n, 1, 0), 'ddl_allreduce_host')
    print(json.dumps({'streams_before': k, 'ms': round((time.perf_counter() - t0) / 6 * 1e3, 3)}), flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1:
        child(int(sys.argv[1]), sys.argv[2] if len(sys.argv) > 2 else '')
    else:
        for rep in range(2):
            for k in range(8):
                r = subprocess.run([sys.executable, os.path.abspath(__file__), str(k)], capture_output=True, text=True,
                                   timeout=120)
                sys.stdout.write(''.join(l + '\n' for l in r.stdout.splitlines() if l.startswith('{')) or
                                 json.dumps({'streams_before': k, 'error': r.stderr[-300:]}) + '\n')
                sys.stdout.flush()
