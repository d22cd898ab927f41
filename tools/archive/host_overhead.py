"""Host cost per call of the engine's program build + stream/event enqueue, measured on P
virtual ranks (ddl_local_ring_allreduce; D2D copies stand in for RCCL, whose own group cost is
in tools/rccl_group_cost.py)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
import torch  # noqa: E402
from ddl.torch.cpp_backend import CPPBackend  # noqa: E402

lib = CPPBackend.c_api()
res = []
s = torch.cuda.current_stream().cuda_stream
for algo in (0, 1):
    lib.ddl_set_config(b'algo', algo)
    for P in (2, 8):
        for nbytes in (4096, 256 << 10, 16 << 20):
            n = nbytes // 4
            ts = [torch.rand(n, device='cuda') for _ in range(P)]
            arr = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ts])
            for _ in range(5):
                lib.ddl_local_ring_allreduce(P, arr, arr, n, 1, 0, s)
            torch.cuda.synchronize()
            reps = 200
            t0 = time.perf_counter()
            for _ in range(reps):
                lib.ddl_local_ring_allreduce(P, arr, arr, n, 1, 0, s)
            host = (time.perf_counter() - t0) / reps
            torch.cuda.synchronize()
            dev = (time.perf_counter() - t0) / reps
            res.append({'algo': ['ring', 'direct'][algo], 'P': P, 'bytes': nbytes,
                        'host_us_per_call': round(host * 1e6, 1), 'wall_us_per_call': round(dev * 1e6, 1)})
            print(res[-1], flush=True)
print(json.dumps(res))
