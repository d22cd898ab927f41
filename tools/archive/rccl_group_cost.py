"""Host-side enqueue cost of one tick's RCCL group (ncclGroupStart; R x (ncclSend + ncclRecv);
ncclGroupEnd) on a one-rank communicator (self send/recv), and the device time of the same
groups. Run on the GPU box: the ring schedule issues 2(P-1)K such groups per allreduce, the
direct schedule 2K, so this bounds how launch-bound a schedule is."""
import ctypes
import os
import sys
import time

import torch

torch.cuda.init()
lib = None
for name in ('librccl.so', 'librccl.so.1', '/opt/rocm/lib/librccl.so.1'):
    try:
        lib = ctypes.CDLL(name, mode=ctypes.RTLD_GLOBAL | getattr(os, 'RTLD_NOLOAD', 4))
        break
    except OSError:
        continue
if lib is None:
    lib = ctypes.CDLL('/opt/rocm/lib/librccl.so.1', mode=ctypes.RTLD_GLOBAL)
class UniqueId(ctypes.Structure):  # ncclUniqueId is passed by value
    _fields_ = [('internal', ctypes.c_char * 128)]


uid = UniqueId()
assert lib.ncclGetUniqueId(ctypes.byref(uid)) == 0
comm = ctypes.c_void_p()
lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UniqueId, ctypes.c_int]
assert lib.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0, 'ncclCommInitRank'
stream = torch.cuda.current_stream().cuda_stream
lib.ncclSend.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
lib.ncclRecv.argtypes = lib.ncclSend.argtypes

res = {}
for R in (1, 7):
    for nbytes in (64 << 10, 2 << 20):
        src = [torch.empty(nbytes, dtype=torch.uint8, device='cuda') for _ in range(R)]
        dst = [torch.empty(nbytes, dtype=torch.uint8, device='cuda') for _ in range(R)]

        def group():
            assert lib.ncclGroupStart() == 0
            for r in range(R):
                assert lib.ncclSend(src[r].data_ptr(), nbytes, 0, 0, comm, stream) == 0
                assert lib.ncclRecv(dst[r].data_ptr(), nbytes, 0, 0, comm, stream) == 0
            assert lib.ncclGroupEnd() == 0

        for _ in range(20):
            group()
        torch.cuda.synchronize()
        n = 200
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(n):
            group()
        e1.record()
        host = (time.perf_counter() - t0) / n
        torch.cuda.synchronize()
        dev = e0.elapsed_time(e1) / 1e3 / n
        res[f'R{R}_{nbytes >> 10}KiB'] = {'host_us_per_group': round(host * 1e6, 1),
                                          'device_us_per_group': round(dev * 1e6, 1)}
        print(f'R={R} bytes={nbytes}: host {host * 1e6:.1f} us/group, device {dev * 1e6:.1f} us/group',
              flush=True)
import json
print(json.dumps(res))
