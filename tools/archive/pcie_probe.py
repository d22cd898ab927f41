"""PCIe ceiling on the box (measurement tool): pinned H2D, D2H and both at once, 256 MiB, plus
the host-resident allreduce pipeline (ddl_allreduce_host) at several chunk sizes."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))


def main():
    import torch
    from ddl.torch.communicator import Communicator
    from ddl.torch.cpp_backend import CPPBackend, check
    S = 256 << 20
    h1 = torch.empty(S, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(S, dtype=torch.uint8).pin_memory()
    d1 = torch.empty(S, dtype=torch.uint8, device='cuda')
    d2 = torch.empty(S, dtype=torch.uint8, device='cuda')
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = {}

    def t(fn, reps=8):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    def h2d():
        with torch.cuda.stream(s1):
            d1.copy_(h1, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)

    def both():
        h2d()
        d2h()
    for name, fn in (('h2d', h2d), ('d2h', d2h), ('both', both)):
        dt = t(fn)
        res[name + '_GBs'] = round((2 if name == 'both' else 1) * S / dt / 1e9, 1)
    lib = CPPBackend.c_api()
    comm = Communicator.world()
    n = S // 4
    src = torch.randn(n).pin_memory()
    dst = torch.empty(n).pin_memory()
    for chunk in (4 << 20, 8 << 20, 16 << 20, 32 << 20, 64 << 20):
        check(lib.ddl_set_config(b'host_chunk_bytes', chunk), 'cfg')
        dt = t(lambda: check(lib.ddl_allreduce_host(comm.id, src.data_ptr(), dst.data_ptr(), n, 1, 0), 'host'), 6)
        res[f'pipeline_{chunk >> 20}MiB_GiBs'] = round(S / dt / 2 ** 30, 2)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
