"""PCIe copy rates right after seconds of HBM-saturating reduce kernels vs after idle (measurement:
the bench's host leg read 10.2 ms per 256 MiB right after its kernel legs and 6.2 ms 2 s later).
Prints H2D-only, D2H-only and both-directions rates (pinned, 256 MiB, torch copies on two streams)
and ddl_allreduce_host, at increasing delays after a load of `load_s` seconds."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
import torch  # noqa: E402

from ddl.torch.communicator import Communicator  # noqa: E402
from ddl.torch.cpp_backend import CPPBackend, check  # noqa: E402


def rates(lib, comm, h_src, h_dst, d_a, d_b, s1, s2):
    out = {}
    n = h_src.numel()
    for name in ('h2d', 'd2h', 'both', 'allreduce_host'):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            if name == 'allreduce_host':
                check(lib.ddl_allreduce_host(comm.id, h_src.data_ptr(), h_dst.data_ptr(), n, 1, 0), 'host')
                continue
            if name in ('h2d', 'both'):
                with torch.cuda.stream(s1):
                    d_a.copy_(h_src, non_blocking=True)
            if name in ('d2h', 'both'):
                with torch.cuda.stream(s2):
                    h_dst.copy_(d_b, non_blocking=True)
        torch.cuda.synchronize()
        out[name + '_ms'] = round((time.perf_counter() - t0) / 4 * 1e3, 3)
    return out


def main():
    torch.cuda.set_device(0)
    lib = CPPBackend.c_api()
    comm = Communicator.world()
    n = (256 << 20) // 4
    h_src, h_dst = torch.rand(n, pin_memory=True), torch.empty(n, pin_memory=True)
    d_a, d_b = torch.empty(n, device='cuda'), torch.rand(n, device='cuda')
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    print(json.dumps(dict(stage='fresh', **rates(lib, comm, h_src, h_dst, d_a, d_b, s1, s2))), flush=True)
    bufs = [(torch.rand(n, device='cuda'), torch.rand(n, device='cuda')) for _ in range(3)]
    sh = torch.cuda.current_stream().cuda_stream
    for load_s in (5, 20):
        t_end = time.perf_counter() + load_s
        i = 0
        while time.perf_counter() < t_end:
            for _ in range(50):
                a, b = bufs[i % 3]
                i += 1
                check(lib.ddl_reduce_sum2_variant(-1, a.data_ptr(), a.data_ptr(), b.data_ptr(), n, 1, sh), 'reduce')
            torch.cuda.synchronize()
        for delay in (0, 0.5, 2, 5):
            time.sleep(delay)
            print(json.dumps(dict(stage=f'after {load_s}s load, {delay}s idle',
                                  **rates(lib, comm, h_src, h_dst, d_a, d_b, s1, s2))), flush=True)


if __name__ == '__main__':
    main()
