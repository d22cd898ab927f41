"""ddl_allreduce_host (256 MiB fp32, pinned buffers) with the allocating / calling thread left where
the OS put it vs bound to the CPUs of the GPU's NUMA node, interleaved rounds; reports the NUMA
node the pinned pages landed on (move_pages query) and the GPU's node (measurement)."""
import ctypes
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


def cpulist(text):
    out = set()
    for part in text.strip().split(','):
        if part:
            a, _, b = part.partition('-')
            out.update(range(int(a), int(b or a) + 1))
    return out


def gpu_node():
    p = torch.cuda.get_device_properties(0)
    bdf = f'{getattr(p, "pci_domain_id", 0):04x}:{getattr(p, "pci_bus_id", 0):02x}:{getattr(p, "pci_device_id", 0):02x}.0'
    return int(open(f'/sys/bus/pci/devices/{bdf}/numa_node').read())


libc = ctypes.CDLL(None, use_errno=True)


def page_nodes(t, samples=64):
    """NUMA node of `samples` pages spread over the tensor (move_pages with nodes = NULL)."""
    base, nbytes = t.data_ptr(), t.numel() * t.element_size()
    pages = (ctypes.c_void_p * samples)(*[base + (nbytes * i // samples) // 4096 * 4096 for i in range(samples)])
    status = (ctypes.c_int * samples)()
    rc = libc.syscall(279, 0, samples, pages, None, status, 0)  # SYS_move_pages on x86_64
    if rc != 0:
        return {'error': ctypes.get_errno()}
    hist = {}
    for s in status:
        hist[s] = hist.get(s, 0) + 1
    return hist


def main():
    torch.cuda.set_device(0)
    lib = CPPBackend.c_api()
    comm = Communicator.world()
    node = gpu_node()
    allowed = os.sched_getaffinity(0)
    local = cpulist(open(f'/sys/devices/system/node/node{node}/cpulist').read()) & allowed if node >= 0 else set()
    print(json.dumps({'gpu_node': node, 'allowed_cpus': len(allowed), 'local_cpus': len(local),
                      'nodes': sorted(os.listdir('/sys/devices/system/node'))}), flush=True)
    n = (256 << 20) // 4
    for rep in range(3):
        for bind in (False, True):
            if bind and local:
                os.sched_setaffinity(0, local)
            src = torch.rand(n, pin_memory=True)
            dst = torch.empty(n, pin_memory=True)
            check(lib.ddl_allreduce_host(comm.id, src.data_ptr(), dst.data_ptr(), n, 1, 0), "ddl_allreduce_host")
            t0 = time.perf_counter()
            for _ in range(6):
                check(lib.ddl_allreduce_host(comm.id, src.data_ptr(), dst.data_ptr(), n, 1, 0), "ddl_allreduce_host")
            ms = (time.perf_counter() - t0) / 6 * 1e3
            print(json.dumps({'rep': rep, 'bind': bind, 'ms': round(ms, 3), 'src_pages': page_nodes(src),
                              'dst_pages': page_nodes(dst), 'cpu': os.sched_getaffinity(0) == local}), flush=True)
            del src, dst
            os.sched_setaffinity(0, allowed)


if __name__ == '__main__':
    main()
